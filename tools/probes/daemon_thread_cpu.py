#!/usr/bin/env python3
"""Where the sidecar daemon's CPU goes: runs `dynolog --enable_gpu_counters`
(1 kHz, lite) for a few seconds with no job, then per-thread CPU time from
/proc/<pid>/task/*/stat (utime + stime) over a measured window.  Prints one
JSON line: threads sorted by CPU %, with their names (comm)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dynolog_amd.utils.daemon import DaemonProcess  # noqa: E402


def threads(pid):
    out = {}
    for t in os.listdir(f"/proc/{pid}/task"):
        try:
            s = open(f"/proc/{pid}/task/{t}/stat").read()
            comm = s[s.index("(") + 1:s.rindex(")")]
            f = s[s.rindex(")") + 2:].split()
            try:
                sc = open(f"/proc/{pid}/task/{t}/syscall").read().split()[0]
            except OSError:
                sc = "?"
            try:
                wchan = open(f"/proc/{pid}/task/{t}/wchan").read().strip()
            except OSError:
                wchan = "?"
            out[int(t)] = (comm, (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK"), sc, wchan)
        except (OSError, ValueError):
            pass
    return out


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 5.0
    with DaemonProcess(["--enable_gpu_counters", "--gpu_counter_hz=1000", "--gpu_counters=lite"]) as d:
        time.sleep(3.0)  # warm: contexts up, visibility scanned
        pid = d.proc.pid
        a = threads(pid)
        t0 = time.time()
        time.sleep(secs)
        b = threads(pid)
        dt = time.time() - t0
        mon = d.rpc({"fn": "getGpuCounterMonitor"})
    rows = sorted(((b[t][1] - a[t][1]) / dt * 100, t, b[t][0], b[t][2], b[t][3]) for t in b if t in a)
    rows.reverse()
    print(json.dumps({"window_s": round(dt, 2), "total_pct": round(sum(r[0] for r in rows), 1),
                      "threads": [{"tid": t, "name": n, "cpu_pct": round(c, 1), "syscall": sc, "wchan": w}
                                  for c, t, n, sc, w in rows[:15]],
                      "gpus": [{k: g.get(k) for k in ("device", "samples", "sample_latency_us_avg", "late_ticks")}
                               for g in mon.get("gpus", [])]}))


if __name__ == "__main__":
    main()
