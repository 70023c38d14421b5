"""Do two counting contexts on one GPU disturb each other's reads?

A child process runs a steady bf16 GEMM loop with the in-process agent
sampling the `lite` set at 1 kHz and prints its newest record every second.
Meanwhile the parent runs five phases of equal length:

  A  no daemon
  B  a daemon sampling the readable-only `xproc` set at 1 kHz (different
     counter selections from the agent's)
  C  no daemon
  D  a daemon sampling `lite` at 1 kHz (the agent's own selections)
  E  no daemon

and prints the agent's per-phase means, plus the daemon's own records of
phases B and D.  If a second context's selections replaced the first one's,
the agent's lite values in B would move away from A / C / E (or go to 0).

Usage (GPU box): python tools/probes/cosample_probe.py [phase_s] [out.json]
"""
import json
import os
import subprocess
import sys
import textwrap
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dynolog_amd.utils.daemon import DaemonProcess  # noqa: E402

CHILD = textwrap.dedent("""
    import json, os, sys, time
    from dynolog_amd import agent
    agent.preinit()
    import torch
    a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=("memory",), log_interval_ms=1000)
    x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    y = x @ x; torch.cuda.synchronize()
    t = time.time()
    while a.stats()["samples_taken"] == 0 and time.time() - t < 30:
        time.sleep(0.01)
    print("READY", os.getpid(), flush=True)
    end = time.time() + float(sys.argv[1])
    last = time.time()
    while time.time() < end:
        for _ in range(10):
            y = x @ x
        torch.cuda.synchronize()
        a.step()
        if time.time() - last >= 1.0:
            last = time.time()
            r = a.latest(0) or {}
            r = {k: v for k, v in r.items() if isinstance(v, (int, float))}
            print("REC " + json.dumps({"t": last, "rec": r}), flush=True)
    s = a.stats()
    print("STATS " + json.dumps({k: s.get(k) for k in ("samples_taken", "sample_latency_us_avg", "late_ticks")}), flush=True)
    a.stop()
""")

KEYS = ("gpu_busy_pct", "mfma_util", "tensorcore_active", "sm_active_ratio", "sm_occupancy", "hbm_read_gbps",
        "hbm_write_gbps", "mfma_bf16_tflops", "counter_samples")


def main():
    phase_s = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    out_path = sys.argv[2] if len(sys.argv) > 2 else "cosample.json"
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, PYTHONPATH=repo)
    env.pop("ROCP_TOOL_LIBRARIES", None)
    child = subprocess.Popen([sys.executable, "-u", "-c", CHILD, str(phase_s * 5 + 30)], stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True, env=env)
    lines = []
    ready = threading.Event()

    def reader():
        for ln in child.stdout:
            lines.append((time.time(), ln.rstrip()))
            if ln.startswith("READY"):
                ready.set()

    th = threading.Thread(target=reader, daemon=True)
    th.start()
    if not ready.wait(120):
        child.kill()
        print("\n".join(l for _, l in lines[-30:]))
        sys.exit(1)
    print("child ready", flush=True)
    phases = []
    daemon_recs = {}
    try:
        for name, dargs in (("A", None), ("B", "xproc"), ("C", None), ("D", "lite"), ("E", None)):
            d = None
            if dargs:
                d = DaemonProcess(["--enable_gpu_counters", "--gpu_counter_hz=1000", f"--gpu_counters={dargs}",
                                   "--gpu_counter_reporting_interval_s=1"]).start()
                t = time.time()  # the daemon's GPU thread publishing before the phase clock starts
                while time.time() - t < 30:
                    m = d.rpc({"fn": "getGpuCounterMonitor"}) or {}
                    if m.get("status") == "ok" and all(g.get("samples", 0) > 100 for g in m.get("gpus", [{}])):
                        break
                    time.sleep(0.2)
            t0 = time.time()
            time.sleep(phase_s)
            t1 = time.time()
            phases.append((name, dargs, t0, t1))
            print(f"phase {name} ({dargs or 'no daemon'}) done", flush=True)
            if d is not None:
                recs = (d.rpc({"fn": "getMetrics", "collector": "gpu_counters", "last": 30}) or {}).get("records", [])
                mon = d.rpc({"fn": "getGpuCounterMonitor"}) or {}
                daemon_recs[name] = {
                    "records": [{k: r.get(k) for k in KEYS + ("counter_set", "counter_visibility") if k in r}
                                for r in recs[-int(phase_s):]],
                    "monitor": [{k: g.get(k) for k in ("samples", "sample_latency_us_avg", "late_ticks", "sampling")}
                                for g in mon.get("gpus", [])]}
                d.stop()
    finally:
        child.wait(timeout=phase_s * 5 + 120)
        th.join(5)
    recs = []
    for ts, ln in lines:
        if ln.startswith("REC "):
            recs.append(json.loads(ln[4:]))
    summary = {"phase_s": phase_s, "phases": {}}
    for name, dargs, t0, t1 in phases:
        inside = [r["rec"] for r in recs if t0 + 1.5 <= r["t"] <= t1]  # a record covers the second before it
        means = {}
        for k in KEYS:
            v = [r[k] for r in inside if k in r]
            if v:
                means[k] = round(sum(v) / len(v), 4)
        summary["phases"][name] = {"daemon": dargs, "agent_records": len(inside), "agent_means": means}
        if name in daemon_recs:
            summary["phases"][name]["daemon_side"] = daemon_recs[name]
    summary["child_tail"] = [l for _, l in lines if l.startswith("STATS")] + [l for _, l in lines[-3:]]
    summary["child_rc"] = child.returncode
    with open(out_path, "w") as f:
        json.dump(summary, f, indent=1)
    for name in summary["phases"]:
        p = summary["phases"][name]
        print(name, p["daemon"], p["agent_records"], json.dumps(p["agent_means"]))
    return 0 if child.returncode == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
