#!/usr/bin/env python3
"""Why did round 4's driver run see 2 dispatches in a 300 ms kernel trace
(tests/test_gpu_daemon.py::test_gpukernels_rpc_through_agent, GPUTEST_r04)?

Replays that test's old ordering -- the child prints its PID right after
GpuAgent.start, BEFORE its first torch.randn / hipBLASLt GEMM -- and asks the
daemon for the 300 ms kernel trace as soon as the agent registers, then once
more after the child is warm.  The summary's window bounds and first / last
dispatch stamps (KernelTracer::summary) tell a cold child (dispatches only
near the end of the window, or none; a first GEMM taking seconds) from
records the tracer dropped (dispatches spread over the window but few, or
dropped_records > 0).  Prints one JSON line per capture."""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import textwrap
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dynolog_amd.utils.daemon import DaemonProcess  # noqa: E402

CHILD = textwrap.dedent("""
    from dynolog_amd import agent
    agent.preinit(kernel_trace=True)
    import os, time, torch
    a = agent.GpuAgent.start(device=0, sample_hz=500, sinks=("daemon",), log_interval_ms=500)
    print("PID", os.getpid(), time.monotonic_ns(), flush=True)        # the old, cold ready line
    t0 = time.monotonic_ns()
    x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    y = x @ x; torch.cuda.synchronize()
    print("FIRST_GEMM_DONE", time.monotonic_ns(), (time.monotonic_ns() - t0) / 1e6, flush=True)
    end = time.time() + 25
    while time.time() < end and not os.path.exists(os.environ["DONE_FLAG"]):
        for _ in range(10):
            y = x @ x
        torch.cuda.synchronize()
        a.step()
    a.stop()
""")


def main() -> int:
    sockdir = tempfile.mkdtemp(prefix="dy", dir="/tmp")
    done = os.path.join(sockdir, "done")
    out = []
    try:
        with DaemonProcess(["--enable_ipc_monitor"], env={"KINETO_IPC_SOCKET_DIR": sockdir}) as d:
            env = dict(os.environ, KINETO_IPC_SOCKET_DIR=sockdir, DONE_FLAG=done,
                       PYTHONPATH=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
            log = open(os.path.join(sockdir, "child.out"), "w")
            p = subprocess.Popen([sys.executable, "-c", CHILD], env=env, stdout=log, stderr=subprocess.STDOUT)
            pid, ready_ns = None, None
            deadline = time.time() + 120
            while time.time() < deadline and pid is None and p.poll() is None:
                for line in open(log.name).read().splitlines():
                    if line.startswith("PID "):
                        pid, ready_ns = int(line.split()[1]), int(line.split()[2])
                time.sleep(0.01)
            assert pid, open(log.name).read()[-3000:]
            while time.time() < deadline:
                if any(a["pid"] == pid for a in d.rpc({"fn": "getGpuAgents"})["agents"]):
                    break
                time.sleep(0.05)
            for label in ("cold", "warm"):
                if label == "warm":
                    time.sleep(5.0)
                r = d.rpc({"fn": "gpuKernelTrace", "pids": [pid], "duration_ms": 300, "top": 3}, timeout=30)
                res = (r.get("results") or [{}])[0]
                s = res.get("summary", {})
                first_gemm = [ln for ln in open(log.name).read().splitlines() if ln.startswith("FIRST_GEMM_DONE")]
                rec = {"capture": label, "status": res.get("status"), "dispatches": s.get("dispatches"),
                       "dropped_records": s.get("dropped_records"), "window_ms": s.get("window_ms"),
                       "window_start_after_ready_ms": (s["window_start_ns"] - ready_ns) / 1e6 if "window_start_ns" in s else None,
                       "first_dispatch_after_window_start_ms":
                           (s["first_dispatch_start_ns"] - s["window_start_ns"]) / 1e6 if "first_dispatch_start_ns" in s else None,
                       "last_dispatch_before_window_end_ms":
                           (s["window_end_ns"] - s["last_dispatch_end_ns"]) / 1e6 if "last_dispatch_end_ns" in s else None,
                       "first_gemm_done_after_ready_ms":
                           (int(first_gemm[0].split()[1]) - ready_ns) / 1e6 if first_gemm else None,
                       "first_gemm_ms": float(first_gemm[0].split()[2]) if first_gemm else None,
                       "top": [(k["name"][:60], k["calls"]) for k in s.get("top_kernels", [])]}
                print(json.dumps(rec), flush=True)
                out.append(rec)
            open(done, "w").close()
            p.wait(timeout=60)
    finally:
        shutil.rmtree(sockdir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
