"""Always-on soak of the in-process agent: 1 kHz sampling plus a per-"step"
gather for SECONDS under a GEMM + elementwise load, sampling the process's
host RSS, the GPU memory in use and the agent's counters every 10 s.  A leak
in the 1 kHz path (host buffers, device staging, HIP events, records) would
show as a trend over the run.

    python tools/probes/agent_soak.py SECONDS OUT.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dynolog_amd import agent  # noqa: E402

agent.preinit()
import torch  # noqa: E402

seconds, out = float(sys.argv[1]), sys.argv[2]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ag = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=("memory",), log_file="/dev/null")
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
x = torch.randn(64 << 20, device=dev, dtype=torch.bfloat16)


def rss_kb():
    with open("/proc/self/status") as f:
        for ln in f:
            if ln.startswith("VmRSS:"):
                return int(ln.split()[1])


samples, steps = [], 0
t0 = time.time()
next_rec = 0.0
while time.time() - t0 < seconds:
    for _ in range(20):          # ~40-50 ms of GPU work per "step"
        c = a @ b
        x.mul_(1.0001)
    ag.step()                    # gather on the current stream, like a training loop
    steps += 1
    if time.time() - t0 >= next_rec:
        torch.cuda.synchronize()
        st = ag.stats()
        free, total = torch.cuda.mem_get_info()
        samples.append({"t": round(time.time() - t0, 1), "rss_kb": rss_kb(),
                        "gpu_used_mb": round((total - free) / 2**20, 1),
                        "samples_taken": st["samples_taken"], "samples_failed": st["samples_failed"],
                        "late_ticks": st.get("late_ticks"), "gathers": st.get("gathers"),
                        "received": st["ranks"][0]["received"]})
        print(json.dumps(samples[-1]), flush=True)
        next_rec += 10.0
torch.cuda.synchronize()
ag.pack_pending()
ag.step()
torch.cuda.synchronize()
ag.flush()
st = ag.stats()
ag.stop()
wall = time.time() - t0
first = samples[1] if len(samples) > 1 else samples[0]
res = {"seconds": round(wall, 1), "steps": steps, "samples_taken": st["samples_taken"],
       "samples_failed": st["samples_failed"], "received_rank0": st["ranks"][0]["received"],
       "samples_per_s": round(st["samples_taken"] / wall, 1),
       "rss_kb_at_10s": first["rss_kb"], "rss_kb_end": samples[-1]["rss_kb"],
       "gpu_used_mb_at_10s": first["gpu_used_mb"], "gpu_used_mb_end": samples[-1]["gpu_used_mb"],
       "trace": samples}
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "trace"}))
