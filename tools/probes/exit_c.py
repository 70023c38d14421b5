# exit-crash probe: torch's ROCm runtime loaded FIRST, then our agent binds to it
import sys, time, os, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from dynolog_amd import agent
agent.preinit()
torch.cuda.set_device(0)
a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=())
x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
t0 = agent.mono_ns()
for _ in range(200):
    y = x @ x
torch.cuda.synchronize()
time.sleep(0.3)
t1 = agent.mono_ns()
a.pack_pending(); a.step(); torch.cuda.synchronize(); a.flush()
print("stats", json.dumps(a.stats()), flush=True)
print("latest", json.dumps(a.latest(0)), flush=True)
a.stop()
maps = open("/proc/self/maps").read()
libs = sorted(set(l.split()[-1] for l in maps.splitlines() if any(k in l for k in ("amdhip64", "hsa-runtime", "rccl", "rocprofiler"))))
print("libs", libs, flush=True)
print("exit_c done", flush=True)
