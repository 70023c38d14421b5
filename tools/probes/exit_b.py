# exit-crash probe: agent + torch
import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from dynolog_amd import agent
agent.preinit()
import torch
torch.cuda.set_device(0)
a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=())
x = torch.randn(1024, 1024, device="cuda")
y = x @ x
torch.cuda.synchronize()
time.sleep(0.3)
a.stop()
print("exit_b done", flush=True)
