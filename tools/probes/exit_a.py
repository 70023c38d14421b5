# exit-crash probe: agent without torch (HIP via our lib only)
import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from dynolog_amd import agent
agent.preinit()
a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=())
time.sleep(0.3)
mode = sys.argv[1] if len(sys.argv) > 1 else "stop"
if mode == "stop":
    a.stop()
print("exit_a done", mode, flush=True)
