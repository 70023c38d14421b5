"""rocprofiler-sdk's own trace log of an agent start with and without
libkineto's daemon mode (KINETO_USE_DAEMON), one file per variant, to see
where the HSA API table goes when libkineto initialises roctracer at import."""
import os
import subprocess
import sys

CODE = r'''
import json, os, sys, time
from dynolog_amd import agent
agent.preinit()
print("after preinit", flush=True)
import torch
print("after import torch", flush=True)
torch.cuda.set_device(0); torch.zeros(1, device="cuda")
print("after cuda init", flush=True)
try:
    a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=("memory",))
    time.sleep(0.3); st = a.stats(); a.stop()
    print("RESULT ok", st["samples_taken"], flush=True)
except Exception as e:
    print("RESULT fail", e, flush=True)
'''

if __name__ == "__main__":
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    base = {k: v for k, v in os.environ.items() if not k.startswith("KINETO_")}
    for name, extra in {"nokineto": {}, "kineto": {"KINETO_USE_DAEMON": "1"}}.items():
        env = dict(base, PYTHONPATH=repo, ROCPROFILER_LOG_LEVEL="trace", **extra)
        with open(os.path.join(out, name + ".log"), "w") as f:
            r = subprocess.run([sys.executable, "-c", CODE], env=env, stdout=f, stderr=subprocess.STDOUT,
                               timeout=120)
        print(name, "rc", r.returncode, flush=True)
