"""Does the agent start in a process whose libkineto runs in daemon mode
(KINETO_USE_DAEMON=1 initialises roctracer at `import torch`)?  Variants:
  A  preinit, import torch, start the agent before any GPU call
  B  same, but after torch.cuda.set_device + a tensor on the GPU
Prints one RESULT line per variant."""
import json
import os
import subprocess
import sys

CODE = r'''
import json, os, sys
from dynolog_amd import agent
agent.preinit()
import torch
if sys.argv[1] == "B":
    torch.cuda.set_device(0); torch.zeros(1, device="cuda")
try:
    a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=("memory",))
    import time; time.sleep(0.3)
    st = a.stats(); a.stop()
    print("RESULT " + json.dumps({"variant": sys.argv[1], "ok": True, "samples": st["samples_taken"]}))
except Exception as e:
    print("RESULT " + json.dumps({"variant": sys.argv[1], "ok": False, "error": str(e)}))
'''

if __name__ == "__main__":
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for kineto in ("1", "0"):
        for v in ("A", "B"):
            env = dict(os.environ, PYTHONPATH=repo, KINETO_USE_DAEMON=kineto, KINETO_DAEMON_INIT_DELAY_S="0")
            r = subprocess.run([sys.executable, "-c", CODE, v], env=env, capture_output=True, text=True, timeout=120)
            lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
            res = json.loads(lines[-1][7:]) if lines else {"variant": v, "rc": r.returncode, "stderr": r.stderr[-500:]}
            res["kineto_daemon"] = kineto
            print(json.dumps(res), flush=True)
