"""Does the agent start in a process whose libkineto runs in daemon mode
(KINETO_USE_DAEMON set: libkineto initialises at `import torch`)?  Variants
(each a fresh process; "set" = the variable is present, whatever its value):
  V1  KINETO_USE_DAEMON unset                       (baseline)
  V2  KINETO_USE_DAEMON set, init delay 0           (init at import)
  V4  KINETO_USE_DAEMON set, init delay 8 s         (agent starts before libkineto's init)
  V5  like V2 with ROCPROFILER_LOG_LEVEL=info       (stderr kept for the failure)
Prints one JSON line per variant."""
import json
import os
import subprocess
import sys

CODE = r'''
import json, os, sys, time
from dynolog_amd import agent
agent.preinit()
import torch
torch.cuda.set_device(0); torch.zeros(1, device="cuda")
try:
    a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=("memory",))
    time.sleep(float(os.environ.get("HOLD_S", "0.3")))
    st = a.stats(); a.stop()
    print("RESULT " + json.dumps({"ok": True, "samples": st["samples_taken"], "failed": st["samples_failed"]}))
except Exception as e:
    print("RESULT " + json.dumps({"ok": False, "error": str(e)}))
'''

if __name__ == "__main__":
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    base = {k: v for k, v in os.environ.items() if not k.startswith("KINETO_")}
    variants = {
        "V1": {},
        "V2": {"KINETO_USE_DAEMON": "1", "KINETO_DAEMON_INIT_DELAY_S": "0"},
        "V4": {"KINETO_USE_DAEMON": "1", "KINETO_DAEMON_INIT_DELAY_S": "8", "HOLD_S": "10"},
        "V5": {"KINETO_USE_DAEMON": "1", "KINETO_DAEMON_INIT_DELAY_S": "0", "ROCPROFILER_LOG_LEVEL": "info"},
    }
    for name, extra in variants.items():
        env = dict(base, PYTHONPATH=repo, **extra)
        r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
        lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        res = json.loads(lines[-1][7:]) if lines else {"rc": r.returncode}
        res["variant"] = name
        if name == "V5" or not res.get("ok", False):
            res["stderr_tail"] = r.stderr[-6000:]
        print(json.dumps(res), flush=True)
