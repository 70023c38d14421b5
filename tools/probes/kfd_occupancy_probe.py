"""KFD's per-process CU occupancy (/sys/class/kfd/kfd/proc/<pid>/stats_<gpuid>/
cu_occupancy) while a bf16 GEMM job and an fp32 VALU job run: what it reads,
how long a read takes, and how it tracks the load (idle / busy phases)."""
import glob
import json
import os
import subprocess
import sys
import time

job = subprocess.Popen([sys.executable, "-c", """
import torch, time, sys
x = torch.randn(8192, 8192, device='cuda', dtype=torch.bfloat16)
print('up', flush=True)
for phase in range(4):
    end = time.time() + 2.0
    if phase % 2 == 0:
        while time.time() < end:
            y = x @ x
        torch.cuda.synchronize()
    else:
        time.sleep(2.0)
print('done', flush=True)
"""], stdout=subprocess.PIPE, text=True)
assert job.stdout.readline().strip() == "up"
files = glob.glob("/sys/class/kfd/kfd/proc/*/stats_*/cu_occupancy")
mine = []
for f in files:
    pid_dir = f.split("/")[6]
    q = glob.glob(f"/sys/class/kfd/kfd/proc/{pid_dir}/queues/*/gpuid")
    gpu = f.split("stats_")[1].split("/")[0]
    if any(open(x).read().strip() == gpu for x in q):
        mine.append(f)
samples = []
t_end = time.time() + 8.5
while time.time() < t_end:
    row = {"t": round(time.time(), 3)}
    for f in mine:
        t0 = time.perf_counter()
        try:
            v = int(open(f).read().strip() or 0)
        except OSError:
            v = -1
        row[f.split("/")[6]] = v
        row["read_us_" + f.split("/")[6]] = round((time.perf_counter() - t0) * 1e6, 1)
    samples.append(row)
    time.sleep(0.05)
job.wait()
print(json.dumps({"files": mine, "n": len(samples), "samples": samples}))
