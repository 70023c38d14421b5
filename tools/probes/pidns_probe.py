"""What can the daemon see to map KFD's process list to processes of its own
PID namespace?  (gpurun boxes run the daemon and the job in one container
whose PID namespace is not the host's; KFD sysfs lists host pids.)"""
import glob
import os
import subprocess
import sys
import time

child = subprocess.Popen([sys.executable, "-c", """
import torch, time, os
x = torch.randn(4096, 4096, device='cuda')
print('PID', os.getpid(), flush=True)
time.sleep(20)
"""], stdout=subprocess.PIPE, text=True)
pid = int(child.stdout.readline().split()[1])
time.sleep(1)


def cat(p, n=20):
    try:
        with open(p) as f:
            return "".join(f.readlines()[:n])
    except Exception as e:  # noqa: BLE001
        return f"<{e}>"


print("self pid", os.getpid(), "child pid", pid)
print("--- /proc/self/status NSpid:", [l for l in cat("/proc/self/status", 100).splitlines() if l.startswith(("NSpid", "NStgid"))])
print("--- child sched:", cat(f"/proc/{pid}/sched", 1))
print("--- ns links:", os.readlink("/proc/self/ns/pid"), os.readlink(f"/proc/{pid}/ns/pid"))
print("--- kfd proc dirs:", sorted(os.listdir("/sys/class/kfd/kfd/proc")) if os.path.isdir("/sys/class/kfd/kfd/proc") else "none")
for d in glob.glob("/sys/class/kfd/kfd/proc/*"):
    print("   ", d, sorted(os.listdir(d))[:30])
    for f in sorted(os.listdir(d)):
        p = os.path.join(d, f)
        if os.path.isfile(p):
            print("      ", f, "=", cat(p, 3).strip()[:200])
        elif os.path.isdir(p):
            for g in sorted(os.listdir(p))[:10]:
                q = os.path.join(p, g)
                if os.path.isfile(q):
                    print("      ", f + "/" + g, "=", cat(q, 3).strip()[:200])
                elif os.path.isdir(q):
                    for h in sorted(os.listdir(q))[:10]:
                        print("      ", f + "/" + g + "/" + h, "=", cat(os.path.join(q, h), 2).strip()[:120])
print("--- child fds:")
for fd in sorted(os.listdir(f"/proc/{pid}/fd"), key=int):
    try:
        tgt = os.readlink(f"/proc/{pid}/fd/{fd}")
    except OSError:
        continue
    if "dri" in tgt or "kfd" in tgt:
        print("   fd", fd, tgt)
        print(cat(f"/proc/{pid}/fdinfo/{fd}", 40))
print("--- topology gpu_id:", [cat(p, 1).strip() for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")])
child.kill()
