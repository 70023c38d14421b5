# round 4 g05: PID-namespace probe (KFD sysfs vs the container's /proc)
set -o pipefail
O=gpurun_out/g05; mkdir -p $O
timeout -k 10 120 python -u tools/probes/pidns_probe.py > $O/pidns_probe.log 2>&1
