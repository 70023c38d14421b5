# counter-rate drop with the fused optimizer: cgroup CPU throttling? host run-ahead?
set -o pipefail
O=gpurun_out/r25; mkdir -p $O
(cat /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; cat /proc/self/status | grep -i cpus_allowed_list) > $O/cgroup_before.txt
timeout -k 10 300 python -u bench.py --ab-rounds 1 > $O/fusedopt.log 2>&1 && \
(cat /sys/fs/cgroup/cpu.stat 2>/dev/null) > $O/cgroup_mid.txt && \
timeout -k 10 300 python -u bench.py --ab-rounds 1 --host-sync > $O/fusedopt_hostsync.log 2>&1 && \
(cat /sys/fs/cgroup/cpu.stat 2>/dev/null) > $O/cgroup_after.txt
