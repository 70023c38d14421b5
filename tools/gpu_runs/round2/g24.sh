# static young-half priority (waves 4-7 s_setprio 1 once) in the 8-wave attention forward and dK/dV kernels, now that the grids are tail-free: A/B both orders
set -o pipefail
O=gpurun_out/g24; mkdir -p $O
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/cur.so abl/prio.so both > $O/ab_prio.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/prio.so abl/cur.so both > $O/ab_prio_rev.log 2>&1
