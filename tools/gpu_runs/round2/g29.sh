# backward kernels with one barrier per iteration (prefetch the next stage right after the barrier) vs two: A/B both orders, determinism
set -o pipefail
O=gpurun_out/g29; mkdir -p $O
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/cur.so abl/b1.so bwd > $O/ab_b1.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/b1.so abl/cur.so bwd > $O/ab_b1_rev.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_determinism.py abl/b1.so 4 > $O/det_b1.log 2>&1
