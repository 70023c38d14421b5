# dK/dV kernel with an XCD-grouped 1-D grid (each XCD owns whole (batch, kv head) groups) vs the (kb, kv, batch) grid: in-process A/B both orders, determinism
set -o pipefail
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/lptx.so abl/kvx.so bwd > $O/ab_kvx.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/kvx.so abl/lptx.so bwd > $O/ab_kvx_rev.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_determinism.py abl/kvx.so 4 > $O/det_kvx.log 2>&1
