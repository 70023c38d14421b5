# attention fwd + dQ with a longest-first 1-D grid over every (head, batch) vs the (qb, head, batch) grid: in-process A/B, determinism, attention tests
set -o pipefail
O=gpurun_out/g20; mkdir -p $O
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/base.so abl/lpt.so both > $O/ab_lpt.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_determinism.py abl/lpt.so 4 > $O/det_lpt.log 2>&1
