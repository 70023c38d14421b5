# attention: longest-first grid (lpt) vs longest-first + XCD-grouped GQA order (lptx), in-process A/B; determinism of lptx
set -o pipefail
O=gpurun_out/g21; mkdir -p $O
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/lpt.so abl/lptx.so both > $O/ab_lptx.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/lptx.so abl/lpt.so both > $O/ab_lptx_rev.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_determinism.py abl/lptx.so 4 > $O/det_lptx.log 2>&1
