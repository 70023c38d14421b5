# attention forward A/B: loop split (diag / non-diag), fma-folded scale, permlane32 pair reductions
set -o pipefail
O=gpurun_out/r69; mkdir -p $O
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/base.so abl/v1.so fwd > $O/ab_v1.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/base.so abl/v2.so fwd > $O/ab_v2.log 2>&1
