# attention forward A/B: s0-then-s1 MFMA chains (v3), + exact wave-uniform rescale skip (v4), vs v2
set -o pipefail
O=gpurun_out/r70; mkdir -p $O
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/v2.so abl/v3.so fwd > $O/ab_v3.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/v2.so abl/v4.so fwd > $O/ab_v4.log 2>&1
