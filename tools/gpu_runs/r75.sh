# attention forward A/B vs the fixed build: early V^T fragment reads (v11), + one barrier per tile pair (v12); determinism of both
set -o pipefail
O=gpurun_out/r75; mkdir -p $O
for v in v11 v12; do timeout -k 10 120 python -u tools/probes/attn_ab.py abl/fix.so abl/$v.so fwd > $O/ab_$v.log 2>&1 && timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/$v.so 6 > $O/det_$v.log 2>&1 || exit 1; done
