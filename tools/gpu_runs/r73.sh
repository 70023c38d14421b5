# bitwise determinism of the attention kernels (base build and current build)
set -o pipefail
O=gpurun_out/r73; mkdir -p $O
timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/cur.so 8 > $O/det_cur.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/base.so 8 > $O/det_base.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/v9.so 8 > $O/det_v9.log 2>&1
