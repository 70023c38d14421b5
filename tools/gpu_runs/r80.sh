# dK/dV kernel: dO^T / Q^T fragments read one MFMA ahead (kv2) vs current; determinism
set -o pipefail
O=gpurun_out/r80; mkdir -p $O
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/cur.so abl/kv2.so bwd > $O/ab_kv2.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/kv2.so 4 > $O/det_kv2.log 2>&1
