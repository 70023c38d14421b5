# attention backward: causal mask only on diagonal tiles (v1: dQ kernel, v2: + dK/dV kernel)
set -o pipefail
O=gpurun_out/g12; mkdir -p $O
for v in v1 v2; do
  timeout -k 10 180 python -u tools/probes/attn_ab.py abl/base.so abl/$v.so bwd > $O/ab_$v.log 2>&1 || exit $?
done
timeout -k 10 180 python -u tools/probes/attn_determinism.py abl/v2.so 4 > $O/det_v2.log 2>&1
