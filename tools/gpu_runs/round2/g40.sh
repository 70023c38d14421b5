# TunableOp over the QKV / O weight-gradient GEMM shapes only (is hipBLASLt's default solution the fastest?)
set -o pipefail
O=gpurun_out/g40; mkdir -p $O
timeout -k 10 400 python -u tools/probes/tunable_qkv_wgrad.py > $O/tunable.log 2>&1
