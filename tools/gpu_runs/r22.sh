# fused AdamW with kernarg tensor lists: counter rate + step time
set -o pipefail
O=gpurun_out/r22; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py > $O/ops.log 2>&1 && \
timeout -k 10 300 python -u bench.py --ab-rounds 2 > $O/fused_fusedopt.log 2>&1
