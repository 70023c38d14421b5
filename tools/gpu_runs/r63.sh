set -o pipefail
O=gpurun_out/r63; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/attn_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/probes/attn_backends.py > $O/attn.log 2>&1
