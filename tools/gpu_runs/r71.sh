# validate the faster attention forward: numerics tests, fwd+bwd A/B vs HEAD~, short bench
set -o pipefail
O=gpurun_out/r71; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_ops_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/base.so abl/cur.so both > $O/ab.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 10 > $O/bench.log 2>&1
