set -o pipefail
O=gpurun_out/r49; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_gpu.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/probes/wgrad_layouts.py > $O/wgrad.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-agent > $O/bench_noagent.log 2>&1
