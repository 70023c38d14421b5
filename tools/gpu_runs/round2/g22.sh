# longest-first attention grids: op + attention tests, headline bench, step kernel profile (no agent)
set -o pipefail
O=gpurun_out/g22; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ops.log 2>&1 && \
timeout -k 10 600 python -u bench.py --json-out $O/bench.json > $O/bench_headline.log 2>&1 && \
export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o step -- python3 bench.py --steps 3 --warmup 2 --no-agent > $O/prof.log 2>&1
