set -o pipefail
O=gpurun_out/r65; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py > $O/tests.log 2>&1 && \
export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o step -- python3 bench.py --steps 3 --warmup 2 --no-agent > $O/prof.log 2>&1
