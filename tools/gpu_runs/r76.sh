# full suite + smoke + headline + step profile after the attention forward work and host PMU co-sampling
set -o pipefail
O=gpurun_out/r76; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $O/bench_headline.log 2>&1 && \
export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o step -- python3 bench.py --steps 3 --warmup 2 --no-agent > $O/prof.log 2>&1
