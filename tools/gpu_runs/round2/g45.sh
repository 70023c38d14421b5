# validation after the fused cross-entropy backward: full GPU suite, smoke, headline bench
set -o pipefail
O=gpurun_out/g45; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py --json-out $O/bench.json > $O/bench_headline.log 2>&1
