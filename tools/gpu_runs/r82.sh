# final validation of round 1: full GPU suite, smoke, headline bench, daemon/agent tests
set -o pipefail
O=gpurun_out/r82; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $O/bench_headline.log 2>&1
