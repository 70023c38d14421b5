# validation after the RMSNorm load hoist, mailbox geometry checks and the shm-outcome agreement: full GPU suite, smoke, headline bench + rate sweep
set -o pipefail
O=gpurun_out/g37; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py --sweep-hz 2000,0 --sweep-out $O/rate_sweep.json --json-out $O/bench.json > $O/bench_headline.log 2>&1
