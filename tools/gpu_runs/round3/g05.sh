# round 3 g05: daemon counter-selection test, smoke, headline bench with the no-agent baseline
# children (before/after) and the agreed-size gather
set -o pipefail
O=gpurun_out/g05; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_daemon.py -x -v -s --timeout 240 --timeout-method thread -k "counter" > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1
