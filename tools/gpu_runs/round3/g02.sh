# round 3 g02: GPU tests after the gather rework (agreed payload size, drain compaction,
# completed-pack gathers), smoke, 10-step headline bench
set -o pipefail
O=gpurun_out/g02; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --json-out $O/bench.json > $O/bench.log 2>&1
