# round 4 g50: the round-end tiers on the final tree: pytest -m gpu, smoke(), default bench
set -o pipefail
O=gpurun_out/g50; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
