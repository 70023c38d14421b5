# round 4 g26: host packing without agent streams or device pack buffers: the agent suite, then
# the headline twice (fresh processes) for the paused-agent and sampling costs
set -o pipefail
O=gpurun_out/g26; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_agent.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_agent.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --ab-rounds 6 --ab-steps 5 --host-pmu off \
  --overhead-matrix "lite,lite,core" --matrix-out $O/overhead_matrix.json > $O/matrix.out 2> $O/matrix.err
