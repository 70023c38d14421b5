#!/bin/bash
# round 6 g17: sampler auto with a pass plan takes a daemon rotating the same
# passes; the sidecar tests and the agent's pass tests
set -o pipefail
O=gpurun_out/r6g17; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v --timeout 240 --timeout-method thread -s -k "sidecar or pass" \
  tests/test_gpu_daemon.py tests/test_gpu_agent.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -25
exit $rc
