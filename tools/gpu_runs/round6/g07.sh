#!/bin/bash
# round 6 g07/g08: the sidecar hand-back (a job that took its GPU's sampling over
# returns to a healthy daemon) and every other sidecar test
set -o pipefail
O=gpurun_out/r6g07; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -s -k sidecar \
  tests/test_gpu_daemon.py tests/test_gpu_agent.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -25
exit $rc
