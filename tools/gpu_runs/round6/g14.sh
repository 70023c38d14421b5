#!/bin/bash
# round 6 g14: the sidecar tests after re-attach / hand-back started checking
# the restarted daemon's rate
set -o pipefail
O=gpurun_out/r6g14; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -s -k sidecar \
  tests/test_gpu_daemon.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -15
exit $rc
