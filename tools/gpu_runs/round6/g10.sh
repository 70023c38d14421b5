#!/bin/bash
# round 6 g10: after g09 -- a gone writer is detected 50 ms into a late
# heartbeat and the hand-back gate averages the daemon's rate over its hold:
# the sidecar tests, then the chaos soak again
set -o pipefail
O=gpurun_out/r6g10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v --timeout 240 --timeout-method thread -s -k sidecar \
  tests/test_gpu_daemon.py > $O/pytest.log 2>&1 || { grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -15; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 420 python -u tools/soak_sidecar.py --minutes 3 --every 10 --chaos-every 30 --chaos-down 2 \
  --out $O/soak_chaos.json > $O/soak_chaos.log 2>&1; rc=$?
grep -E "^\{" $O/soak_chaos.log | tail -20
exit $rc
