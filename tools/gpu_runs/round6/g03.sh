#!/bin/bash
# round 6 g03: the whole GPU suite after the mfma pass, the monitor seam, the
# sidecar's rate guard / re-attach, the retired modes and the growable staging
set -o pipefail
O=gpurun_out/r6g03; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
grep -E "passed|failed" $O/pytest.log | tail -3
exit $rc
