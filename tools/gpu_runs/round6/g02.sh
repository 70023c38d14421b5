#!/bin/bash
# round 6 g02: the sidecar's new takeover / re-attach paths and the strict
# 8-simulated-GPU daemon rates on the GPU box
set -o pipefail
O=gpurun_out/r6g02; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_daemon.py tests/test_native.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -k "sidecar or devmon" -s > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
tail -15 $O/pytest.log
exit $rc
