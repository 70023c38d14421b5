#!/bin/bash
# round 6 g08: the broadcast writer's liveness lock (a killed daemon is called
# stale after 500 ms, not 3 s) with every sidecar test, and the native
# DevMon suite under the strict rates of the GPU box
set -o pipefail
O=gpurun_out/r6g08; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -s -k "sidecar or strict" \
  tests/test_gpu_daemon.py tests/test_gpu_agent.py tests/test_native.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -25
exit $rc
