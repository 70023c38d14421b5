#!/bin/bash
# Round 5 g39: the sidecar takes the sampling over when a daemon on the auto set
# drops to its readable-only set; the daemon and agent test files after the change.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g39
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_daemon.py tests/test_gpu_agent.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -8
exit $rc
