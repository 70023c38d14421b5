#!/bin/bash
# Round 5 g27: agent, kernel and daemon tests after the sidecar fallback.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/${RUN_ID:-g27}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_agent.py tests/test_gpu_kernels.py tests/test_gpu_daemon.py > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
