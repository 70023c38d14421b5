#!/bin/bash
# Round 5 g12: the multi-rank rehearsals (now with the daemon sidecar as the
# bench default) and the fused-op checks after them.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g12
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py tests/test_ops_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
