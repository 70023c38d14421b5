#!/bin/bash
# Round 5 g13: the catch-up accounting in the multi-rank rehearsals, the
# non-root member path, then the fused-op checks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g13
mkdir -p $O
cd $R
timeout -k 10 1050 python -u -m pytest tests/test_multirank_gpu.py tests/test_ops_gpu.py "tests/test_gpu_agent.py::test_rccl_gather_path_as_non_root_member" -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
tail -5 $O/gputest.log
exit $rc
