#!/bin/bash
# Round 5 g17: after splitting Agent.cpp: the agent, kernel and sidecar tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g17
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_agent.py tests/test_gpu_kernels.py "tests/test_gpu_daemon.py::test_agent_sidecar_takes_daemon_slots" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
