#!/bin/bash
# Round 5 g20: the dead-daemon test and the sidecar test after the stale check.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g20
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_daemon.py::test_sidecar_reports_a_dead_daemon" "tests/test_gpu_daemon.py::test_agent_sidecar_takes_daemon_slots" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
