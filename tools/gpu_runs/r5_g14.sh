#!/bin/bash
# Round 5 g14: the raw sidecar (the daemon broadcasts raw samples, the job's
# step kernel reduces them): its GPU test, then the headline with it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g14
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  "tests/test_gpu_daemon.py::test_agent_sidecar_takes_daemon_slots" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|passed" $O/tests.log | tail -2
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
