#!/bin/bash
# round 6 g19: g18's hand-back test failure in the whole suite (handed back in
# every sidecar-only run): the agent tests first (the runner then holds the
# GPU, as in the suite), then the sidecar tests, with the gate's diagnostics
set -o pipefail
O=gpurun_out/r6g19; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -v --timeout 240 --timeout-method thread -s \
  tests/test_gpu_agent.py tests/test_gpu_daemon.py -k "not smi and not gputrace" > $O/pytest.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $O/pytest.log | tail -8
grep -o '"sidecar_handback[a-z_]*": [^,]*' $O/pytest.log | sort | uniq -c | head -20
exit $rc
