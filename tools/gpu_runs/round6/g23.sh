#!/bin/bash
# round 6 g23: the agent test file after the agent started marking every GPU
# countable (countable_other_gpus), then smoke()
set -o pipefail
O=gpurun_out/r6g23; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_agent.py -m gpu -v --timeout 240 --timeout-method thread \
  > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
grep -E "passed|failed" $O/pytest.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
exit $rc
