#!/bin/bash
# round 6 g13: the whole GPU suite after the hand-back, liveness lock, late join and departing-process changes, then
# smoke() and the default headline bench (the round-end sequence)
set -o pipefail
O=gpurun_out/r6g13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
grep -E "passed|failed" $O/pytest.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(json.dumps({k:d.get(k) for k in ('value','ms_per_step','tracing_overhead_pct','overhead_vs_no_agent_pct','vs_reference_ceiling','node_sampling_cpu')}))"
exit $rc
