#!/bin/bash
# Round 5 g40: the driver's round-end sequence after the reduced-set takeover, in one lease:
# full `pytest -m gpu` in one pass, smoke(), one default headline bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g40
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d.get('tracing_overhead_pct'), d.get('overhead_vs_no_agent_pct'), d['config']['sampler'])"
