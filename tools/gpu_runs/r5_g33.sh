#!/bin/bash
# Round 5 g33: smoke() and two more headline runs on the final tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g33
mkdir -p $O
cd $R
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench_$i.json > $O/bench_$i.log 2>&1 || { tail -30 $O/bench_$i.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print($i, d['value'], d['ms_per_step'], d.get('tracing_overhead_pct'), d.get('overhead_vs_no_agent_pct'), d['config']['sampler'])"
done
