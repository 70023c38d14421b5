#!/bin/bash
# Round 5 g05: why the 1-rank RCCL gather path (force_collective) cost 12 %
# in g04 -- host time in step() and what it waits on, step vs host packing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
for pm in step host; do
  timeout -k 10 300 python -u bench.py --force-collective --pack-mode $pm --steps 8 --warmup 3 --ab-rounds 1 \
    --no-agent-baseline off --host-pmu off --json-out $O/g05_fc_$pm.json > $O/g05_fc_$pm.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('$O/g05_fc_$pm.json'));print('$pm', d['ms_per_step'], d.get('baseline_ms_per_step'), json.dumps({k:d['agent'].get(k) for k in ('step_host_us_avg','step_host_us_max','rccl_settle_waits','rccl_settle_wait_ms','gather_run_ahead_waits','run_ahead_wait_ms','recv_ingest_waits','gather_latency_us_avg','samples_taken')}))"
done
