#!/bin/bash
# Round 5 g30: the headline with the sidecar daemon killed at warmup step 2:
# the agent falls back to in-process sampling, the run completes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g30
mkdir -p $O
cd $R
timeout -k 10 600 python -u bench.py --steps 20 --warmup 15 --fault-kill-daemon 2 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep -E "fault injection|stopped publishing|has not been updated|RPC failed" $O/bench.log | head -5
python3 -c "import json;d=json.load(open('$O/bench.json'));a=d['agent'];print(d['value'], d.get('tracing_overhead_pct'), d.get('overhead_vs_no_agent_pct'), {k:a.get(k) for k in ('sampler','sidecar_stale','sidecar_fell_back','sidecar_fallback_after_ms')}, d.get('sidecar_rpc_errors'))"
