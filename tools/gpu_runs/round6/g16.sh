#!/bin/bash
# round 6 g16: sidecar vs in-process sampling alternated in one lease on the
# final tree (two pairs), each entry a fresh bench process with its own
# no-agent children
set -o pipefail
O=gpurun_out/r6g16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u bench.py --overhead-matrix "lite@daemon,lite@step,lite@daemon,lite@step" \
  --steps 20 --warmup 5 --matrix-out $O/matrix.json > $O/matrix.log 2>&1; rc=$?
python3 - <<PY
import json
d = json.load(open("$O/matrix.json"))
for r in d.get("rows", []):
    print(json.dumps({k: r.get(k) for k in ("entry", "rc", "samples_per_sec", "ms_per_step", "pooled_overhead_pct",
                                            "overhead_vs_no_agent_pct", "sample_latency_us_avg")}))
print(json.dumps({"countable_only_vs_no_agent_pct": d.get("countable_only_vs_no_agent_pct")}))
PY
exit $rc
