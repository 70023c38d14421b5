#!/bin/bash
# Round 5 g05b: the 1-rank RCCL gather path's 12 % -- per-window kernel breakdown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --force-collective --pack-mode step --steps 8 --warmup 3 --ab-rounds 2 \
  --kernel-breakdown --no-agent-baseline off --host-pmu off --json-out $O/g05b_fc_kb.json > $O/g05b_fc_kb.log 2>&1 || exit $?
python3 - <<PY
import json
d=json.load(open("$O/g05b_fc_kb.json"))
kb=d["kernel_breakdown"]
print(d["ms_per_step"], d["baseline_ms_per_step"])
print(json.dumps({k: kb[k] for k in ("per_step_active","per_step_paused","delta_wall_ms","delta_gpu_busy_ms","delta_idle_ms","agent_kernels_ms_per_step","trainer_kernel_delta_ms_per_step")}, indent=1))
for k in kb["top_slower_kernels"]: print(round(k["delta_ms_per_step"],3), k["name"][:100])
PY
