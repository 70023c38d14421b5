#!/bin/bash
# Round 5 g09: the catch-up gather (step(catch_up=True)) on the RCCL path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g09
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_agent.py -k "rccl_gather_path" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --force-collective --steps 20 --warmup 5 --skip-baseline --no-agent-baseline off \
  --json-out $O/fc.json > $O/fc.log 2>&1 || { tail -20 $O/fc.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/fc.json'));a=d['agent'];print(d['value'], d['ms_per_step'], d.get('samples_per_rank'), {k:a.get(k) for k in ('gather_backlog','gather_slots','step_packed','gather_cap_slots_now')})"
