#!/bin/bash
# Round 5 g06: every agent launch on the trainer's stream (no drain stream):
# kernel / agent / multi-rank tests, then the fc probe against no-agent.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g06
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_agent.py tests/test_multirank_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in none fc; do
  timeout -k 10 300 python -u tools/probes/fc_trace.py --mode $m --out $O/t_$m.json > $O/$m.json 2> $O/$m.err || exit $?
  python3 -c "import json;d=json.loads(open('$O/$m.json').read().strip().splitlines()[-1]);print('$m', d['ms_per_step'], d['gpu_busy_ms'], d['agent'], flush=True)"
done
