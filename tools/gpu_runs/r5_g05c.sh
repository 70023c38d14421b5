#!/bin/bash
# Round 5 g05c: kernel traces of the step with the agent on the RCCL gather path vs local
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g05c
mkdir -p $O
cd $R
for m in fc local; do
  timeout -k 10 300 python -u tools/probes/fc_trace.py --mode $m --out $O/trace_$m.json > $O/$m.json 2> $O/$m.err || exit $?
  cat $O/$m.json
done
