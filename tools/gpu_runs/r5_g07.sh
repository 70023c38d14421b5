#!/bin/bash
# Round 5 g07: the g04 matrix again after the single-stream agent (g06) and
# the step-mode staging change (cacheable scratch + streaming copy).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 1100 python -u bench.py --overhead-matrix "lite@step@kb,lite@host@kb,lite@step@fc,lite@daemon" \
  --steps 20 --warmup 5 --matrix-out $O/g07_matrix.json > $O/g07_matrix.log 2>&1
rc=$?
tail -5 $O/g07_matrix.log
exit $rc
