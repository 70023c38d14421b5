#!/bin/bash
# Round 5 g37: sidecar vs in-process, alternated twice in one lease, in-process first (the reverse of g35).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 1100 python -u bench.py --overhead-matrix "lite@step,lite@daemon,lite@step,lite@daemon" \
  --steps 20 --warmup 5 --matrix-out $O/g37_matrix.json > $O/g37_matrix.log 2>&1
rc=$?
tail -1 $O/g37_matrix.log | cut -c1-300
exit $rc
