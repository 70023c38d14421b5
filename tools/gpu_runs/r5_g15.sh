#!/bin/bash
# Round 5 g15: the sidecar's two forms and in-process step packing priced in
# one lease, each with the kernel breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 1100 python -u bench.py --overhead-matrix "lite@daemon@kb,lite@daemon@dslots@kb,lite@step@kb" \
  --steps 20 --warmup 5 --matrix-out $O/g15_matrix.json > $O/g15_matrix.log 2>&1
rc=$?
tail -3 $O/g15_matrix.log | cut -c1-600
exit $rc
