#!/bin/bash
# Round 5 g19: the non-default paths after the single-stream fix: host
# packing on the RCCL gather path (round 4's world > 1 path, never timed
# before g05), and device packing (its side stream) with the kernel breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 1100 python -u bench.py --overhead-matrix "lite@host@fc,lite@device@kb" \
  --steps 20 --warmup 5 --matrix-out $O/g19_matrix.json > $O/g19_matrix.log 2>&1
rc=$?
tail -2 $O/g19_matrix.log | cut -c1-400
exit $rc
