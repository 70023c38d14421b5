#!/bin/bash
# Round 5 g04: the three pack modes priced in one lease (fresh process per
# entry, own no-agent children, per-window kernel breakdown), plus the step
# mode on the 1-rank RCCL gather path and the daemon sidecar.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 1140 python -u bench.py --overhead-matrix "lite@step@kb,lite@host@kb,lite@device@kb,lite@step@fc,lite@daemon" \
  --steps 20 --warmup 5 --matrix-out $O/g04_matrix.json > $O/g04_matrix.log 2>&1
rc=$?
tail -5 $O/g04_matrix.log
exit $rc
