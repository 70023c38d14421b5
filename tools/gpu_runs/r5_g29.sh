#!/bin/bash
# Round 5 g29: 6-minute soak of the always-on sidecar.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g29
mkdir -p $O
cd $R
timeout -k 10 540 python -u tools/soak_sidecar.py --minutes 6 --every 30 --out $O/soak.json > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
grep -E '^\{' $O/soak.log | tail -3
