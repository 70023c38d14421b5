#!/bin/bash
# Round 5 g24: the headline as the driver runs it, on the final tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g24
mkdir -p $O
cd $R
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
