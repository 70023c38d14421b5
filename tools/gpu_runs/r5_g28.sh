#!/bin/bash
# Round 5 g28: the default path after the fallback change: multi-rank
# rehearsals and the headline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/${RUN_ID:-g28}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multirank_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
