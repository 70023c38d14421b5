#!/bin/bash
# round 6 g30: rocprofv3 kernel statistics of the Llama-3-8B training step on
# the final tree (no agent: the workload's own kernels, bs2 x 4096)
set -o pipefail
O=gpurun_out/r6g30; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o llama -- python3 bench.py --no-agent --steps 3 --warmup 2 \
  --no-agent-baseline off --host-pmu off --json-out $O/bench_noagent.json > $O/rocprof.log 2>&1 || { tail -20 $O/rocprof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
echo "stats: $f"
head -25 "$f" | cut -c1-220
