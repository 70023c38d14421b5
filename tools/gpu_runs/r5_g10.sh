#!/bin/bash
# Round 5 g10: the headline exactly as the driver runs it (defaults: daemon
# sidecar sampler, step packing), twice, then the in-process sampler once.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g10
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench_$i.json > $O/bench_$i.log 2>&1 || { tail -30 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --sampler agent --json-out $O/bench_agent.json > $O/bench_agent.log 2>&1 || { tail -30 $O/bench_agent.log; exit 1; }
tail -1 $O/bench_agent.log
