# step kernel profile of the current tree (no agent) + sample-rate sweep with the catch-up pacing
set -o pipefail
O=gpurun_out/g33; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o step -- python3 bench.py --steps 3 --warmup 2 --no-agent --host-pmu off > $O/prof.log 2>&1 && \
timeout -k 10 900 python -u bench.py --ab-rounds 4 --sweep-hz 500,1000,2000,3000,4000,0 --sweep-out $O/rate_sweep.json --json-out $O/bench.json > $O/bench.log 2>&1
