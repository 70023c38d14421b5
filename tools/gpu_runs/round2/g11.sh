# sample-rate sweep on the current step (no counting buffer, faster workload)
set -o pipefail
O=gpurun_out/g11; mkdir -p $O
timeout -k 10 900 python -u bench.py --ab-rounds 4 --sweep-hz 500,1000,2000,3000,4000,0 --sweep-out $O/rate_sweep.json --json-out $O/bench.json > $O/bench.log 2>&1
