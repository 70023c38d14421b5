# round 3 g37: overhead vs sampling rate on the final tree
set -o pipefail
O=gpurun_out/g37; mkdir -p $O
timeout -k 10 700 python -u bench.py --steps 10 --warmup 3 --no-agent-baseline off --sweep-hz 500,1000,2000,4000 --sweep-out $O/rate_sweep.json > $O/sweep.log 2>&1
