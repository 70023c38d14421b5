# sample-rate sweep on the current workload (overhead vs rate)
set -o pipefail
O=gpurun_out/r66; mkdir -p $O
timeout -k 10 900 python -u bench.py --steps 10 --sweep-hz 250,500,1000,2000,3000,0 --sweep-out $O/sweep.json > $O/bench.log 2>&1
