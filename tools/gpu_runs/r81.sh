# overhead precision on one box: two default headline runs + one with 20 interleaved A/B rounds
set -o pipefail
O=gpurun_out/r81; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_1.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench_2.log 2>&1 &&
timeout -k 10 900 python -u bench.py --ab-rounds 20 > $O/bench_ab20.log 2>&1
