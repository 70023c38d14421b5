# round 4 g40: the default 1-GPU headline (six settle steps before paused windows)
set -o pipefail
O=gpurun_out/g40; mkdir -p $O
timeout -k 10 800 python -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1
