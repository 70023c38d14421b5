# round 4 g43: the headline with the kernel breakdown, no-agent children tracing their window too
set -o pipefail
O=gpurun_out/g43; mkdir -p $O
timeout -k 10 900 python -u bench.py --kernel-breakdown --no-agent-children 2 --json-out $O/bench.json > $O/bench.log 2>&1
