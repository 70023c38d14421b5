# round 4 g52: g49 again with the daemon's achieved sample rate recorded while each daemon-sampled child runs
# started-once / countable / paused / in-process sampling / daemon sampling a countable child
set -o pipefail
O=gpurun_out/g52; mkdir -p $O
timeout -k 10 900 python -u bench.py --child-probe 3 --child-probe-soak 0 --child-probe-daemon \
  --json-out $O/probe.json > $O/probe.log 2>&1
