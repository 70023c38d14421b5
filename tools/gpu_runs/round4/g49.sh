# round 4 g49: in-process vs daemon-side 1 kHz lite reads, interleaved in one run: plain /
# started-once / countable / paused / in-process sampling / daemon sampling a countable child
set -o pipefail
O=gpurun_out/g49; mkdir -p $O
timeout -k 10 900 python -u bench.py --child-probe 5 --child-probe-soak 0 --child-probe-daemon \
  --json-out $O/probe.json > $O/probe.log 2>&1
