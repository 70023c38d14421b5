# round 4 g32 (and g33 with the soaked child, g37 / g38 with the paused / sampling-agent children):
# no-agent child probes, interleaved
set -o pipefail
O=gpurun_out/${1:-g32}; mkdir -p $O
timeout -k 10 800 python -u bench.py --child-probe 3 ${2:---child-probe-soak 0} --json-out $O/probe.json > $O/probe.log 2>&1
