# round 3 g01: rotating counter passes feasibility (config switch cost, per-precision VALU counters)
set -o pipefail
O=gpurun_out/g01; mkdir -p $O
timeout -k 10 120 ./build/probes/probe_passes $O/counters.txt > $O/probe_passes.log 2>&1
