# round 4 g01: cross-process visibility of every device counter the daemon / agent use
set -o pipefail
O=gpurun_out/g01; mkdir -p $O
timeout -k 10 180 ./build/probes/probe_visibility $O/visibility.json > $O/probe_visibility.log 2>&1
