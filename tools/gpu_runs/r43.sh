set -o pipefail
O=gpurun_out/r43; mkdir -p $O
timeout -k 10 300 python -u tools/probes/wgrad_layouts.py > $O/wgrad.log 2>&1
