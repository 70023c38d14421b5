# sampler starvation probe
set -o pipefail
O=gpurun_out/r24; mkdir -p $O
timeout -k 10 240 python -u tools/probes/sampler_starvation.py > $O/starve.log 2>&1
