# transpose kernel variants at the step's shapes
set -o pipefail
O=gpurun_out/g06; mkdir -p $O
timeout -k 10 300 python -u tools/probes/transpose_variants.py > $O/transpose.log 2>&1
