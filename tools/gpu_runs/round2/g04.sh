# dgrad operand layouts (W as stored vs transposed copy) + transpose kernel bandwidth at weight shapes
set -o pipefail
O=gpurun_out/g04; mkdir -p $O
timeout -k 10 300 python -u tools/probes/dgrad_layouts.py > $O/dgrad_layouts.log 2>&1
