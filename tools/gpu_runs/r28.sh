# SDPA backends for the Llama-3-8B attention shape
set -o pipefail
O=gpurun_out/r28; mkdir -p $O
timeout -k 10 300 python -u tools/probes/attn_backends.py > $O/attn.log 2>&1
