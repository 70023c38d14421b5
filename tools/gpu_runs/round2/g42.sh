# always-on agent soak: 1 kHz sampling + per-step gathers for 6 minutes under GEMM load (host RSS, GPU memory, counters)
set -o pipefail
O=gpurun_out/g42; mkdir -p $O
timeout -k 10 480 python -u tools/probes/agent_soak.py 360 $O/agent_soak.json > $O/agent_soak.log 2>&1
