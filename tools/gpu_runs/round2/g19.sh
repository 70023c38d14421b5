# (1) attention forward main-loop efficiency: causal kernel vs the same kernel run non-causal (abl/attn_nc.hip: all key tiles, no mask);
# (2) lean counter set: GPU test + overhead split next to lite on the same box
set -o pipefail
O=gpurun_out/g19; mkdir -p $O
P=tools/probes/overhead_split.py
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/base.so abl/nc.so fwd > $O/attn_nc.log 2>&1 && \
timeout -k 10 200 python -u -m pytest tests/test_gpu_agent.py -x -v -k lean --timeout 120 --timeout-method thread > $O/pytest_lean.log 2>&1 && \
timeout -k 10 240 python -u $P --counter-set lean --out $O/lean.json > $O/lean.log 2>&1 && \
timeout -k 10 240 python -u $P --counter-set lite --out $O/lite.json > $O/lite.log 2>&1
