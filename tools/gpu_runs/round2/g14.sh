# attention forward with a deferred running max (rescale only when the max grows by > 2^8)
set -o pipefail
O=gpurun_out/g14; mkdir -p $O
timeout -k 10 180 python -u tools/probes/attn_ab.py abl/base2.so abl/v4.so fwd > $O/ab_v4.log 2>&1 && \
timeout -k 10 180 python -u tools/probes/attn_determinism.py abl/v4.so 4 > $O/det_v4.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1
