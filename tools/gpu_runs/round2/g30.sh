# does the HBM-bound AdamW overlap with compute-bound GEMMs on two streams? (+ attention tests on the one-barrier backward)
set -o pipefail
O=gpurun_out/g30; mkdir -p $O
timeout -k 10 200 python -u tools/probes/overlap_probe.py > $O/overlap.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1
