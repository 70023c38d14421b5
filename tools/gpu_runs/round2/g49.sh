# final check of the in-tree build after reverting the second RoPE attempt: op + attention tests, smoke
set -o pipefail
O=gpurun_out/g49; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ops.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
