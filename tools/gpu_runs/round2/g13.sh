# shm gather mode: multi-rank rehearsals (2 and 4 ranks on one GPU) + agent regression
set -o pipefail
O=gpurun_out/g13; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_gpu_agent.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
