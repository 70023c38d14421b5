# per-rank window counting in bench.py: multi-rank rehearsals (2/4/8 ranks on the one GPU) + agent suite
set -o pipefail
O=gpurun_out/g38; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_multirank_gpu.py tests/test_gpu_agent.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
