# round 3 g29: SQTT suite incl. kernel trace + SQTT + sampling in one process
set -o pipefail
O=gpurun_out/g29; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sqtt.py -m gpu -x -v --timeout 320 --timeout-method thread > $O/pytest_sqtt.log 2>&1
