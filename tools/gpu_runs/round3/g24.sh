# round 3 g24: first SQTT capture (dispatch thread trace) runs
set -o pipefail
O=gpurun_out/g24; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_sqtt.py -m gpu -x -v -s --timeout 320 --timeout-method thread > $O/pytest_sqtt.log 2>&1
