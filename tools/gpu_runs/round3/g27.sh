# round 3 g27: SQTT over 4 shader engines
set -o pipefail
O=gpurun_out/g27; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sqtt.py -k several -m gpu -x -v -s --timeout 320 --timeout-method thread > $O/pytest_sqtt.log 2>&1
