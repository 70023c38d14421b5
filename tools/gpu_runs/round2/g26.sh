# per-kernel counters (NNLS de-mixing) GPU test + agent suite (pacing change)
set -o pipefail
O=gpurun_out/g26; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_agent.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest_agent.log 2>&1
