# multi-rank rehearsals (2/4/8 ranks on the shm mailbox, RCCL-init fallback) + headline with per-rank step times
set -o pipefail
O=gpurun_out/g17; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_multirank.log 2>&1 && \
timeout -k 10 600 python -u bench.py --json-out $O/bench.json > $O/bench_headline.log 2>&1
