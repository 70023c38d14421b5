# bench with host PMU co-sampling (config 5 plumbing) + 2-rank rehearsal
set -o pipefail
O=gpurun_out/r68; mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 10 > $O/bench.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_gpu.py > $O/multirank.log 2>&1
