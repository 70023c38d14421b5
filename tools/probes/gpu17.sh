cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r17
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r17/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r17/pytest.log; exit 1; }
tail -2 gpurun_out/r17/pytest.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r17/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/r17/bench.log; exit 1; }
tail -1 gpurun_out/r17/bench.log
