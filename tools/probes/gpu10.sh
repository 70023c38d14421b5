cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r10
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r10/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r10/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r10/pytest_gpu.log
timeout -k 10 400 python bench.py --log-file gpurun_out/r10/agent.log --json-out gpurun_out/r10/bench.json > gpurun_out/r10/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/r10/bench.log; exit 1; }
cat gpurun_out/r10/bench.json
