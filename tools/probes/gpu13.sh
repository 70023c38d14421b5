cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r13
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r13/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r13/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r13/pytest_gpu.log
timeout -k 10 400 python bench.py --phases --json-out gpurun_out/r13/bench_phases.json --log-file gpurun_out/r13/agent.log > gpurun_out/r13/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/r13/bench.log; exit 1; }
cat gpurun_out/r13/bench_phases.json
