cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r11
timeout -k 10 600 python -m pytest tests/test_gpu_agent.py tests/test_gpu_daemon.py -m gpu -x -q -k "kernel_trace or gpukernels or forwards or topology" > gpurun_out/r11/pytest_new.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r11/pytest_new.log; exit 1; }
tail -3 gpurun_out/r11/pytest_new.log
timeout -k 10 400 python bench.py --kernel-trace-ready --json-out gpurun_out/r11/bench_ktready.json --log-file gpurun_out/r11/agent.log > gpurun_out/r11/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/r11/bench.log; exit 1; }
cat gpurun_out/r11/bench_ktready.json
