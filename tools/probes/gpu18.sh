cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r18
timeout -k 10 600 python tools/bench_daemon.py status smi gputrace --out gpurun_out/r18/daemon_configs.json > gpurun_out/r18/daemon.log 2>&1 || { echo "bench_daemon rc=$?"; tail -40 gpurun_out/r18/daemon.log; exit 1; }
cat gpurun_out/r18/daemon_configs.json
