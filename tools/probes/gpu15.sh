cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r15
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r15/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r15/pytest.log; exit 1; }
tail -2 gpurun_out/r15/pytest.log
timeout -k 10 400 python bench.py --ab-rounds 6 --json-out gpurun_out/r15/bench.json --log-file gpurun_out/r15/agent.log > gpurun_out/r15/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 gpurun_out/r15/bench.log; exit 1; }
cat gpurun_out/r15/bench.json
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r15/smoke.log 2>&1 && echo smoke-ok
