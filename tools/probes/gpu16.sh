cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r16
timeout -k 10 600 python -m pytest tests/test_gpu_agent.py -m gpu -x -q -k "slot_ring or phase or fault" > gpurun_out/r16/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r16/pytest.log; exit 1; }
tail -2 gpurun_out/r16/pytest.log
