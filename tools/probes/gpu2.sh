set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r2/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1 && \
timeout -k 10 500 python bench.py --steps 10 --warmup 3 --log-file gpurun_out/r2/agent.log > gpurun_out/r2/bench.log 2>&1
echo "rc=$?"
