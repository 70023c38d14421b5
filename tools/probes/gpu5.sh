# round-1 GPU validation: gpu tests, bench + rate sweep, rocprofv3 kernel stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r5/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --log-file gpurun_out/r5/agent.log \
   --sweep-hz 100,500,1000,2000,0 --sweep-out gpurun_out/r5/sweep.json > gpurun_out/r5/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --skip-baseline > gpurun_out/r5/prof_bench.log 2>&1
echo "rc=$?"
