cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r14
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_agent.py -m gpu -x -q > gpurun_out/r14/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r14/pytest.log; exit 1; }
tail -2 gpurun_out/r14/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r14/prof -o kern -- python3 $GRAFT_REPO_ROOT/tools/bench_pack_kernel.py --iters 200 > $GRAFT_REPO_ROOT/gpurun_out/r14/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r14/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r14/prof -name "*kernel_stats.csv" -exec cat {} \;
