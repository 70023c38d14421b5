# rocprofv3 kernel stats: (a) sampler kernels at production shapes, (b) the Llama-3-8B workload
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_pack -o pack --output-format csv -- python3 tools/bench_pack_kernel.py --iters 200 > gpurun_out/r6/prof_pack.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_llama -o llama --output-format csv -- python3 bench.py --no-agent --steps 3 --warmup 2 > gpurun_out/r6/prof_llama.log 2>&1
echo "rc=$?"
