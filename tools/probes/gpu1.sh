cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1/smoke.log 2>&1; echo "smoke rc=$?" >> gpurun_out/r1/smoke.log
timeout -k 10 500 python bench.py --steps 8 --warmup 3 --log-file gpurun_out/r1/agent.log > gpurun_out/r1/bench.log 2>&1; echo "bench rc=$?" >> gpurun_out/r1/bench.log
