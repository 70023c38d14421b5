cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r7
timeout -k 10 600 python tools/overhead_probe.py --out gpurun_out/r7/overhead.json > gpurun_out/r7/overhead.log 2>&1
echo "rc=$?"
