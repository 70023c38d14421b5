cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r9
for cs in full lite core; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --counter-set $cs \
    --log-file gpurun_out/r9/agent_$cs.log --json-out gpurun_out/r9/bench_$cs.json \
    --sweep-hz 1000,2000,0 --sweep-out gpurun_out/r9/sweep_$cs.json > gpurun_out/r9/bench_$cs.log 2>&1 || { echo "bench $cs rc=$?"; exit 1; }
done
echo ok
