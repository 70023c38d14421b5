cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r12
for hz in 1000 2000 3000; do
  timeout -k 10 400 python bench.py --sample-hz $hz --ab-rounds 6 --json-out gpurun_out/r12/bench_${hz}.json \
    --log-file gpurun_out/r12/agent_${hz}.log > gpurun_out/r12/bench_${hz}.log 2>&1 || { echo "bench $hz rc=$?"; tail -20 gpurun_out/r12/bench_${hz}.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r12/bench_${hz}.json'));print($hz,d['value'],d['tracing_overhead_pct'],d['overhead_pct_headline_window'],d['baseline_ms_per_step'],d['agent']['sample_latency_us_avg'],d['agent']['late_ticks'])"
done
