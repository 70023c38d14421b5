# round 4 g29: the Llama-3-8B headline for 1200 sampled steps (~7 min at 1 kHz, host packing):
# host RSS after warm-up against the end of the run
set -o pipefail
O=gpurun_out/g29; mkdir -p $O
timeout -k 10 900 python -u bench.py --steps 1200 --warmup 3 --ab-rounds 0 --skip-baseline --no-agent-baseline off \
  --host-pmu off --json-out $O/bench_long.json > $O/bench_long.log 2>&1
