# round 4 g04: overhead per counter set on the Llama-3-8B headline (1 kHz, pooled A/B and
# vs no-agent children, + a countable-only child)
set -o pipefail
O=gpurun_out/g04; mkdir -p $O
timeout -k 10 1100 python -u bench.py --steps 10 --warmup 3 --ab-rounds 6 --ab-steps 5 --host-pmu off \
  --overhead-matrix "core,lean,lite,full,core:3/lite:1" --matrix-out $O/overhead_matrix.json \
  > $O/matrix.out 2> $O/matrix.err
