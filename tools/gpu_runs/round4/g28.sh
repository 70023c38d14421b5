# round 4 g28: rate curve with host packing: lite at 2 kHz, 4 kHz and free-running, each a fresh
# headline process (pooled A/B + no-agent children)
set -o pipefail
O=gpurun_out/g28; mkdir -p $O
timeout -k 10 700 python -u bench.py --steps 10 --warmup 3 --ab-rounds 6 --ab-steps 5 --host-pmu off \
  --overhead-matrix "lite@hz2000,lite@hz4000,lite@hz0" --matrix-out $O/overhead_matrix.json > $O/matrix.out 2> $O/matrix.err
