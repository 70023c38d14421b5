# round 4 g11: the headline with pack_mode host vs device (kernel breakdown for both), and
# host-packed core / full, each in a fresh process with its own no-agent children
set -o pipefail
O=gpurun_out/g11; mkdir -p $O
timeout -k 10 1100 python -u bench.py --steps 10 --warmup 3 --ab-rounds 6 --ab-steps 5 --host-pmu off \
  --overhead-matrix "lite@host@kb,lite@device@kb,lite@host,core@host,full@host" \
  --matrix-out $O/overhead_matrix.json > $O/matrix.out 2> $O/matrix.err
