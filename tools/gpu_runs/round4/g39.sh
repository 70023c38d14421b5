# round 4 g39: paused windows with 0, 2 and 6 untimed settle steps after the pause (lite, 1 kHz,
# host packing; fresh process each, two no-agent children per side)
set -o pipefail
O=gpurun_out/g39; mkdir -p $O
timeout -k 10 1000 python -u bench.py --steps 10 --warmup 3 --host-pmu off \
  --overhead-matrix "lite@s0,lite@s2,lite@s6" --matrix-out $O/overhead_matrix.json > $O/matrix.out 2> $O/matrix.err
