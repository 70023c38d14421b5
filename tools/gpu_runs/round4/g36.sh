# round 4 g36: the default headline three times in fresh processes on one box (host packing,
# lite, 1 kHz, two no-agent children per side each): the spread of both overhead figures
set -o pipefail
O=gpurun_out/g36; mkdir -p $O
timeout -k 10 1000 python -u bench.py --steps 10 --warmup 3 --host-pmu off \
  --overhead-matrix "lite,lite,lite" --matrix-out $O/overhead_matrix.json > $O/matrix.out 2> $O/matrix.err
