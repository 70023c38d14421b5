# round 3 g07: vector-ALU peak FLOP/clk/SIMD per precision (pins the fp*_active denominators)
set -o pipefail
O=gpurun_out/g07; mkdir -p $O
timeout -k 10 120 ./build/probes/valu_peak > $O/valu_peak.log 2>&1
