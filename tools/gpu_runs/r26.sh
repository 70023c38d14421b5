# deeper staging: counter rate with the fused optimizer (run-ahead host)
set -o pipefail
O=gpurun_out/r26; mkdir -p $O
timeout -k 10 300 python -u bench.py --ab-rounds 2 > $O/fusedopt.log 2>&1
