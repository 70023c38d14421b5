# round 4 g20: 10-minute soak of the 1 kHz agent with an on-demand capture every 5 s (SQTT,
# RCCL comm trace, kernel trace in turn; dispatch counting is soaked apart, g18): host RSS
# and heap must level off once the bounded histories are full (~131 s)
set -o pipefail
O=gpurun_out/g20; mkdir -p $O
timeout -k 10 720 python -u tools/soak_ondemand.py --minutes 10 --services sqtt,comm_trace,kernel_trace \
  --out $O/soak_10min.json > $O/soak_10min.log 2>&1
