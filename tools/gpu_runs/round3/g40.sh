# round 3 g40: 3-minute soak of dispatch counters / SQTT / RCCL traces next to the 1 kHz agent
set -o pipefail
O=gpurun_out/g40; mkdir -p $O
timeout -k 10 400 python -u tools/soak_ondemand.py --minutes 3 --out $O/soak_ondemand.json > $O/soak.log 2>&1
