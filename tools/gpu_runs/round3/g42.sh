# round 3 g42: soak RSS with SQTT only / dispatch counters only configured and exercised
set -o pipefail
O=gpurun_out/g42; mkdir -p $O
timeout -k 10 300 python -u tools/soak_ondemand.py --minutes 1.7 --services sqtt --out $O/sqtt.json > $O/sqtt.log 2>&1 && \
timeout -k 10 300 python -u tools/soak_ondemand.py --minutes 1.7 --services dispatch_counters --out $O/dcount.json > $O/dcount.log 2>&1
