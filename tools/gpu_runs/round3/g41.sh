# round 3 g41: where does the soak's host RSS growth come from? 100 s soaks with subsets of services
set -o pipefail
O=gpurun_out/g41; mkdir -p $O
timeout -k 10 300 python -u tools/soak_ondemand.py --minutes 1.7 --services none --out $O/none.json > $O/none.log 2>&1 && \
timeout -k 10 300 python -u tools/soak_ondemand.py --minutes 1.7 --services comm_trace --out $O/comm.json > $O/comm.log 2>&1 && \
timeout -k 10 300 python -u tools/soak_ondemand.py --minutes 1.7 --services kernel_trace --out $O/ktrace.json > $O/ktrace.log 2>&1
