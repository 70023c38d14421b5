# round 4 g47: the daemon's always-on device counters (100 Hz and 1 kHz) against a training job
# without the agent: no daemon / daemon + plain job / daemon + countable job, interleaved
set -o pipefail
O=gpurun_out/g47; mkdir -p $O
timeout -k 10 500 python -u tools/daemon_counter_overhead.py --rounds 3 --hz 100 --out $O/daemon_overhead_100hz.json \
  > $O/daemon_overhead_100hz.log 2>&1 && \
timeout -k 10 500 python -u tools/daemon_counter_overhead.py --rounds 3 --hz 1000 --out $O/daemon_overhead_1khz.json \
  > $O/daemon_overhead_1khz.log 2>&1
