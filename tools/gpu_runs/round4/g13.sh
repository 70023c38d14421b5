# round 4 g13: heap growth with on-demand services configured but never used (~10 kernel
# dispatches per step, ~1000 steps/s): dispatch counting configured; kernel tracing configured
set -o pipefail
O=gpurun_out/g13; mkdir -p $O
timeout -k 10 240 python -u tools/soak_ondemand.py --minutes 2.5 --services dispatch_counters --no-captures \
  --out $O/soak_dcount_idle.json > $O/soak_dcount_idle.log 2>&1 && \
timeout -k 10 240 python -u tools/soak_ondemand.py --minutes 2.5 --services kernel_trace --no-captures \
  --out $O/soak_ktrace_idle.json > $O/soak_ktrace_idle.log 2>&1
