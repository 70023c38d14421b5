# round 4 g19: does a kernel-dispatch tracing context that was started once also keep heap per
# later dispatch?  And the same loop with dispatch counting started once at 1/10 the dispatch rate.
set -o pipefail
O=gpurun_out/g19; mkdir -p $O
timeout -k 10 150 python -u tools/soak_ondemand.py --minutes 1.2 --services kernel_trace --no-sampler \
  --capture-once --out $O/ktrace_once.json > $O/ktrace_once.log 2>&1 && \
timeout -k 10 150 python -u tools/soak_ondemand.py --minutes 1.2 --services kernel_trace --no-sampler \
  --out $O/ktrace_every5s.json > $O/ktrace_every5s.log 2>&1
