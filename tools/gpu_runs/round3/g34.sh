# round 3 g34: RCCL collective tracing (in process and through the daemon); dispatch counters with cached configs
set -o pipefail
O=gpurun_out/g34; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_comm_trace.py tests/test_gpu_dispatch_counters.py -m gpu -x -v -s --timeout 320 --timeout-method thread > $O/pytest_ctrace.log 2>&1
