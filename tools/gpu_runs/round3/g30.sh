# round 3 g30: first exact per-dispatch counter captures (in process and through the daemon)
set -o pipefail
O=gpurun_out/g30; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dispatch_counters.py tests/test_gpu_daemon.py -k "dispatch_counters or gpupmc" -m gpu -x -v -s --timeout 320 --timeout-method thread > $O/pytest_dcount.log 2>&1
