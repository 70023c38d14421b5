# per-kernel counters of the Llama-3-8B step (KernelTrace.counters over 6 traced steps) + the daemon kernel-trace RPC with counters
set -o pipefail
O=gpurun_out/g27; mkdir -p $O
timeout -k 10 400 python -u tools/kernel_counters_llama3.py --steps 6 --out $O/kernel_counters.json > $O/kernel_counters.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_daemon.py -x -v -k "gpukernels" --timeout 200 --timeout-method thread > $O/pytest_daemon.log 2>&1
