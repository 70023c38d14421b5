# round 3 g09: per-kernel counters across rotating counter passes (vector TFLOP/s per kernel
# class from the precision pass), the other kernel-counter / precision tests, counter tracks
set -o pipefail
O=gpurun_out/g09; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_agent.py -k "kernel_counters or precision or counter_tracks" -x -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
