# round 3 g04: GPU kernel / agent / daemon-counter tests after the FLOPS x64 fix; smoke
set -o pipefail
O=gpurun_out/g04; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_agent.py tests/test_gpu_daemon.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
