# round 3 g03: VALU FLOPS counter calibration probe; GPU kernel + agent tests after the
# counter-pass rework (pass-aware pack kernel, precision pass, rotation); smoke
set -o pipefail
O=gpurun_out/g03; mkdir -p $O
timeout -k 10 120 ./build/probes/probe_passes $O/counters.txt > $O/probe_passes.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_agent.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
