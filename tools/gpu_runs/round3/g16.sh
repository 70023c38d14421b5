# round 3 g16: the same probe after binding to torch's runtime without importing torch; then the gputrace --gpu-counters test
set -o pipefail
O=gpurun_out/g16; mkdir -p $O
timeout -k 10 300 python -u tools/probes/agent_kineto_logs.py $O > $O/probe.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_daemon.py -k "gpu_counter_tracks" -x -v -s --timeout 300 --timeout-method thread > $O/pytest_ctrace.log 2>&1
