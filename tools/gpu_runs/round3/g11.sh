# round 3 g11: collective path as a non-root member, step() inside a hipGraph capture with the
# sampler running, visible devices, agent thread CPU share; then the agent suite
set -o pipefail
O=gpurun_out/g11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_agent.py -k "non_root or graph_capture or visible_devices or samples_busy" -x -v -s --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_daemon.py -x -v --timeout 300 --timeout-method thread > $O/pytest_agent.log 2>&1
