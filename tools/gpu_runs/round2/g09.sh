# counter tracks in agent kernel traces: agent GPU tests
set -o pipefail
O=gpurun_out/g09; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_daemon.py -x -v --timeout 120 --timeout-method thread > $O/pytest_agent.log 2>&1
