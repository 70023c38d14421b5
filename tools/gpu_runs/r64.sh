set -o pipefail
O=gpurun_out/r64; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_agent.py > $O/agent_tests.log 2>&1
