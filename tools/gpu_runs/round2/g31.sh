# agent + multi-rank suites after moving the communicator bring-up to the top of Agent::start
set -o pipefail
O=gpurun_out/g31; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_agent.py tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
