# round 3 g13: agent start inside a process whose libkineto runs in daemon mode (with the
# hipFree(nullptr) runtime init at agent start), then the gputrace --gpu-counters test
set -o pipefail
O=gpurun_out/g13; mkdir -p $O
timeout -k 10 300 python -u tools/probes/agent_with_kineto.py > $O/agent_with_kineto.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_daemon.py -k "gpu_counter_tracks" -x -v -s --timeout 300 --timeout-method thread > $O/pytest_ctrace.log 2>&1
