# round 3 g17: the rocprofiler tool split into libdyno_rocprof.so (no HIP dependency) and
# registered through rocprofiler-sdk discovery under KINETO_USE_DAEMON: probes, the gputrace
# --gpu-counters test, then the agent suite on the force-configure path
set -o pipefail
O=gpurun_out/g17; mkdir -p $O
timeout -k 10 300 python -u tools/probes/agent_kineto_logs.py $O > $O/probe_logs.log 2>&1 && \
timeout -k 10 300 python -u tools/probes/agent_with_kineto.py > $O/agent_with_kineto.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_daemon.py -k "gpu_counter_tracks" -x -v -s --timeout 300 --timeout-method thread > $O/pytest_ctrace.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests/test_gpu_agent.py -x -v --timeout 300 --timeout-method thread > $O/pytest_agent.log 2>&1 && exit $rc
