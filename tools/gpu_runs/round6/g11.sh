#!/bin/bash
# round 6 g11: sampler auto joins a daemon that comes up later; the agent
# test file (the sampler thread's loop now serves every mode) and the sidecar
# tests
set -o pipefail
O=gpurun_out/r6g11; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread -s \
  tests/test_gpu_agent.py "tests/test_gpu_daemon.py::test_sidecar_auto_joins_a_daemon_started_later" \
  tests/test_gpu_daemon.py -k "not test_gputrace and not smi" > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -60
exit $rc
