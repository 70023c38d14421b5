#!/bin/bash
# Round 5 g03: step-pack / sidecar GPU tests, the cold-capture probe of the
# round-4 gate failure, and rocprofv3 of the step pack kernel microbenchmark.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5
mkdir -p $O/g03_prof
cd $R
timeout -k 10 780 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_agent.py tests/test_gpu_dispatch_counters.py \
  tests/test_gpu_daemon.py -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  -k "step or pack_modes_agree or stuck_consumer or dispatch or sidecar or gpukernels or rccl_gather" > $O/g03_tests.log 2>&1
rc=$?
tail -30 $O/g03_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # a test failure still lets the probes run; a crash / timeout does not
timeout -k 10 180 python -u tools/probes/cold_capture.py > $O/g03_cold_capture.jsonl 2> $O/g03_cold_capture.err || exit $?
cat $O/g03_cold_capture.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/g03_prof -o step_pack -- python3 $R/tools/bench_step_pack.py --iters 50 --json-out $O/g03_step_pack.json > $O/g03_rocprof.log 2>&1 || exit $?
cat $O/g03_step_pack.json
exit $rc
