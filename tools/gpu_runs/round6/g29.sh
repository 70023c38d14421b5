#!/bin/bash
# round 6 g29: the chaos soak on the final tree (daemon SIGKILLed every 30 s
# and restarted 2 s later under a sidecar job, 5 minutes)
set -o pipefail
O=gpurun_out/r6g29; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 540 python -u tools/soak_sidecar.py --minutes 5 --every 10 --chaos-every 30 --chaos-down 2 \
  --out $O/soak_chaos.json > $O/soak_chaos.log 2>&1; rc=$?
grep -E "^\{" $O/soak_chaos.log | tail -40
exit $rc
