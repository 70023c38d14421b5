#!/bin/bash
# round 6 g09: chaos soak of the always-on sidecar -- the daemon is killed
# every 30 s and a new one started 2 s later, for 3 minutes; the job's agent
# takes over each time and hands back to the new daemon (tools/soak_sidecar.py)
set -o pipefail
O=gpurun_out/r6g09; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u tools/soak_sidecar.py --minutes 3 --every 10 --chaos-every 30 --chaos-down 2 \
  --out $O/soak_chaos.json > $O/soak_chaos.log 2>&1; rc=$?
grep -v "^\[\|^I2\|^W2\|^E2" $O/soak_chaos.log | tail -25
exit $rc
