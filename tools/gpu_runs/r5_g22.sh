#!/bin/bash
# Round 5 g22: which threads burn CPU in a job process (torch only, agent tool
# registered, in-process sampling, sidecar) and in the daemon.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g22
mkdir -p $O
cd $R
for m in none preinit agent daemon; do
  timeout -k 10 120 python -u tools/probes/agent_thread_cpu.py --mode $m > $O/$m.json 2> $O/$m.err || { tail -5 $O/$m.err; exit 1; }
  grep '^{' $O/$m.json
done
timeout -k 10 120 python -u tools/probes/daemon_thread_cpu.py 4 > $O/daemon_threads.json 2> $O/daemon_threads.err || exit 1
grep '^{' $O/daemon_threads.json
