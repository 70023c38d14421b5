#!/bin/bash
# Round 5 g25: does an HSA runtime knob stop the spinning thread of a process
# with device counting configured?  (g22: a KFD ioctl loop in libhsa-runtime64)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g25
mkdir -p $O
cd $R
run() {  # label, env...
  local l=$1; shift
  timeout -k 10 100 env "$@" python -u tools/probes/agent_thread_cpu.py --mode preinit > $O/$l.json 2> $O/$l.err || { tail -3 $O/$l.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]);print('$l', d['total_pct'], d['threads'][0]['cpu_pct'], d['busiest_thread_pcs'][:1])"
}
run base X=1
run no_pcs HSA_DISABLE_PC_SAMPLING=1
run intr HSA_ENABLE_INTERRUPT=1
run mwaitx HSA_ENABLE_MWAITX=1
