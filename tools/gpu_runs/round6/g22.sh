#!/bin/bash
# round 6 g22: what the spinning HSA runtime thread of a countable process asks
# the kernel for (its /proc syscall file read 20000 times: syscall number, fd,
# request code), with and without a HIP queue created
set -o pipefail
O=gpurun_out/r6g22; mkdir -p $O
export TMPDIR=/tmp
P=tools/probes/agent_thread_cpu.py
timeout -k 10 120 python -u $P --mode none --syscalls 2000 > $O/none.json 2> $O/none.err || exit $?
timeout -k 10 120 python -u $P --mode countable --syscalls 20000 > $O/countable.json 2> $O/countable.err || exit $?
timeout -k 10 120 python -u $P --mode countable --no-kernel --syscalls 20000 > $O/countable_nokernel.json 2> $O/countable_nokernel.err || exit $?
timeout -k 10 120 python -u $P --mode preinit --syscalls 20000 > $O/preinit.json 2> $O/preinit.err || exit $?
cat $O/*.json
# the runtime's own WaitAny trace in a countable process (first 1 MB of it)
(HSA_WAIT_ANY_DEBUG=1 timeout -k 10 60 python -u $P --mode countable --secs 1 2>&1 >/dev/null | head -c 1000000 > $O/countable_waitany.txt) || true
wc -l $O/countable_waitany.txt; head -c 1500 $O/countable_waitany.txt
