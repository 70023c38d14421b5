cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
timeout -k 10 120 python tools/probes/exit_c.py > gpurun_out/r4/c.log 2>&1; echo "c rc=$?" >> gpurun_out/r4/c.log
