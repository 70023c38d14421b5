cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r14; mkdir -p $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof2 -o kern -- python3 $GRAFT_REPO_ROOT/tools/bench_pack_kernel.py --iters 200 > $R/prof2.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $R/prof2.log; exit 1; }
find $R/prof2 -name "*kernel_stats.csv" -exec cat {} \;
