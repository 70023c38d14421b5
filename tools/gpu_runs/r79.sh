# sampler kernels: occupancy / wave counters under rocprofv3 --pmc (one pass, kernel-trace only), and per-phase counters of the current step
set -o pipefail
O=gpurun_out/r79; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc -o pack -- python3 tools/bench_pack_kernel.py --iters 50 > $O/pmc.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 10 --phases > $O/bench_phases.log 2>&1
