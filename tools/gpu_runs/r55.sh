set -o pipefail
O=gpurun_out/r55; mkdir -p $O
export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o step -- python3 bench.py --steps 3 --warmup 2 --no-agent > $O/prof.log 2>&1
