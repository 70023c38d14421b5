# round 4 g31: smoke and the default 1-GPU headline on the final tree
set -o pipefail
O=gpurun_out/g31; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 700 python -u bench.py --json-out $O/bench.json > $O/bench.log 2>&1
