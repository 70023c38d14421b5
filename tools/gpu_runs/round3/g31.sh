# round 3 g31: per-kernel counters of the Llama-3-8B step, NNLS de-mix vs exact dispatch counting
set -o pipefail
O=gpurun_out/g31; mkdir -p $O
timeout -k 10 500 python -u tools/exact_vs_demix_llama3.py --out $O/exact_vs_demix.json > $O/exact_vs_demix.log 2>&1
