# round 3 g26: SQTT captures of the Llama-3-8B step's attention and GEMM kernels
set -o pipefail
O=gpurun_out/g26; mkdir -p $O
timeout -k 10 400 python -u tools/sqtt_llama3.py --out $O/sqtt_llama > $O/sqtt_llama.log 2>&1
