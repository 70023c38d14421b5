set -o pipefail
O=gpurun_out/r57; mkdir -p $O
timeout -k 10 400 python -u tools/probes/op_attrib.py > $O/attrib.log 2>&1
