# TunableOp: tune the QKV weight-gradient GEMM, write the result file, check it pinned in a fresh process
set -o pipefail
O=gpurun_out/g41; mkdir -p $O
timeout -k 10 200 python -u tools/probes/tunable_pin.py tune $O/tunableop_qkv_wgrad.csv > $O/tune.log 2>&1 && \
timeout -k 10 200 python -u tools/probes/tunable_pin.py check $O/tunableop_qkv_wgrad.csv > $O/check.log 2>&1
