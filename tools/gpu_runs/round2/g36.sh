# RMSNorm kernels with the residual / weight loads hoisted above the row reduction: numerics, bandwidth probe, step A/B-free profile
set -o pipefail
O=gpurun_out/g36; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -k "rms or adamw or tiny_llama" > $O/pytest_ops.log 2>&1 && \
timeout -k 10 120 python -u tools/probes/norm_bw.py > $O/norm_bw.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o step -- python3 bench.py --steps 3 --warmup 2 --no-agent --host-pmu off > $O/prof.log 2>&1
