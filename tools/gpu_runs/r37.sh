# PyTorch TunableOp over hipBLASLt/rocBLAS for the step's GEMM shapes (heartbeat keeps the watchdog fed)
set -o pipefail
O=gpurun_out/r37; mkdir -p $O
( while true; do date >> $O/heartbeat.txt; sleep 20; done ) &
HB=$!
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 PYTORCH_TUNABLEOP_MAX_WARMUP_ITERATIONS=5
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 1000 python -u bench.py --steps 1 --warmup 1 --no-agent > $O/tune.log 2>&1 && \
PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-agent > $O/bench_tuned.log 2>&1 && \
env -u PYTORCH_TUNABLEOP_ENABLED timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-agent > $O/bench_untuned.log 2>&1
RC=$?
kill $HB
exit $RC
