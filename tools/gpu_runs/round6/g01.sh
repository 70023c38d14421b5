#!/bin/bash
# round 6 g01: mfma-pass calibration (exact-count FP8/FP6/FP4/INT8/BF16 loads,
# FP8 GEMM), PCIe directional-bytes probe, daemon per-thread CPU at 1 kHz
set -o pipefail
O=gpurun_out/r6g01; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_agent.py -x -v --timeout 280 --timeout-method thread \
  -k "mfma_pass or precision_pass" -s > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
tail -5 $O/pytest.log
[ $rc -le 1 ] || exit $rc   # a GPU failure: nothing more on the GPU
timeout -k 10 90 python -u tools/probes/pci_throughput.py > $O/pci.json 2> $O/pci.err || exit $?
timeout -k 10 90 python -u tools/probes/daemon_thread_cpu.py 5 > $O/daemon_cpu.json 2> $O/daemon_cpu.err || exit $?
