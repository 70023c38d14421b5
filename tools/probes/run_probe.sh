#!/bin/bash
# GPU feasibility probe driver (run via gpurun)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/probe
id > gpurun_out/probe/id.txt
rocm-smi --showtopo > gpurun_out/probe/topo.txt 2>&1 || true
ls -la /dev/kfd /dev/dri >> gpurun_out/probe/id.txt 2>&1 || true
cat /proc/sys/kernel/perf_event_paranoid >> gpurun_out/probe/id.txt 2>&1 || true
ls /sys/devices | tr '\n' ' ' >> gpurun_out/probe/id.txt; echo >> gpurun_out/probe/id.txt
grep -m1 "model name\|cpu family" /proc/cpuinfo >> gpurun_out/probe/id.txt; grep -m1 "^model\s" /proc/cpuinfo >> gpurun_out/probe/id.txt
timeout -k 10 120 ./tools/probes/probe_counters inproc > gpurun_out/probe/inproc.log 2>&1 && \
timeout -k 10 120 ./tools/probes/probe_counters external > gpurun_out/probe/external.log 2>&1 && \
timeout -k 10 400 python tools/probes/probe_llama.py 1 4096 > gpurun_out/probe/llama_1x4096.log 2>&1
echo done rc=$?
