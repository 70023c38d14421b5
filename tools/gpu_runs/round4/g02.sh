# round 4 g02: counter visibility across processes, with the job plain / with an idle
# rocprofiler-sdk tool / with a configured-but-stopped device counting context; MFMA types
set -o pipefail
O=gpurun_out/g02; mkdir -p $O
timeout -k 10 240 ./build/probes/probe_visibility $O/vis_plain.json plain $O/gfx950_counters.txt > $O/vis_plain.log 2>&1 && \
timeout -k 10 240 ./build/probes/probe_visibility $O/vis_tool.json tool > $O/vis_tool.log 2>&1 && \
timeout -k 10 240 ./build/probes/probe_visibility $O/vis_tool_dc.json tool_dc > $O/vis_tool_dc.log 2>&1
