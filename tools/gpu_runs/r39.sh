# PMC passes on the attention kernels
set -o pipefail
O=gpurun_out/r39; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/p1 -o p1 -- python3 tools/probes/attn_only.py bwd > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O/p2 -o p2 -- python3 tools/probes/attn_only.py bwd > $O/p2.log 2>&1
