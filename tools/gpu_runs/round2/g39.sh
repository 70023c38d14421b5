# PMC passes over the round-2 attention kernels (fwd, bwd) and the RMSNorm probe: MFMA busy, LDS traffic / bank conflicts, waves
set -o pipefail
O=gpurun_out/g39; mkdir -p $O
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $O/fwd -o fwd -- python3 tools/probes/attn_only.py fwd > $O/fwd.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $O/bwd -o bwd -- python3 tools/probes/attn_only.py bwd > $O/bwd.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/norm -o norm -- python3 tools/probes/norm_bw.py > $O/norm.log 2>&1
