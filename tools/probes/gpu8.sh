cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r8
P=./tools/probes/probe_counters
timeout -k 10 120 $P inproc GRBM_GUI_ACTIVE GRBM_COUNT > gpurun_out/r8/grbm.log 2>&1 && \
timeout -k 10 120 $P inproc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE > gpurun_out/r8/sq.log 2>&1 && \
timeout -k 10 120 $P inproc TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ_32B > gpurun_out/r8/tcc.log 2>&1 && \
timeout -k 10 120 $P inproc TCC_EA0_RDREQ TCC_EA0_WRREQ > gpurun_out/r8/tcc2.log 2>&1 && \
timeout -k 10 120 $P inproc SQ_WAVES GRBM_COUNT > gpurun_out/r8/sq1.log 2>&1
echo "rc=$?"
