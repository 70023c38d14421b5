# where the tracing overhead comes from: paused vs counters-on-at-1-Hz vs 1 kHz sampling, pooled interleaved windows, per counter set
set -o pipefail
O=gpurun_out/g18; mkdir -p $O
P=tools/probes/overhead_split.py
timeout -k 10 240 python -u $P --counter-set lite --out $O/lite.json > $O/lite.log 2>&1 && \
timeout -k 10 240 python -u $P --counter-set core --out $O/core.json > $O/core.log 2>&1 && \
timeout -k 10 240 python -u $P --counter-set GRBM_COUNT,GRBM_GUI_ACTIVE --out $O/grbm.json > $O/grbm.log 2>&1 && \
timeout -k 10 240 python -u $P --counter-set GRBM_COUNT,GRBM_GUI_ACTIVE,TCC_EA0_RDREQ,TCC_EA0_WRREQ --out $O/tcc.json > $O/tcc.log 2>&1
