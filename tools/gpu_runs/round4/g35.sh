# round 4 g35: which counter blocks the per-read cost comes from (host packing, 1 kHz, fresh
# process each): GRBM only; GRBM + TCC requests; one SQ counter + GRBM; lite
set -o pipefail
O=gpurun_out/g35; mkdir -p $O
timeout -k 10 900 python -u bench.py --steps 10 --warmup 3 --ab-rounds 6 --ab-steps 5 --host-pmu off \
  --no-agent-children 1 \
  --overhead-matrix "GRBM_GUI_ACTIVE+GRBM_COUNT:1,GRBM_GUI_ACTIVE+GRBM_COUNT+TCC_EA0_RDREQ+TCC_EA0_WRREQ:1,SQ_WAVES+GRBM_GUI_ACTIVE+GRBM_COUNT:1,lite" \
  --matrix-out $O/overhead_matrix.json > $O/matrix.out 2> $O/matrix.err
