# ping-pong forward with the exp/sum moved into the V-load segment (pp3), + static prio for the lagging half (pp4), vs current
set -o pipefail
O=gpurun_out/r78; mkdir -p $O
for v in pp3 pp4; do timeout -k 10 120 python -u tools/probes/attn_ab.py abl/cur.so abl/$v.so fwd > $O/ab_$v.log 2>&1 || exit 1; done
timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/pp3.so 4 > $O/det_pp3.log 2>&1
