# ping-pong attention forward (waves 4-7 one segment behind, K/V time-sharing registers) vs current
set -o pipefail
O=gpurun_out/r77; mkdir -p $O
timeout -k 10 120 python -u tools/probes/attn_ab.py abl/cur.so abl/pp2.so fwd > $O/ab_pp2.log 2>&1 &&
timeout -k 10 120 python -u tools/probes/attn_determinism.py abl/pp2.so 6 > $O/det_pp2.log 2>&1
