# round 4 g14: is the ~2 MB of heap per on-demand capture the counting context's restart?
# agent paused / resumed every 5 s; agent rotating two counter passes every pack batch
set -o pipefail
O=gpurun_out/g14; mkdir -p $O
timeout -k 10 200 python -u tools/soak_ondemand.py --minutes 1.5 --services none --pause-rounds \
  --out $O/soak_pause.json > $O/soak_pause.log 2>&1 && \
timeout -k 10 200 python -u tools/soak_ondemand.py --minutes 1.5 --services none --counter-passes lite:1,core:1 \
  --out $O/soak_passes.json > $O/soak_passes.log 2>&1
