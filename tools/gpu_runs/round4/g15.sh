# round 4 g15: the heap cost of one dispatch-counting capture vs what it counts: 1 and 16
# dispatches per capture (lite), 4 dispatches of the 272-instance core set
set -o pipefail
O=gpurun_out/g15; mkdir -p $O
for v in "1 lite" "16 lite" "4 core"; do set -- $v
  timeout -k 10 150 python -u tools/soak_ondemand.py --minutes 1.2 --services dispatch_counters \
    --dc-dispatches $1 --dc-set $2 --out $O/soak_dc$1_$2.json > $O/soak_dc$1_$2.log 2>&1 || exit $?
done
