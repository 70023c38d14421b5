# attention forward A/B vs current: static prio for waves 4-7 (v6), per-cluster prio flips (v7), one barrier per tile pair (v9)
set -o pipefail
O=gpurun_out/r72; mkdir -p $O
for v in v6 v7 v9; do timeout -k 10 120 python -u tools/probes/attn_ab.py abl/cur.so abl/$v.so fwd > $O/ab_$v.log 2>&1 || exit 1; done
