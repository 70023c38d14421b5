# round 4 g16: dispatch-counting captures every 5 s with the 1 kHz sampler not running (so no
# device-counting restart after each capture)
set -o pipefail
O=gpurun_out/g16; mkdir -p $O
timeout -k 10 150 python -u tools/soak_ondemand.py --minutes 1.2 --services dispatch_counters --no-sampler \
  --out $O/soak_dc_nosampler.json > $O/soak_dc_nosampler.log 2>&1
