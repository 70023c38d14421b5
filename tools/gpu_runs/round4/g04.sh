# round 4 g04: overhead per counter set on the Llama-3-8B headline (1 kHz): the headline run
# once per entry in a fresh process (pooled A/B, vs its own no-agent children) + a countable-only
# child.  (The first g04 run restarted the agent inside one process; its train step kept
# calling the stopped first agent, so it was re-run this way.)
#   a: core,lite,full   b: lean, core:3/lite:1, lite with the kernel breakdown, at 500 Hz, at 10 Hz (counting enabled, hardly sampled), pack batch 128
set -o pipefail
H=${1:-a}; O=gpurun_out/g04$H; mkdir -p $O
case "$H" in
  a) M="core,lite,full" ;;
  b) M="lean,core:3/lite:1,lite@kb,lite@hz500,lite@hz10,lite@b128" ;;
  *) M="$2" ;;
esac
timeout -k 10 1100 python -u bench.py --steps 10 --warmup 3 --ab-rounds 6 --ab-steps 5 --host-pmu off \
  --overhead-matrix "$M" --matrix-out $O/overhead_matrix.json > $O/matrix.out 2> $O/matrix.err
