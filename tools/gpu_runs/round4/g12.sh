# round 4 g12: where the soak's heap growth comes from: the same loop (GEMMs + all_gather +
# step, ~1 kHz agent) with no on-demand service, and without the agent at all
set -o pipefail
O=gpurun_out/g12; mkdir -p $O
timeout -k 10 240 python -u tools/soak_ondemand.py --minutes 2.5 --services none \
  --out $O/soak_agent_only.json > $O/soak_agent_only.log 2>&1 && \
timeout -k 10 240 python -u tools/soak_ondemand.py --minutes 2.5 --no-agent \
  --out $O/soak_no_agent.json > $O/soak_no_agent.log 2>&1
