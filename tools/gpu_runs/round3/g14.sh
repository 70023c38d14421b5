# round 3 g14: which libkineto daemon-mode setting keeps the agent's counting context startable
set -o pipefail
O=gpurun_out/g14; mkdir -p $O
timeout -k 10 400 python -u tools/probes/agent_with_kineto.py > $O/agent_with_kineto.log 2>&1
