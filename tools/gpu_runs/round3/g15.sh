# round 3 g15: rocprofiler-sdk trace logs of the agent start with / without libkineto daemon mode
set -o pipefail
O=gpurun_out/g15; mkdir -p $O
timeout -k 10 300 python -u tools/probes/agent_kineto_logs.py $O > $O/probe.log 2>&1
