# round 4 g25: rocprofv3 kernel statistics of the Llama-3-8B headline step without the agent
# (rocprofv3's own tool takes the rocprofiler configuration, so the agent cannot run under it;
# the agent's kernel cost under sampling is bench.py --kernel-breakdown, profiles/round4/g11)
set -o pipefail
O=gpurun_out/g25; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --no-agent --steps 5 --warmup 3 > $O/prof_bench.log 2>&1
