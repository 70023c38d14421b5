#!/bin/bash
# Round 5 g08: why does the 1-rank RCCL path deliver ~900 samples/s of 1000?
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5/g08
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --force-collective --steps 20 --warmup 5 --skip-baseline --no-agent-baseline off \
  --json-out $O/fc.json > $O/fc.log 2>&1 || { tail -20 $O/fc.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/fc.json'));print(d['value'], d.get('samples_per_rank'), json.dumps(d.get('agent')))"
