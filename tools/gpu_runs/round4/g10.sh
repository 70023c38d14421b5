# round 4 g10: pack_mode host (sampler-thread packing into a pinned host ring) — agent,
# dispatch-counting and multi-rank suites, then the headline in both pack modes with the
# kernel breakdown
set -o pipefail
O=gpurun_out/g10; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_dispatch_counters.py \
  -x -v --timeout 300 --timeout-method thread > $O/pytest_agent.log 2>&1
