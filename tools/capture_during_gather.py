"""torchrun script: an exact dispatch-counter capture on ONE rank while every
rank keeps issuing its per-step RCCL gathers (tests/test_multirank_gpu.py).

A capture holds only the capturing rank's counter sampler (Agent::
holdSampler); its step() keeps gathering, so the ranks' collectives stay
matched.  Before that fix the capture paused the whole agent on that rank,
which skipped its gathers while its peers enqueued theirs (a hang, or
mismatched gathers).  Prints one RESULT line per rank."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynolog_amd import agent  # noqa: E402

agent.preinit([0], dispatch_counters=True)

import torch  # noqa: E402
from dynolog_amd.parallel import dist as pdist  # noqa: E402

env = pdist.init()
torch.cuda.set_device(0)
ag = agent.GpuAgent.start(device=0, rank=env.rank, world=env.world, sample_hz=1000, gather_mode="gather",
                          sinks=("memory",), comm_init_timeout_ms=60000)
x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
res = {"rank": env.rank, "gather_mode": ag.config.get("gather_mode"), "fallback": ag.config.get("fallback_from")}
steps = 30
dc = None
held = []
for it in range(steps):
    if env.rank == 1 and it == 10:
        dc = agent.DispatchCounters(kernel_regex="Cijk", dispatches=2).start()
    for _ in range(4):
        y = x @ x  # noqa: F841
    ag.step()
    torch.cuda.synchronize()
    if dc is not None:
        held.append(ag.stats().get("sampler_held"))
    if env.rank == 1 and it == 12:
        out = dc.finish(timeout_s=20)
        res["counted"] = out.get("counted")
        dc = None
pdist.barrier()
ag.pack_pending()
pdist.barrier()
ag.step()
torch.cuda.synchronize()
pdist.barrier()
if ag.is_aggregator:
    ag.flush()
st = ag.stats()
res.update(gathers=st["gathers"], steps=st["steps"], samples_taken=st["samples_taken"],
           samples_failed=st["samples_failed"], sampler_held_during=any(held), sampler_held_end=st["sampler_held"],
           last_error=st.get("last_error"), gather_failed=st.get("gather_failed"))
if ag.is_aggregator:
    res["received"] = [r["received"] for r in st["ranks"]]
ag.stop()
print("RESULT " + json.dumps(res), flush=True)
pdist.shutdown()
