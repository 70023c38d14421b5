"""Per-kernel GPU counters of the Llama-3-8B training step from the agent's
1 kHz device-wide samples (KernelTrace.counters, src/gpu/KernelCounters.h):
MFMA-busy share, bf16 TFLOP/s and HBM read / write GB/s while each kernel
class runs, without serialising kernels the way rocprofv3 --pmc does.

    python tools/kernel_counters_llama3.py --steps 6 --out gpurun_out/kc.json

Most of the step's kernels are shorter than the 1 ms sample period, so each
class's numbers are a least-squares estimate over the sample intervals it
touches; `purity` (kernel time / time of the touched intervals) and the
fit's R^2 say how well separated they are.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from dynolog_amd import agent as dagent
    dagent.preinit([0], kernel_trace=True)
    import torch
    from dynolog_amd.models.llama import CONFIGS, build_llama, lm_loss
    from dynolog_amd.ops.optim import FusedAdamW

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = CONFIGS[a.model]
    model = build_llama(a.model, device=dev, dtype=torch.bfloat16, seed=0)
    opt = FusedAdamW(model.parameters(), lr=1e-5, betas=(0.9, 0.95), weight_decay=0.1)
    d = torch.randint(0, cfg.vocab_size, (2, 4097), device=dev)
    x, y = d[:, :-1].contiguous(), d[:, 1:].contiguous()
    ag = dagent.GpuAgent.start(device=0, sample_hz=1000, sinks=())

    def step():
        loss = lm_loss(model(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        ag.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with dagent.KernelTrace() as kt:
        for _ in range(a.steps):
            step()
    ag.pack_pending()
    ag.step()
    torch.cuda.synchronize()
    ag.flush()
    res = kt.counters(top=a.top)
    ag.stop()
    print(f"{res['samples']} samples, {res['dispatches']} dispatches, clock shift "
          f"{res['clock_shift_us']:.0f} us, R^2 " +
          " ".join(f"{k}={v:.2f}" for k, v in res["r2"].items()))
    print(f"{'kernel':60s} {'calls':>6s} {'ms':>8s} {'purity':>6s} {'MFMA%':>6s} {'TF/s':>7s} "
          f"{'rdGB/s':>7s} {'wrGB/s':>7s}")
    for k in res["kernels"]:
        c = k["counters"]
        print(f"{k['name'][:60]:60s} {k['calls']:6d} {k['kernel_ms']:8.1f} {k['purity']:6.2f} "
              f"{c['mfma_busy_pct']:6.1f} {c['bf16_tflops']:7.0f} {c['hbm_read_gbps']:7.0f} "
              f"{c['hbm_write_gbps']:7.0f}"
              f"{'' if k['resolved'] else ('  (unresolved)' if k['solved'] else '  (mixed)')}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
