"""Per-kernel counters of the Llama-3-8B step two ways, on the same process:

* statistical: the agent's 1 kHz device-wide samples de-mixed per kernel
  class by the NNLS fit over the sample intervals (KernelTrace.counters,
  src/gpu/KernelCounters.h; nothing is serialised);
* exact: rocprofiler-sdk dispatch counting of a few dispatches of each
  kernel family (DispatchCounters, src/gpu/DispatchCounters.h; serialised).

    python tools/exact_vs_demix_llama3.py --out gpurun_out/exact_vs_demix.json

Prints MFMA busy %, bf16 TFLOP/s and HBM read / write GB/s per family both
ways, so the statistical path the daemon serves for every kernel can be
checked against ground truth on the kernels that matter.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FAMILIES = [
    ("attn_fwd", r"attn_fwd_kernel"),
    ("attn_bwd_dkdv", r"attn_bwd_dkdv8_kernel"),
    ("attn_bwd_dq", r"attn_bwd_dq_kernel"),
    ("gemm", r"Cijk"),
    ("adamw", r"adamw"),
    ("swiglu", r"swiglu"),
    ("rmsnorm", r"rmsnorm"),
]
KEYS = (("mfma_busy_pct", "mfma_util"), ("bf16_tflops", "mfma_bf16_tflops"),
        ("hbm_read_gbps", "hbm_read_gbps"), ("hbm_write_gbps", "hbm_write_gbps"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--dispatches", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from dynolog_amd import agent as dagent
    dagent.preinit([0], kernel_trace=True, dispatch_counters=True)
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
    # statistical: NNLS de-mix of the 1 kHz samples over a kernel trace
    with dagent.KernelTrace() as kt:
        for _ in range(a.steps):
            step()
    ag.pack_pending()
    ag.step()
    torch.cuda.synchronize()
    ag.flush()
    demix = kt.counters(top=60)

    # exact: dispatch counting of each family, one family per step
    exact = {}
    for fam, regex in FAMILIES:
        dc = dagent.DispatchCounters(kernel_regex=regex, dispatches=a.dispatches).start()
        step()
        torch.cuda.synchronize()
        exact[fam] = dc.finish(timeout_s=30)
    ag.stop()

    rows = []
    for fam, regex in FAMILIES:
        rx = re.compile(regex)
        ks = [k for k in demix["kernels"] if rx.search(k["name"])]
        t = sum(k["kernel_ms"] for k in ks)
        est = {ours: (sum(k["counters"][ours] * k["kernel_ms"] for k in ks) / t if t else None)
               for ours, _ in KEYS}
        ex = exact[fam]
        us = sum(dd["duration_us"] for dd in ex.get("dispatches", []))
        tru = {ours: (sum(dd["derived"][theirs] * dd["duration_us"] for dd in ex["dispatches"]) / us if us else None)
               for ours, theirs in KEYS}
        rows.append({"family": fam, "demix_kernel_ms": round(t, 2), "demix_classes": len(ks),
                     "demix_resolved": all(k["resolved"] for k in ks) if ks else None,
                     "exact_dispatches": ex.get("counted", 0), "exact_avg_us": round(us / max(ex.get("counted", 0), 1), 1),
                     "demix": {k: (round(v, 1) if v is not None else None) for k, v in est.items()},
                     "exact": {k: (round(v, 1) if v is not None else None) for k, v in tru.items()}})
    print(f"{'family':14s} {'n':>3s} {'us':>7s} | {'MFMA% est/exact':>16s} | {'TF/s est/exact':>15s} | "
          f"{'rdGB/s est/exact':>17s} | {'wrGB/s est/exact':>17s}")
    for r in rows:
        e, t = r["demix"], r["exact"]
        f = lambda k: f"{e[k] if e[k] is not None else '-':>7} / {t[k] if t[k] is not None else '-':<7}"
        print(f"{r['family']:14s} {r['exact_dispatches']:3d} {r['exact_avg_us']:7.1f} | {f('mfma_busy_pct'):>16s} | "
              f"{f('bf16_tflops'):>15s} | {f('hbm_read_gbps'):>17s} | {f('hbm_write_gbps'):>17s}")
    res = {"model": a.model, "demix_r2": demix.get("r2"), "demix_samples": demix.get("samples"), "rows": rows}
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
