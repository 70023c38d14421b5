"""Probe: does HBM-bound work (the fused AdamW kernel) overlap with
compute-bound GEMMs when they run on two streams?  If it does, the
optimizer step of layer l could run while the next step's forward already
computes layer l-1 (per-layer events), hiding most of its ~19 ms.

    python tools/probes/overlap_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dynolog_amd.ops.optim import FusedAdamW  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def main():
    dev = "cuda"
    x = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.randn(28672, 4096, device=dev, dtype=torch.bfloat16) * 0.02
    params = [torch.nn.Parameter(torch.randn(4096, 14336, device=dev, dtype=torch.bfloat16) * 0.02)
              for _ in range(16)]  # ~0.94 G params, ~1/8 of Llama-3-8B
    for p in params:
        p.grad = torch.randn_like(p) * 1e-3
    opt = FusedAdamW(params, lr=1e-5)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    n_gemm = 12

    def gemms():
        for _ in range(n_gemm):
            torch.matmul(x, w.t())

    def adam():
        opt.step()

    def both():
        with torch.cuda.stream(s1):
            gemms()
        with torch.cuda.stream(s2):
            adam()

    def both_low():  # optimizer on a low-priority stream
        with torch.cuda.stream(s1):
            gemms()
        with torch.cuda.stream(s_low):
            adam()

    s_low = torch.cuda.Stream(priority=0)
    s_hi = torch.cuda.Stream(priority=-1)

    def both_hi_gemm():
        with torch.cuda.stream(s_hi):
            gemms()
        with torch.cuda.stream(s2):
            adam()

    r = {"gemm_ms": timed(gemms), "adam_ms": timed(adam)}
    r["sum_ms"] = r["gemm_ms"] + r["adam_ms"]
    r["both_two_streams_ms"] = timed(both)
    r["both_low_prio_adam_ms"] = timed(both_low)
    r["both_high_prio_gemm_ms"] = timed(both_hi_gemm)
    r["hidden_pct_of_adam"] = round(100 * (r["sum_ms"] - r["both_two_streams_ms"]) / r["adam_ms"], 1)
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in r.items()}))


if __name__ == "__main__":
    main()
