"""Probe: hipBLASLt throughput of the input-gradient (dgrad) GEMMs of the
Llama-3-8B step, dX = dY W, with W [out, in] as stored (N-contiguous B
operand) vs a transposed copy W^T [in, out] (K-contiguous), plus the cost of
making that copy with ops.transpose2d.  Forward x W^T for reference."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dynolog_amd import ops  # noqa: E402


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


T = 8192
out = {}
for name, N, K in [("w13", 28672, 4096), ("w2", 4096, 14336), ("qkv", 6144, 4096), ("o", 4096, 4096),
                   ("head", 128256, 4096)]:
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    fl = 2 * T * N * K
    r = {}
    r["fwd x@W.t"] = bench(lambda: x @ w.t())
    r["dgrad dY@W"] = bench(lambda: dy @ w)
    wt = ops.transpose2d(w)
    r["dgrad dY@WT.t"] = bench(lambda: dy @ wt.t())
    r["transpose W"] = bench(lambda: ops.transpose2d(w))
    r["dgrad dY@T(W).t"] = bench(lambda: dy @ ops.transpose2d(w).t())
    res = {}
    for k, v in r.items():
        tf = None if k.startswith("transpose") else round(fl / v * 1e-9, 1)
        res[k] = {"ms": round(v, 4), "tflops": tf}
    res["transpose W"]["tbps"] = round(2 * N * K * 2 / (r["transpose W"] * 1e-3) * 1e-12, 2)
    out[name] = res
    print(name, json.dumps(res), flush=True)
    del w, dy, x, wt
    torch.cuda.empty_cache()
print(json.dumps(out))
