"""Probe: can hipBLASLt do better than its default solution on the one GEMM of
the step that runs on a 256 x 192 tile (the QKV weight gradient, dW [6144, 4096]
= dQKV^T X over 8192 tokens, both operands token-contiguous)?  PyTorch's
TunableOp times every hipBLASLt/rocBLAS solution for that shape only."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.cuda.tunable as tn


def bench(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


T = 8192
out = {}
for name, N, K in [("qkv_wgrad", 6144, 4096), ("o_wgrad", 4096, 4096)]:
    dyt = torch.randn(N, T, device="cuda", dtype=torch.bfloat16)
    xt = torch.randn(K, T, device="cuda", dtype=torch.bfloat16)
    fl = 2 * T * N * K
    f = lambda: dyt @ xt.t()
    tn.enable(False)
    default_ms = bench(f)
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_filename(f"/tmp/tunableop_{name}.csv")
    tn.set_max_tuning_duration(3000)
    t0 = time.perf_counter()
    f()
    torch.cuda.synchronize()
    tune_s = time.perf_counter() - t0
    tn.tuning_enable(False)
    tuned_ms = bench(f)
    res = tn.get_results()
    tn.enable(False)
    out[name] = {"default_ms": round(default_ms, 4), "default_TFLOPs": round(fl / default_ms * 1e-9, 1),
                 "tuned_ms": round(tuned_ms, 4), "tuned_TFLOPs": round(fl / tuned_ms * 1e-9, 1),
                 "tuning_s": round(tune_s, 1), "results": [list(map(str, r)) for r in res][-3:]}
    print(name, json.dumps(out[name]), flush=True)
print(json.dumps(out))
