"""RMSNorm kernel bandwidth at the Llama-3-8B step's shape (T 8192, D 4096):
add_rms_norm forward (reads x, delta; writes h, y) and its backward with the
residual gradient (reads dy, h, dres; writes dx), per-call time and TB/s."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from dynolog_amd import ops

T, D, IT = 8192, 4096, 50
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(T, D, device=dev, generator=g).bfloat16().requires_grad_(True)
d = torch.randn(T, D, device=dev, generator=g).bfloat16().requires_grad_(True)
w = torch.ones(D, device=dev, dtype=torch.bfloat16).requires_grad_(True)
dh = torch.randn(T, D, device=dev, generator=g).bfloat16()
dy = torch.randn(T, D, device=dev, generator=g).bfloat16()


def timed(fn):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(IT):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / IT * 1e3  # us


fwd_us = timed(lambda: ops.add_rms_norm(x, d, w, 1e-5))
h, y = ops.add_rms_norm(x, d, w, 1e-5)
bwd_total = timed(lambda: torch.autograd.grad((h, y), (x, d, w), (dh, dy), retain_graph=True))
out = {"fwd_us": round(fwd_us, 1), "fwd_TBps": round(4 * T * D * 2 / fwd_us * 1e-6, 2),
       "bwd_call_us": round(bwd_total, 1),
       "bwd_TBps_main_kernel_lower_bound": round(4 * T * D * 2 / bwd_total * 1e-6, 2)}
print(json.dumps(out))
