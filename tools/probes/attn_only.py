"""Run only the CDNA4 attention kernels (Llama-3-8B shape) N times, for rocprofv3 PMC passes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dynolog_amd import ops

mode = sys.argv[1] if len(sys.argv) > 1 else "fwd"
B, H, KV, S, D = 2, 32, 8, 4096, 128
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, KV, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, KV, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
go = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
for _ in range(10):
    if mode == "fwd":
        with torch.no_grad():
            ops.attention(q, k, v)
    else:
        ops.attention(q, k, v).backward(go)
torch.cuda.synchronize()
print("done", mode)
