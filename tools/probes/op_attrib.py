"""Attribute the remaining small ATen kernels of the Llama-3-8B step (copies,
fills, adds) to operators and shapes with torch.profiler."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from torch.profiler import profile, ProfilerActivity
from dynolog_amd.models.llama import build_llama, lm_loss
from dynolog_amd.ops.optim import FusedAdamW

dev = torch.device("cuda", 0)
model = build_llama("llama3-8b", device=dev)
opt = FusedAdamW(model.parameters(), lr=1e-5, betas=(0.9, 0.95), weight_decay=0.1)
data = torch.randint(0, model.cfg.vocab_size, (2, 4097), device=dev)
x, y = data[:, :-1].contiguous(), data[:, 1:].contiguous()

def step():
    loss = lm_loss(model(x), y)
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)

for _ in range(2):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
             with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=40, max_shapes_column_width=70))
# the small ATen kernels left between the fused ops, with their callers
for e in prof.key_averages(group_by_input_shape=True, group_by_stack_n=6):
    if e.key in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::to",
                 "aten::_to_copy", "aten::contiguous", "aten::clone", "aten::zeros", "aten::zeros_like"):
        print(e.key, e.count, f"{e.device_time_total/1e3:.2f}ms", e.input_shapes[:3])
        print("   ", " <- ".join(str(f) for f in (e.stack or [])[:6]))
