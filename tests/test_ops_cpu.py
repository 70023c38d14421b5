"""Host-side contract of dynolog_amd.ops (no GPU needed): every op refuses
non-CUDA / non-bf16 inputs loudly instead of silently falling back, and the
model keeps its plain PyTorch path for CPU tensors."""
import pytest
import torch

from dynolog_amd import ops
from dynolog_amd.models import llama


def _bf(*shape):
    return torch.zeros(*shape, dtype=torch.bfloat16)


@pytest.mark.parametrize("call", [
    lambda: ops.rms_norm(_bf(4, 8), _bf(8), 1e-5),
    lambda: ops.add_rms_norm(_bf(4, 8), _bf(4, 8), _bf(8), 1e-5),
    lambda: ops.swiglu(_bf(4, 32)),
    lambda: ops.rope_qkv(_bf(1, 4, 3 * 32), torch.zeros(4, 8), torch.zeros(4, 8), 1, 1),
    lambda: ops.cross_entropy(_bf(4, 16), torch.zeros(4, dtype=torch.long)),
    lambda: ops.attention(_bf(1, 128, 2, 128), _bf(1, 128, 1, 128), _bf(1, 128, 1, 128)),
    lambda: ops.linear(_bf(4, 8), _bf(8, 8)),
    lambda: ops.ffn(_bf(64, 64), _bf(128, 64), _bf(64, 64)),
    lambda: ops.transpose2d(_bf(8, 8)),
])
def test_ops_refuse_cpu_tensors(call):
    with pytest.raises(TypeError, match="CUDA"):
        call()


def test_model_cpu_path_is_plain_pytorch():
    torch.manual_seed(0)
    m = llama.build_llama("tiny", device="cpu", dtype=torch.float32)
    ids = torch.randint(0, m.cfg.vocab_size, (2, 17))
    loss = llama.lm_loss(m(ids[:, :-1]), ids[:, 1:])
    loss.backward()
    assert torch.isfinite(loss)
    assert all(p.grad is not None for p in m.parameters())
    assert not llama.fused_ops_enabled(ids)


def test_weight_transpose_registry_invalidation():
    """ops.cached_transpose: a W^T registered by the optimizer is served until
    the weight changes through torch (version bump), is unregistered, or is
    freed; a shape mismatch never matches (pure host logic, CPU tensors)."""
    w = torch.nn.Parameter(torch.randn(4, 6))
    wt = w.detach().t().contiguous()
    ops.register_transposed(w, wt)
    assert ops.cached_transpose(w) is wt
    assert ops.cached_transpose(w.detach()) is wt  # same storage, same version counter
    with torch.no_grad():
        w.add_(1.0)
    assert ops.cached_transpose(w) is None  # stale after an in-place torch write
    ops.register_transposed(w, wt)
    ops.unregister_transposed(w)
    assert ops.cached_transpose(w) is None
    ops.register_transposed(w, torch.empty(4, 6))  # wrong shape for w^T
    assert ops.cached_transpose(w) is None
    v = torch.nn.Parameter(torch.randn(3, 3))
    ops.register_transposed(v, v.detach().t().contiguous())
    ptr = v.data_ptr()
    del v
    assert ops._WT[ptr][0]() is None  # freed weight: its entry can no longer match
    ops.unregister_transposed(torch.empty(0))  # unknown pointer: no-op
    assert ops.dgrad_weights(llama.build_llama("tiny", device="cpu", dtype=torch.float32)) != []


def test_activation_transpose_slot_offer_take():
    """ops.offer_transposed / take_transposed: one slot, served once to a 2-D
    view of the same storage, refused after a write or for another tensor
    (and then dropped: every take empties the slot), replaced by the next offer."""
    x = torch.randn(8, 6)
    xt = x.t().contiguous()
    ops.offer_transposed(x, xt)
    assert ops.take_transposed(torch.randn(8, 6)) is None  # another tensor: the offer is stale
    assert ops._ACT_T[0] is None  # ... and dropped, never served later
    ops.offer_transposed(x, xt)
    assert ops.take_transposed(x.view(2, 4, 6).reshape(-1, 6)) is xt  # a view of it: served
    assert ops.take_transposed(x) is None  # served once
    ops.offer_transposed(x, xt)
    x.add_(1.0)
    assert ops.take_transposed(x) is None  # written since the offer
    y = torch.randn(4, 4)
    ops.offer_transposed(y, y.t().contiguous())
    assert ops._ACT_T[0][0][0] == y.data_ptr()  # one slot: the newest offer
    assert ops.take_transposed(y) is not None and ops._ACT_T[0] is None


def test_fused_adamw_state_dict_loads_into_torch_adamw():
    """FusedAdamW.state_dict() -> torch.optim.AdamW.load_state_dict() -> step():
    the step count goes out as torch stores it (a tensor), while FusedAdamW's
    own state keeps its int; and a torch state dict loads back."""
    import torch
    from dynolog_amd.ops.optim import FusedAdamW

    p = torch.nn.Parameter(torch.randn(4, 3))
    opt = FusedAdamW([p], lr=1e-2)
    st = opt.state[p]
    st["step"] = 3  # as FusedAdamW.step() leaves it
    st["exp_avg"] = torch.full_like(p, 0.1)
    st["exp_avg_sq"] = torch.full_like(p, 0.01)
    sd = opt.state_dict()
    assert torch.is_tensor(sd["state"][0]["step"]) and float(sd["state"][0]["step"]) == 3.0
    assert opt.state[p]["step"] == 3 and isinstance(opt.state[p]["step"], int)  # live state untouched
    q = torch.nn.Parameter(p.detach().clone())
    ref = torch.optim.AdamW([q], lr=1e-2)
    ref.load_state_dict(sd)
    q.grad = torch.ones_like(q)
    ref.step()  # raised 'state_steps ... singleton tensors' with an int step
    assert float(ref.state[q]["step"]) == 4.0
    back = FusedAdamW([torch.nn.Parameter(q.detach().clone())], lr=1e-2)
    back.load_state_dict(ref.state_dict())
    assert float(back.state_dict()["state"][0]["step"]) == 4.0
