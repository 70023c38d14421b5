"""Feasibility probe: full-size Llama-3-8B train step (random init) on one MI355X.

Measures step time / memory for a plain PyTorch implementation so the workload
harness can be sized.  Not part of the framework.
"""
import math
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

D, L, H, KV, FF, V = 4096, 32, 32, 8, 14336, 128256
HD = D // H


class Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.n1 = nn.RMSNorm(D, eps=1e-5)
        self.qkv = nn.Linear(D, (H + 2 * KV) * HD, bias=False)
        self.o = nn.Linear(D, D, bias=False)
        self.n2 = nn.RMSNorm(D, eps=1e-5)
        self.gu = nn.Linear(D, 2 * FF, bias=False)
        self.down = nn.Linear(FF, D, bias=False)

    def forward(self, x, cos, sin):
        b, s, _ = x.shape
        h = self.n1(x)
        q, k, v = self.qkv(h).split([H * HD, KV * HD, KV * HD], dim=-1)
        q = q.view(b, s, H, HD).transpose(1, 2)
        k = k.view(b, s, KV, HD).transpose(1, 2)
        v = v.view(b, s, KV, HD).transpose(1, 2)

        def rope(t):
            t1, t2 = t[..., : HD // 2], t[..., HD // 2:]
            return torch.cat([t1 * cos - t2 * sin, t2 * cos + t1 * sin], dim=-1)

        q, k = rope(q), rope(k)
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
        x = x + self.o(a.transpose(1, 2).reshape(b, s, D))
        g, u = self.gu(self.n2(x)).chunk(2, dim=-1)
        return x + self.down(F.silu(g) * u)


class Llama(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(V, D)
        self.blocks = nn.ModuleList([Block() for _ in range(L)])
        self.norm = nn.RMSNorm(D, eps=1e-5)
        self.head = nn.Linear(D, V, bias=False)

    def forward(self, ids):
        s = ids.shape[1]
        inv = 1.0 / (500000.0 ** (torch.arange(0, HD, 2, device=ids.device).float() / HD))
        f = torch.outer(torch.arange(s, device=ids.device).float(), inv)
        cos, sin = f.cos().to(torch.bfloat16), f.sin().to(torch.bfloat16)
        x = self.emb(ids)
        for b in self.blocks:
            x = b(x, cos, sin)
        return self.head(self.norm(x))


def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    seq = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    torch.manual_seed(0)
    dev = "cuda"
    t0 = time.time()
    m = Llama().to(dev, dtype=torch.bfloat16)
    print("params", sum(p.numel() for p in m.parameters()) / 1e9, "B; build", time.time() - t0, flush=True)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-5, fused=True)
    ids = torch.randint(0, V, (bs, seq + 1), device=dev)
    for i in range(6):
        torch.cuda.synchronize()
        t = time.time()
        logits = m(ids[:, :-1])
        loss = F.cross_entropy(logits.float().view(-1, V), ids[:, 1:].reshape(-1))
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        dt = time.time() - t
        tok = bs * seq
        print(f"step {i} loss {loss.item():.3f} {dt*1e3:.1f} ms {tok/dt:.0f} tok/s "
              f"mfu~{6*8.03e9*tok/dt/2.5e15*100:.1f}% mem {torch.cuda.max_memory_allocated()/2**30:.1f} GiB",
              flush=True)


if __name__ == "__main__":
    main()
