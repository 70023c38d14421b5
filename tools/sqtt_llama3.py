"""SQTT captures of the Llama-3-8B training step's hot kernels through the
in-process agent (agent.ThreadTrace, src/gpu/ThreadTracer.h): the causal
flash-attention forward, its dK/dV backward and a hipBLASLt GEMM, one
dispatch each, while the counter agent samples at 1 kHz.

    python tools/sqtt_llama3.py --out gpurun_out/sqtt_llama

Prints, per capture, the traced kernel, the raw SQTT bytes per shader engine
and the time of the training step that contained the capture next to an
untraced step (the traced kernel runs serialised with the trace on).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--out", default="gpurun_out/sqtt_llama")
    ap.add_argument("--kernels", default="attn_fwd_kernel,attn_bwd_dkdv8_kernel,Cijk")
    a = ap.parse_args()

    from dynolog_amd import agent as dagent
    dagent.preinit([0], thread_trace=True)
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

    def step() -> float:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss = lm_loss(model(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        ag.step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for _ in range(3):
        step()
    plain = [step() for _ in range(2)]
    caps = []
    for i, regex in enumerate(k for k in a.kernels.split(",") if k):
        tt = dagent.ThreadTrace(os.path.join(a.out, f"cap{i}"), kernel_regex=regex, dispatches=1).start()
        ms = step()
        idx = tt.finish(timeout_s=30)
        ses = idx["dispatches"][0]["shader_engines"] if idx.get("dispatches") else []
        caps.append({"regex": regex, "step_ms": round(ms, 2), "traced": idx.get("traced"),
                     "kernel": (idx["dispatches"][0].get("kernel", "")[:120] if idx.get("dispatches") else ""),
                     "bytes_per_se": {str(s["shader_engine"]): s["bytes"] for s in ses},
                     "index": idx.get("index_path"), "error": idx.get("error")})
    after = [step() for _ in range(2)]
    st = ag.stats()
    ag.stop()
    res = {"model": a.model, "plain_step_ms": [round(v, 2) for v in plain + after], "captures": caps,
           "agent": {k: st.get(k) for k in ("samples_taken", "samples_failed")}}
    print(json.dumps(res, indent=1))
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    return 0 if all(c["traced"] == 1 for c in caps) else 1


if __name__ == "__main__":
    sys.exit(main())
