#!/usr/bin/env python3
"""Kernel trace of the Llama-3-8B step with the agent on the RCCL gather path
(force_collective at world 1: the path every rank takes at world > 1):
which kernels run during a step, their durations and overlaps, RCCL's
included -- to find why memory-bound trainer kernels ran up to 2x slower
while the agent gathered (profiles/round5/g05b).  Writes a Chrome trace and
prints a JSON summary."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--mode", default="fc", choices=["fc", "local", "none", "torch_ar"])
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    from dynolog_amd import agent
    agent.preinit(kernel_trace=True)
    import torch
    from dynolog_amd.models.llama import build_llama, lm_loss
    from dynolog_amd.ops.optim import FusedAdamW
    from dynolog_amd.ops import dgrad_weights
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = build_llama("llama3-8b", device=dev, dtype=torch.bfloat16, seed=0)
    opt = FusedAdamW(model.parameters(), lr=1e-5, transposed=dgrad_weights(model))
    data = torch.randint(0, model.cfg.vocab_size, (2, 4097), device=dev)
    x, y = data[:, :-1].contiguous(), data[:, 1:].contiguous()
    a = None
    small = None
    if args.mode == "torch_ar":
        # no agent: a 1-rank torch process group (RCCL) all-reducing 8 bytes per step
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29671")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        small = torch.zeros(1, dtype=torch.float64, device=dev)
    elif args.mode != "none":
        a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=("memory",), force_collective=args.mode == "fc")

    def step():
        loss = lm_loss(model(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        if a is not None:
            a.step()
        if small is not None:
            import torch.distributed as dist
            dist.all_reduce(small)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    kt = agent.KernelTrace().start()
    t0 = time.time()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = (time.time() - t0) / args.steps * 1e3
    kt.stop()
    kt.write_chrome(args.out)
    s = kt.summary(top=40)
    st = a.stats() if a is not None else {}
    if a is not None:
        a.stop()
    with open(args.out) as f:
        ev = [e for e in json.load(f)["traceEvents"] if e.get("ph") == "X"]
    long = sorted(ev, key=lambda e: -e["dur"])[:12]
    nccl = [e for e in ev if "nccl" in e["name"].lower() or "rccl" in e["name"].lower()]
    print(json.dumps({"mode": args.mode, "ms_per_step": round(wall, 2), "dispatches": s["dispatches"],
                      "gpu_busy_ms": s["gpu_busy_ms"],
                      "top": [(k["name"][:70], k["calls"], round(k["total_ms"], 3)) for k in s["top_kernels"][:15]],
                      "longest": [(e["name"][:60], round(e["dur"], 1), e["tid"]) for e in long],
                      "rccl_kernels": [(e["name"][:80], round(e["dur"], 1), e["tid"], e["args"].get("grid"),
                                        e["args"].get("block")) for e in nccl[:12]],
                      "agent": {k: st.get(k) for k in ("gather_latency_us_avg", "step_host_us_avg", "collective")}}))


if __name__ == "__main__":
    main()
