"""Probe: where does the tracing overhead come from?

Interleaved, pooled windows of the Llama-3-8B training step (as bench.py) in
three agent states:
  paused  - counting context stopped, no samples
  on_1hz  - counting context running (counters programmed), one sample / s
  on_rate - counting context running, sampling at --hz (default 1 kHz)
If on_1hz costs about as much as on_rate, the cost is the counters being
enabled (a device state), not the per-sample command-processor reads.

    python tools/probes/overhead_split.py --counter-set lite --rounds 8 --out x.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--counter-set", default="lite")
    ap.add_argument("--hz", type=float, default=1000.0)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=4, help="timed steps per window")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from dynolog_amd import agent as dagent
    dagent.preinit([0])
    import torch
    from dynolog_amd.models.llama import CONFIGS, build_llama, lm_loss
    from dynolog_amd.ops.optim import FusedAdamW

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = CONFIGS[a.model]
    model = build_llama(a.model, device=dev, dtype=torch.bfloat16, seed=0)
    opt = FusedAdamW(model.parameters(), lr=1e-5, betas=(0.9, 0.95), weight_decay=0.1)
    pool = []
    for _ in range(16):
        d = torch.randint(0, cfg.vocab_size, (2, 4097), device=dev)
        pool.append((d[:, :-1].contiguous(), d[:, 1:].contiguous()))
    ag = dagent.GpuAgent.start(device=0, sample_hz=a.hz, counter_set=a.counter_set, sinks=())
    n = [0]

    def step():
        x, y = pool[n[0] % len(pool)]
        n[0] += 1
        loss = lm_loss(model(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        ag.step()

    def window(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def state(s):
        if s == "paused":
            ag.pause()
        else:
            ag.resume()
            ag.set_rate(1.0 if s == "on_1hz" else a.hz)
        time.sleep(0.05)
        step()  # settle outside the window
        torch.cuda.synchronize()

    for _ in range(3):
        step()
    arms = ["paused", "on_1hz", "on_rate"]
    tot = {s: 0.0 for s in arms}
    cnt = {s: 0 for s in arms}
    per = {s: [] for s in arms}
    for r in range(a.rounds):
        order = arms[r % 3:] + arms[:r % 3]
        if r % 2:
            order = order[::-1]
        for s in order:
            state(s)
            t = window(a.steps)
            tot[s] += t
            cnt[s] += a.steps
            per[s].append(round(t / a.steps * 1e3, 3))
    st = ag.stats()
    ag.stop()
    ms = {s: tot[s] / cnt[s] * 1e3 for s in arms}
    res = {"counter_set": a.counter_set, "hz": a.hz, "raw_instances": st.get("raw_instances"),
           "sample_latency_us_avg": st.get("sample_latency_us_avg"),
           "ms_per_step": {s: round(v, 3) for s, v in ms.items()},
           "overhead_pct": {s: round((ms[s] / ms["paused"] - 1) * 100, 3) for s in arms[1:]},
           "windows_ms": per, "rounds": a.rounds, "steps_per_window": a.steps}
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
