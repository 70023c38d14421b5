#!/usr/bin/env python3
"""Low-noise sampling-overhead curve on fixed GPU work.

Interleaves A/B windows (agent paused vs sampling at each rate) over a
compute-bound bf16 GEMM loop and a bandwidth-bound copy loop, so clock and
thermal drift cancel.  Prints one JSON document."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynolog_amd import agent  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="250,500,1000,2000,0")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--window-s", type=float, default=2.0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    agent.preinit([0])
    import torch
    torch.cuda.set_device(0)
    ag = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=())
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    big = torch.empty(1 << 30, device="cuda", dtype=torch.uint8)  # 1 GiB
    big2 = torch.empty_like(big)

    def gemm():
        torch.mm(a, a)

    def copy():
        big2.copy_(big)

    workloads = {"gemm_bf16_8192": gemm, "copy_1GiB": copy}

    def window(fn):
        # run fn for ~window_s; return seconds per call
        torch.cuda.synchronize()
        n = 0
        t0 = time.perf_counter()
        while True:
            for _ in range(8):
                fn()
            n += 8
            torch.cuda.synchronize()
            if time.perf_counter() - t0 >= args.window_s:
                break
        return (time.perf_counter() - t0) / n

    res = {}
    for wname, fn in workloads.items():
        for _ in range(3):
            window(fn)  # warm clocks
        rows = {}
        for hz in [float(x) for x in args.rates.split(",")]:
            base, meas = [], []
            for _ in range(args.reps):
                ag.pause()
                time.sleep(0.02)
                base.append(window(fn))
                ag.set_rate(hz)
                ag.resume()
                time.sleep(0.02)
                s0 = ag.stats()["samples_taken"]
                t = time.perf_counter()
                meas.append(window(fn))
                rate = (ag.stats()["samples_taken"] - s0) / (time.perf_counter() - t)
            b, m = sum(base) / len(base), sum(meas) / len(meas)
            rows[str(hz)] = {"base_ms": round(b * 1e3, 4), "sampled_ms": round(m * 1e3, 4),
                             "overhead_pct": round((m / b - 1) * 100, 3),
                             "achieved_hz": round(rate, 1)}
            print(wname, hz, rows[str(hz)], file=sys.stderr, flush=True)
        res[wname] = rows
    st = ag.stats()
    ag.stop()
    doc = {"results": res, "sample_latency_us_avg": st["sample_latency_us_avg"]}
    print(json.dumps(doc, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
