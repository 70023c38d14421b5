"""Probe: tune the QKV weight-gradient GEMM (dW [6144, 4096] = dQKV^T X over
8192 tokens, TN) with TunableOp, write the result file, then, in this process
and with the file re-read, time the default solution vs the pinned one.

    python tools/probes/tunable_pin.py tune OUT.csv     # tune + write
    python tools/probes/tunable_pin.py check IN.csv     # fresh process: default vs pinned
"""
import json
import os
import sys
import time

import torch
import torch.cuda.tunable as tn


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(iters // 5):
            fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / (iters // 5) * 1e3)
    return min(ts), sum(ts) / len(ts)


mode, path = sys.argv[1], sys.argv[2]
T, N, K = 8192, 6144, 4096
dyt = torch.randn(N, T, device="cuda", dtype=torch.bfloat16)
xt = torch.randn(K, T, device="cuda", dtype=torch.bfloat16)
f = lambda: dyt @ xt.t()
if mode == "tune":
    tn.enable(True)
    tn.tuning_enable(True)
    tn.set_max_tuning_duration(10000)
    tn.set_max_tuning_iterations(100)
    tn.set_filename(path)
    f()
    torch.cuda.synchronize()
    # the file is written when the process exits (tuning enabled, filename set)
    print(json.dumps({"results": [list(map(str, r)) for r in tn.get_results()],
                      "validators": [list(map(str, v)) for v in tn.get_validators()]}))
else:
    tn.enable(False)
    d = bench(f)
    tn.enable(True)
    tn.tuning_enable(False)
    tn.set_filename("/tmp/tunableop_check_unused.csv")
    ok = tn.read_file(path)
    p = bench(f)
    tn.enable(False)
    d2 = bench(f)
    fl = 2 * T * N * K
    print(json.dumps({"read_ok": ok, "default_ms_min_mean": d, "pinned_ms_min_mean": p,
                      "default_again_ms_min_mean": d2,
                      "default_TFLOPs": round(fl / d[0] * 1e-9, 1), "pinned_TFLOPs": round(fl / p[0] * 1e-9, 1)}))
