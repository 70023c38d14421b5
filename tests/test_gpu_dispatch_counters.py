"""Exact per-dispatch counters (src/gpu/DispatchCounters.h) on a real
MI355X: rocprofiler-sdk dispatch counting on the next N matching kernels of
a live process, with the same derived metrics as the 1 kHz sampler."""
import json

import pytest

from test_gpu_agent import _run

pytestmark = pytest.mark.gpu


def test_dispatch_counters_gemm_and_copy(native_built):
    res = _run("""
        from dynolog_amd import agent
        agent.preinit(dispatch_counters=True)
        import json, time, torch
        torch.cuda.set_device(0)
        a = agent.GpuAgent.start(device=0, sample_hz=1000, sinks=("memory",))
        x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        src = torch.ones(1 << 28, dtype=torch.float32, device="cuda")   # 1 GiB
        dst = torch.empty_like(src)
        y = x @ x; torch.add(src, 1.0, out=dst); torch.cuda.synchronize()
        assert agent.DispatchCounters.configured()
        dc = agent.DispatchCounters(kernel_regex="Cijk", dispatches=3).start()
        for _ in range(5):
            y = x @ x
        torch.cuda.synchronize()
        gemm = dc.finish(timeout_s=20)
        dc = agent.DispatchCounters(kernel_regex="elementwise", dispatches=2).start()
        for _ in range(3):
            torch.add(src, 1.0, out=dst)
        torch.cuda.synchronize()
        copy = dc.finish(timeout_s=20)
        prec = agent.DispatchCounters(kernel_regex="Cijk", dispatches=1, counter_set="precision").start()
        y = x @ x; torch.cuda.synchronize()
        prec = prec.finish(timeout_s=20)
        time.sleep(0.2)
        st = a.stats()
        a.stop()
        print("RESULT " + json.dumps(dict(gemm=gemm, copy=copy, prec=prec, st=st)))
    """, timeout=300)
    gemm, copy, prec, st = res["gemm"], res["copy"], res["prec"], res["st"]
    print(json.dumps(gemm["kernels"], indent=1), json.dumps(copy["kernels"], indent=1))
    assert "error" not in gemm and gemm["counted"] == 3, gemm
    g = gemm["dispatches"][0]
    flops = 2.0 * 8192 ** 3
    # the bf16 MFMA rate from the counters matches the GEMM's FLOPs over its duration
    tf_expected = flops / (g["duration_us"] * 1e-6) * 1e-12
    assert g["derived"]["mfma_bf16_tflops"] == pytest.approx(tf_expected, rel=0.1), g
    assert g["derived"]["mfma_util"] > 30 and g["derived"]["gpu_busy_pct"] > 90, g
    assert g["counters"]["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 == pytest.approx(flops, rel=0.02), g
    c = copy["dispatches"][0]
    assert copy["counted"] == 2, copy
    assert c["derived"]["mfma_util"] < 1 and c["derived"]["hbm_read_gbps"] > 1000, c
    # 1 GiB read and 1 GiB written: the TCC request counts, priced as the
    # sampler prices them, account for the bytes
    rd = c["derived"]["hbm_read_gbps"] * c["duration_us"] * 1e3
    wr = c["derived"]["hbm_write_gbps"] * c["duration_us"] * 1e3
    print("copy bytes read %.3g written %.3g" % (rd, wr))
    assert rd == pytest.approx(1 << 30, rel=0.25) and wr == pytest.approx(1 << 30, rel=0.25), c
    p = prec["dispatches"][0]["derived"]
    assert "fp32_active" in p and p["mfma_bf16_tflops"] > 100, prec
    assert st["samples_failed"] == 0
    assert st["dispatch_counting_started"] is True and st["pack_mode"] == "step", st


def test_reduced_rate_hbm_pass_matches_dispatch_counting(native_built):
    """HBM traffic read only in every fourth batch (pass plan core:3,lite:1:
    the 256 TCC instances at a quarter of the sample rate) still prices a
    steady 1 GiB copy loop: the sampled read / write GB/s of the copy phase
    agree with exact per-dispatch counting of the same kernel and account for
    the bytes the loop moved.  (Overhead matrix, profiles/round4/README.md.)"""
    res = _run("""
        from dynolog_amd import agent
        agent.preinit(dispatch_counters=True)
        import json, time, torch
        torch.cuda.set_device(0)
        src = torch.ones(1 << 28, dtype=torch.float32, device="cuda")   # 1 GiB
        dst = torch.empty_like(src)
        torch.add(src, 1.0, out=dst); torch.cuda.synchronize()
        a = agent.GpuAgent.start(device=0, sample_hz=1000, batch=8, sinks=("memory",),
                                 counter_passes="core:3,lite:1")
        n = 0
        t0 = time.perf_counter()
        with a.phase("copy"):
            while time.perf_counter() - t0 < 3.0:
                for _ in range(20):
                    torch.add(src, 1.0, out=dst)
                n += 20
                torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        a.pack_pending(); a.step(); torch.cuda.synchronize(); a.flush()
        time.sleep(0.3)
        ps = a.phase_stats(); st = a.stats()
        dc = agent.DispatchCounters(kernel_regex="elementwise", dispatches=2).start()
        for _ in range(3):
            torch.add(src, 1.0, out=dst)
        torch.cuda.synchronize()
        exact = dc.finish(timeout_s=20)
        a.stop()
        print("RESULT " + json.dumps(dict(ps=ps, st=st, exact=exact, n=n, wall=wall)))
    """, timeout=300)
    st, exact = res["st"], res["exact"]
    copy = res["ps"]["0"]["copy"]
    print(json.dumps(dict(copy=copy, exact=exact["dispatches"][0]["derived"], n=res["n"], wall=res["wall"]), indent=1))
    assert st["samples_failed"] == 0 and [p["set"] for p in st["counter_passes"]] == ["core", "lite"], st
    assert exact["counted"] == 2, exact
    ex = exact["dispatches"][0]["derived"]
    assert copy["hbm_read_gbps"] == pytest.approx(ex["hbm_read_gbps"], rel=0.15), (copy, ex)
    assert copy["hbm_write_gbps"] == pytest.approx(ex["hbm_write_gbps"], rel=0.15), (copy, ex)
    moved = (copy["hbm_read_gbps"] + copy["hbm_write_gbps"]) * 1e9 * res["wall"]
    assert moved == pytest.approx(2.0 * (1 << 30) * res["n"], rel=0.2), (moved, res["n"])
