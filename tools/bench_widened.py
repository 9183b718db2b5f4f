"""Throughput of the widened rows (SURVEY §8 a3-a11 variants and §8f), device
resident, against the HBM roofline (dev tool; the headline is bench.py).

One JSON object per workload: kernel time per call from HIP events on the
objects' stream (20 warm-up + 30 timed calls), samples/s and algorithmic
GB/s (bytes stated per workload) as a fraction of the 8 TB/s spec.
    python tools/bench_widened.py > gpurun_out/widened.json
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
import liquidmi as LQ  # noqa: E402

PEAK = 8000.0
STREAM = torch.cuda.Stream()
S = STREAM.cuda_stream


def timed(fn, it=30, w=20, floor_ms=150.0):
    """w warm-up calls, then more until floor_ms of wall time (clock ramp, as
    bench.py), then `it` timed calls"""
    import time
    t0 = time.perf_counter()
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    while (time.perf_counter() - t0) * 1e3 < floor_ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(STREAM)
    for _ in range(it):
        fn()
    e1.record(STREAM)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def cbuf(n, seed=1):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.rand(2 * n, generator=g, device="cuda") - 0.5


def rbuf(n, seed=1):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.rand(n, generator=g, device="cuda") - 0.5


def report(name, ms, units, unit_name, nbytes, note):
    gbps = nbytes / (ms * 1e-3) / 1e9
    print(json.dumps({"workload": name, "ms": round(ms, 4), "value": units / (ms * 1e-3) / 1e6,
                      "unit": "M %s/s" % unit_name, "achieved_GBps": round(gbps, 1),
                      "frac_of_8TBps": round(gbps / PEAK, 3), "bytes": note}))
    sys.stdout.flush()


def main():
    L = LQ.lib()
    # firfilt rrrf / cccf, h = 64
    n = 1 << 27
    for t, esz in (("rrrf", 4), ("cccf", 8)):
        x = rbuf(n) if t == "rrrf" else cbuf(n)
        y = torch.empty_like(x)
        h = torch.rand(64 * (2 if t == "cccf" else 1)).numpy() - 0.5
        h = h.view("complex64") if t == "cccf" else h.astype("float32")
        q = LQ.FirFilt(t, h)
        q.set_stream(S)
        fn = getattr(L, "firfilt_%s_execute_block_dev" % t)
        ms = timed(lambda: fn(q.q, x.data_ptr(), n, y.data_ptr()))
        report("firfilt_%s h=64" % t, ms, n, "samples", 2 * esz * n, "%d B/sample" % (2 * esz))
        q.destroy()
    # firfilt crcf at other lengths (h <= 32 and h > 64: the VALU kernel)
    n = 1 << 27
    x = cbuf(n)
    y = torch.empty_like(x)
    for hl in (16, 32, 48, 128, 256):
        h = (torch.rand(hl) - 0.5).numpy().astype("float32")
        q = LQ.FirFilt("crcf", h)
        q.set_stream(S)
        ms = timed(lambda: L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr()))
        report("firfilt_crcf h=%d" % hl, ms, n, "samples", 16 * n, "16 B/sample")
        q.destroy()
    del x, y
    # firdecim / firinterp crcf M = 8, m = 8 (Kaiser, 2Mm taps)
    n = 1 << 27
    x = cbuf(n)
    y = torch.empty(2 * n, device="cuda")
    d = LQ.FirDecim(8, m=8, As=60.0)
    d.set_stream(S)
    ms = timed(lambda: L.firdecim_crcf_execute_block_dev(d.q, x.data_ptr(), n // 8, y.data_ptr()))
    report("firdecim_crcf M=8 m=8", ms, n, "input samples", 8 * n + n, "8 B/input + 8 B/output")
    xi = cbuf(n // 8)
    it = LQ.FirInterp(8, m=8, As=60.0)
    it.set_stream(S)
    ms = timed(lambda: L.firinterp_crcf_execute_block_dev(it.q, xi.data_ptr(), n // 8, y.data_ptr()))
    report("firinterp_crcf M=8 m=8", ms, n, "output samples", 8 * n + n, "8 B/output + 8 B/input")
    # firpfbch2 analyzer at other channel counts (M = 1024 is the bench's
    # fused fast path; the others take the generic polyphase + transform kernels)
    n = 1 << 27
    x = cbuf(n)
    y = torch.empty(4 * n, device="cuda")
    for M in (64, 128, 256, 512, 1024, 2048, 4096):
        a2 = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, 4, 60.0)
        a2.set_stream(S)
        nb = n // (M // 2)
        ms = timed(lambda: L.firpfbch2_crcf_execute_block_dev(a2.q, x.data_ptr(), nb, y.data_ptr()))
        report("firpfbch2_crcf analyzer M=%d m=4" % M, ms, n, "input samples", 24 * n,
               "8 B/input + 16 B/output (2 per input)")
        a2.destroy()
    del x, y
    # firpfbch2 synthesizer, firpfbch analyzer / synthesizer, M = 1024
    M, nb = 1024, 1 << 17
    X = cbuf(nb * M)
    Y = torch.empty(2 * nb * M, device="cuda")
    q2 = LQ.FirPfbch2(LQ.LIQUID_SYNTHESIZER, M, 4, 60.0)
    q2.set_stream(S)
    ms = timed(lambda: L.firpfbch2_crcf_execute_block_dev(q2.q, X.data_ptr(), nb, Y.data_ptr()))
    report("firpfbch2_crcf synthesizer M=1024 m=4", ms, nb * M // 2, "output samples", 12 * nb * M,
           "8 B/channel sample in + 8 B/output (M/2 per block)")
    for typ, nm in ((LQ.LIQUID_ANALYZER, "analyzer"), (LQ.LIQUID_SYNTHESIZER, "synthesizer")):
        for Mc in (64, 256, 1024, 4096):
            nbc = nb * M // Mc
            p = LQ.FirPfbch(typ, Mc, m=4, As=60.0)
            p.set_stream(S)
            ms = timed(lambda: L.firpfbch_crcf_execute_block_dev(p.q, X.data_ptr(), nbc, Y.data_ptr()))
            report("firpfbch_crcf %s M=%d m=4" % (nm, Mc), ms, nbc * Mc, "samples", 16 * nbc * Mc, "16 B/sample")
            p.destroy()
    for Mc in (256, 4096):
        nbc = nb * M // Mc
        q2 = LQ.FirPfbch2(LQ.LIQUID_SYNTHESIZER, Mc, 4, 60.0)
        q2.set_stream(S)
        ms = timed(lambda: L.firpfbch2_crcf_execute_block_dev(q2.q, X.data_ptr(), nbc, Y.data_ptr()))
        report("firpfbch2_crcf synthesizer M=%d m=4" % Mc, ms, nbc * Mc // 2, "output samples", 12 * nbc * Mc,
               "8 B/channel sample in + 8 B/output (M/2 per block)")
        q2.destroy()
    # resamp timing plans (host/resamp.c): wall clock per call including the
    # host's plan work -- a periodic rate (plan built once, then cached), a
    # rate whose float32 timing has no period <= 2^25 inputs (a direct plan of
    # the call's inputs built serially on the host per call), and a
    # symsync-style loop that steers the rate before every 4096-input call
    import time
    n = 1 << 24
    x = cbuf(n)
    y = torch.empty(2 * 2 * n, device="cuda")
    # (float32 timing periods at npfb = 64: r = 1.037 1 011 163 inputs,
    # r = 0.9999999 8 388 609; every rate tried has a period below 2^24)
    for name, rate in (("r=1.037", 1.037), ("r=0.9999999", 0.9999999)):
        rs = LQ.Resamp(rate, 7, 0.4, 60.0, 64)
        rs.set_stream(S)
        t0 = time.perf_counter()
        rs.execute_block_dev(x.data_ptr(), n, y.data_ptr())   # first call: period search + plan build
        rs.synchronize()
        print(json.dumps({"workload": "resamp_crcf %s m=7, first 2^24-input call (host period search + plan)" % name,
                          "ms": round((time.perf_counter() - t0) * 1e3, 2)}))
        t0 = time.perf_counter()
        for _ in range(4):
            rs.execute_block_dev(x.data_ptr(), n, y.data_ptr())
        rs.synchronize()
        dt = (time.perf_counter() - t0) / 4
        print(json.dumps({"workload": "resamp_crcf %s m=7, later 2^24-input calls (plan cached), wall clock" % name,
                          "ms": round(dt * 1e3, 3), "value": n / dt / 1e6, "unit": "M input samples/s"}))
        rs.destroy()
    rs = LQ.Resamp(1.037, 7, 0.4, 60.0, 64)
    rs.set_stream(S)
    nc, calls = 4096, 200
    t0 = time.perf_counter()
    for i in range(calls):
        rs.set_rate(1.037 + (1e-6 if i & 1 else -1e-6))   # (adjust_rate clips the rate to 0.5, resamp.c:222-239)
        rs.execute_block_dev(x.data_ptr(), nc, y.data_ptr())
    rs.synchronize()
    dt = (time.perf_counter() - t0) / calls
    print(json.dumps({"workload": "resamp_crcf set_rate before every 4096-input call (direct plan per call)",
                      "ms": round(dt * 1e3, 4), "value": nc / dt / 1e6, "unit": "M input samples/s"}))
    rs.destroy()
    del x, y
    # resamp away from config 5: r = 0.3 (k_resamp4's 1/4 < r <= 1/2 class since
    # r05zj), r = 3.7 and 60 (its r > 2 class since r05ze / r05zi);
    # device-resident calls on a cached periodic plan, kernel time from HIP events
    for rate, nin in ((0.3, 1 << 24), (3.7, 1 << 22), (60.0, 1 << 18)):
        rs = LQ.Resamp(rate, 7, 0.4, 60.0, 64)
        rs.set_stream(S)
        x = cbuf(nin)
        nout = rs.num_output(nin)
        y = torch.empty(2 * (nout + 64), device="cuda")
        ms = timed(lambda: rs.execute_block_dev(x.data_ptr(), nin, y.data_ptr()))
        kern = "k_resamp4" if rate > 0.25 else "k_resamp3"
        report("resamp_crcf r=%g m=7 (%s)" % (rate, kern), ms, nout,
               "output samples", 8 * nin + 8 * nout, "8 B/input + 8 B/output")
        rs.destroy()
    del x, y
    # resamp2 decim / interp (m = 12), msresamp r = 0.3 / 3.3
    n = 1 << 26
    x = cbuf(n)
    y = torch.empty(2 * 4 * n, device="cuda")
    r2 = LQ.Resamp2(12, 0.0, 60.0)
    r2.set_stream(S)
    ms = timed(lambda: L.resamp2_crcf_execute_block_dev(r2.q, LQ.RESAMP2_DECIM, x.data_ptr(), n // 2,
                                                         y.data_ptr(), None))
    report("resamp2_crcf decim m=12", ms, n, "input samples", 8 * n + 4 * n, "8 B/input + 8 B/output")
    ms = timed(lambda: L.resamp2_crcf_execute_block_dev(r2.q, LQ.RESAMP2_INTERP, x.data_ptr(), n,
                                                         y.data_ptr(), None))
    report("resamp2_crcf interp m=12", ms, n, "input samples", 8 * n + 16 * n, "8 B/input + 16 B/output")
    for rate in (0.3, 3.3):
        ms_ = LQ.MsResamp(rate, 60.0)
        ms_.set_stream(S)
        nin = n if rate < 1 else n // 4
        nout = ms_.num_output(nin)
        ms = timed(lambda: ms_.execute_block_dev(x.data_ptr(), nin, y.data_ptr()))
        report("msresamp_crcf r=%g" % rate, ms, nin, "input samples", 8 * nin + 8 * nout,
               "8 B/input + 8 B/output")
        ms_.destroy()
    # FFT API batches
    for N in (256, 512, 1024, 2048, 4096, 8192, 16384, 65536, 12345):
        B = (1 << 26) // N
        Z = cbuf(B * N)
        pl = L.fft_create_plan(N, None, None, 1, 0)
        L.fft_set_stream(pl, S)
        ms = timed(lambda: L.fft_execute_batch_dev(pl, Z.data_ptr(), Z.data_ptr(), B))
        report("fft n=%d batch %d" % (N, B), ms, B * N, "points", 16 * B * N, "16 B/point (one pass)")
        L.fft_destroy_plan(pl)
    # spgram estimate, nfft = 1024 (window 512, transforms every 256 samples)
    n = 1 << 26
    x = cbuf(n)
    psd = torch.empty(1024, device="cuda")
    sg = LQ.Spgram(1024, default=True)
    L.spgramcf_set_stream(sg.q, S)
    ms = timed(lambda: L.spgramcf_estimate_psd_dev(sg.q, x.data_ptr(), n, psd.data_ptr()), it=5, w=2)
    report("spgramcf estimate_psd nfft=1024", ms, n, "input samples", 8 * n, "8 B/input (transform batch "
           "staged through HBM: +32 B/input)")


if __name__ == "__main__":
    main()
