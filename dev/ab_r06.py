"""Round-6 A/B timing of one workload per process (dev tool).

    python dev/ab_r06.py fftfilt 512        # fftfilt_crcf h=512, 2^26 samples
    python dev/ab_r06.py firfilt 64         # firfilt_crcf h=64, 2^28 samples
    python dev/ab_r06.py pfb2 1024          # firpfbch2 analyzer M=1024 m=4, 2^27 samples
    python dev/ab_r06.py resamp 1.037       # resamp_crcf r m=7 npfb=64, 2^25 samples
    python dev/ab_r06.py spgram 1024        # spgramcf estimate_psd, 2^26 samples

Each workload: launches until 150 ms of warm-up have passed, then three
passes of 20 timed launches (HIP events on the object's stream); prints the
best and all passes with the fraction of 8 TB/s.  Variant selection comes
from the environment (dev switches), so one process = one variant.
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
import liquidmi as LQ  # noqa: E402

ST = torch.cuda.Stream()


def timed(fn, it=20):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:
        for _ in range(4):
            fn()
        ST.synchronize()
    res = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(ST)
        for _ in range(it):
            fn()
        e1.record(ST)
        e1.synchronize()
        res.append(e0.elapsed_time(e1) / it)
    return res


def cbuf(n, seed=1):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.rand(2 * n, generator=g, device="cuda") - 0.5


def main():
    what, arg = sys.argv[1], float(sys.argv[2])
    tag = os.environ.get("AB_TAG", "")
    if what == "fftfilt":
        n = 1 << 26
        x, y = cbuf(n), torch.empty(2 * n, device="cuda")
        h = (torch.rand(int(arg)) - 0.5).numpy()
        q = LQ.FftFilt(h, max(int(arg) - 1, 1))
        q.set_stream(ST.cuda_stream)
        ms = timed(lambda: q.execute_block_dev(x.data_ptr(), n, y.data_ptr()))
        nb = 16.0 * n
    elif what == "firfilt":
        n = 1 << 28
        x, y = cbuf(n), torch.empty(2 * n, device="cuda")
        h = (torch.rand(int(arg)) - 0.5).numpy()
        q = LQ.FirFilt("crcf", h)
        q.set_stream(ST.cuda_stream)
        ms = timed(lambda: q.execute_block_dev(x.data_ptr(), n, y.data_ptr()))
        nb = 16.0 * n
    elif what in ("firfilt_rrrf", "firfilt_cccf"):   # 2^27 samples
        n = 1 << 27
        real = what.endswith("rrrf")
        x = (torch.rand(n if real else 2 * n, device="cuda") - 0.5)
        y = torch.empty_like(x)
        h = (torch.rand(int(arg) * (1 if real else 2)) - 0.5).numpy()
        if not real:
            h = (h[0::2] + 1j * h[1::2]).astype("complex64")
        q = LQ.FirFilt(what[-4:], h)
        q.set_stream(ST.cuda_stream)
        ms = timed(lambda: q.execute_block_dev(x.data_ptr(), n, y.data_ptr()))
        nb = (8.0 if real else 16.0) * n
    elif what == "pfb2":
        M, m = int(arg), 4
        n = 1 << 27
        nblk = n // (M // 2)
        x, y = cbuf(n), torch.empty(2 * nblk * M, device="cuda")
        q = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, m, 60.0)
        q.set_stream(ST.cuda_stream)
        ms = timed(lambda: q.execute_block_dev(x.data_ptr(), nblk, y.data_ptr()))
        nb = 24.0 * n
    elif what == "resamp":
        n = 1 << 25
        x, y = cbuf(n), torch.empty(2 * (int(n * arg) + 4096), device="cuda")
        q = LQ.Resamp(arg, 7, 0.25, 60.0, 64)
        q.set_stream(ST.cuda_stream)
        nout = [0]

        def step():
            nout[0] = q.execute_block_dev(x.data_ptr(), n, y.data_ptr())
        ms = timed(step)
        nb = 8.0 * n + 8.0 * nout[0]
    elif what == "fft":
        N = int(arg)
        B = (1 << 26) // N
        Z = cbuf(B * N)
        L = LQ.lib()
        pl = L.fft_create_plan(N, None, None, 1, 0)
        L.fft_set_stream(pl, ST.cuda_stream)
        ms = timed(lambda: L.fft_execute_batch_dev(pl, Z.data_ptr(), Z.data_ptr(), B))
        nb = 16.0 * B * N
    elif what == "firdecim":   # firdecim_crcf M = arg, m = 8, 2^27 inputs
        M = int(arg)
        n = 1 << 27
        x, y = cbuf(n), torch.empty(2 * (n // M), device="cuda")
        q = LQ.FirDecim(M, m=8, As=60.0)
        q.set_stream(ST.cuda_stream)
        L = LQ.lib()
        ms = timed(lambda: L.firdecim_crcf_execute_block_dev(q.q, x.data_ptr(), n // M, y.data_ptr()))
        nb = 8.0 * n + 8.0 * (n // M)
    elif what == "firinterp":   # firinterp_crcf M = arg, m = 8, 2^27 outputs
        M = int(arg)
        n = (1 << 27) // M
        x, y = cbuf(n), torch.empty(2 * n * M, device="cuda")
        q = LQ.FirInterp(M, m=8, As=60.0)
        q.set_stream(ST.cuda_stream)
        L = LQ.lib()
        ms = timed(lambda: L.firinterp_crcf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr()))
        nb = 8.0 * n + 8.0 * n * M
    elif what == "resamp2":   # resamp2_crcf m = 12, 2^26 inputs: arg 0 decim, 1 interp
        n = 1 << 26
        x, y = cbuf(n), torch.empty(2 * 2 * n, device="cuda")
        q = LQ.Resamp2(12, 0.0, 60.0)
        q.set_stream(ST.cuda_stream)
        L = LQ.lib()
        if arg == 0:
            ms = timed(lambda: L.resamp2_crcf_execute_block_dev(q.q, LQ.RESAMP2_DECIM, x.data_ptr(), n // 2,
                                                                 y.data_ptr(), None))
            nb = 12.0 * n
        else:
            ms = timed(lambda: L.resamp2_crcf_execute_block_dev(q.q, LQ.RESAMP2_INTERP, x.data_ptr(), n,
                                                                 y.data_ptr(), None))
            nb = 24.0 * n
    elif what == "msresamp":   # msresamp_crcf rate arg, 2^26 inputs (2^24 for r > 1)
        n = 1 << 26 if arg < 1 else 1 << 24
        x, y = cbuf(n), torch.empty(2 * (int(n * arg) + 4096), device="cuda")
        q = LQ.MsResamp(arg, 60.0)
        q.set_stream(ST.cuda_stream)
        nout = q.num_output(n)
        ms = timed(lambda: q.execute_block_dev(x.data_ptr(), n, y.data_ptr()))
        nb = 8.0 * n + 8.0 * nout
    elif what == "pfbsyn":   # firpfbch2 synthesizer M, m=4, 2^26 outputs
        M = int(arg)
        nout = 1 << 26
        nblk = nout // (M // 2)
        X, y = cbuf(nblk * M), torch.empty(2 * nout, device="cuda")
        q = LQ.FirPfbch2(LQ.LIQUID_SYNTHESIZER, M, 4, 60.0)
        q.set_stream(ST.cuda_stream)
        ms = timed(lambda: q.execute_block_dev(X.data_ptr(), nblk, y.data_ptr()))
        nb = 8.0 * nblk * M + 8.0 * nout
    elif what == "pfbsyn1":   # firpfbch synthesizer M, m=4, 2^27 samples
        M = int(arg)
        nblk = (1 << 27) // M
        X, y = cbuf(nblk * M), torch.empty(2 * nblk * M, device="cuda")
        q = LQ.FirPfbch(LQ.LIQUID_SYNTHESIZER, M, m=4, As=60.0)
        q.set_stream(ST.cuda_stream)
        L = LQ.lib()
        ms = timed(lambda: L.firpfbch_crcf_execute_block_dev(q.q, X.data_ptr(), nblk, y.data_ptr()))
        nb = 16.0 * nblk * M
    elif what == "pfban1":   # firpfbch analyzer M, m=4, 2^27 samples
        M = int(arg)
        nblk = (1 << 27) // M
        x, Y = cbuf(nblk * M), torch.empty(2 * nblk * M, device="cuda")
        q = LQ.FirPfbch(LQ.LIQUID_ANALYZER, M, m=4, As=60.0)
        q.set_stream(ST.cuda_stream)
        L = LQ.lib()
        ms = timed(lambda: L.firpfbch_crcf_execute_block_dev(q.q, x.data_ptr(), nblk, Y.data_ptr()))
        nb = 16.0 * nblk * M
    elif what == "spgram":   # spgramcf estimate_psd, nfft = arg (default window), 2^26 samples
        n = 1 << 26
        x, psd = cbuf(n), torch.empty(int(arg), device="cuda")
        sg = LQ.Spgram(int(arg), default=True)
        L = LQ.lib()
        L.spgramcf_set_stream(sg.q, ST.cuda_stream)
        ms = timed(lambda: L.spgramcf_estimate_psd_dev(sg.q, x.data_ptr(), n, psd.data_ptr()))
        nb = 8.0 * n
    else:
        sys.exit("unknown workload " + what)
    best = min(ms)
    print(json.dumps({"what": what, "arg": arg, "tag": tag, "best_ms": round(best, 4),
                      "frac": round(nb / (best * 1e-3) / 8e12, 4), "passes": [round(v, 4) for v in ms]}), flush=True)


if __name__ == "__main__":
    main()
