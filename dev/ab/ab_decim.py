"""firdecim M = 8, m = 8: the persistent prefetching phase-layout kernel
(LQ_DECIM_PF=1, k_firdecim_pf) against the one-shot k_firdecim_ph2, same
process and buffers (dev tool): bitwise equality on streamed / ragged inputs
for rrrf / crcf / cccf, then alternated timings on 2^27 crcf inputs.  The
LQ_DECIM_PF switch lived only in the A/B build (r05zf); the product build
runs k_firdecim_pf whenever x is 16-byte aligned."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()


def setenv(v):
    if v:
        os.environ["LQ_DECIM_PF"] = "1"
    else:
        os.environ.pop("LQ_DECIM_PF", None)


def run(t, M, v, x, calls, es):
    setenv(v)
    d = W.LQ.FirDecim(M, m=8, As=60.0, t=t)
    d.set_stream(W.S)
    fn = getattr(L, "firdecim_%s_execute_block_dev" % t)
    y = torch.empty(x.numel() // M + 64, device="cuda")
    o = 0
    for m in calls:   # m outputs per call
        fn(d.q, x.data_ptr() + es * o * M, m, y.data_ptr() + es * o)
        o += m
    torch.cuda.synchronize()
    return y[: (o * es) // 4].clone()


ok = True
for t, es in (("rrrf", 4), ("crcf", 8), ("cccf", 8)):
    for M in (2, 8, 16):
        for calls in ([100_000, 3, 1, 77_777, 512 * 40 + 5], [7]):
            n = sum(calls) * M
            x = W.rbuf(n * es // 4, seed=M)
            a = run(t, M, False, x, calls, es)
            b = run(t, M, True, x, calls, es)
            same = torch.equal(a.view(torch.int32), b.view(torch.int32))
            ok &= same
            print("%s M=%d calls %s bitwise %s" % (t, M, calls[:2], same))
sys.stdout.flush()
setenv(False)
if not ok:
    sys.exit(1)
n = 1 << 27
x = W.cbuf(n)
y = torch.empty(2 * n // 8 + 64, device="cuda")
res = {}
for rep in range(3):
    for v in (False, True):
        setenv(v)
        d = W.LQ.FirDecim(8, m=8, As=60.0)
        d.set_stream(W.S)
        res.setdefault(v, []).append(
            W.timed(lambda: L.firdecim_crcf_execute_block_dev(d.q, x.data_ptr(), n // 8, y.data_ptr())))
print("crcf M=8 m=8 2^27 in: ph2 %s  pf %s" % (" ".join("%.4f" % t for t in res[False]),
                                               " ".join("%.4f" % t for t in res[True])))
setenv(False)
