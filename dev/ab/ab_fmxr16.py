"""firfilt rrrf h=64: 16x16x32 tiles (LQ_FMXR16=<workgroups per CU>) against
the 32x32x16 kernel, same process and buffers (dev tool): normwise agreement
with a float64 convolution on streamed / ragged inputs, matching Inf/NaN
masks, then alternated timings on 2^27 samples.  The LQ_FMXR16 switch lived
only in the A/B build (the working tree before the commit that made the
16x16 kernel the product path); the product build has no switch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
rs = np.random.default_rng(7)
VS = (None, "3", "4")


def setenv(v):
    if v is None:
        os.environ.pop("LQ_FMXR16", None)
    else:
        os.environ["LQ_FMXR16"] = v


def run(h, v, x, calls):
    setenv(v)
    q = W.LQ.FirFilt("rrrf", h)
    q.set_stream(W.S)
    y = torch.empty_like(x)
    o = 0
    for m in calls:
        L.firfilt_rrrf_execute_block_dev(q.q, x.data_ptr() + 4 * o, m, y.data_ptr() + 4 * o)
        o += m
    torch.cuda.synchronize()
    return y


ok = True
for hl in (33, 64):
    h = rs.standard_normal(hl).astype(np.float32)
    for name, n, calls in [("two calls", 3 << 20, [(3 << 19) + 4096 * 5 + 17, (3 << 19) - 4096 * 5 - 17]),
                           ("small", 5000, [1234, 3766])]:
        x = W.rbuf(n, seed=hl)
        ref = np.convolve(x.cpu().numpy().astype(np.float64), h.astype(np.float64))[:n]
        for v in VS:
            y = run(h, v, x, calls).cpu().numpy().astype(np.float64)
            err = np.linalg.norm(y - ref) / np.linalg.norm(ref)
            good = err < 2e-6
            ok &= bool(good)
            print("h=%d %-9s LQ_FMXR16=%-4s nrm err %.2e %s" % (hl, name, v, err, "ok" if good else "FAIL"))
        del x
    n = 1 << 22
    x = W.rbuf(n, seed=3)
    x[123457] = float("inf")
    x[3000001] = float("nan")
    ya = run(h, None, x, [n])
    for v in VS[1:]:
        yb = run(h, v, x, [n])
        fa, fb = torch.isfinite(ya), torch.isfinite(yb)
        same = torch.equal(fa, fb)
        d = (ya[fa] - yb[fa]).abs().max().item() / ya[fa].abs().max().item()
        ok &= same and d < 1e-5
        print("h=%d inf/nan LQ_FMXR16=%s finite mask equal %s, max rel diff %.2e" % (hl, v, same, d))
    del x, ya, yb
sys.stdout.flush()
setenv(None)
if not ok:
    sys.exit(1)

n = 1 << 27
h = rs.standard_normal(64).astype(np.float32)
for pair in range(2):
    x = W.rbuf(n, seed=pair + 1)
    y = torch.empty_like(x)
    res = {}
    for rep in range(3):
        for v in VS:
            setenv(v)
            q = W.LQ.FirFilt("rrrf", h)
            q.set_stream(W.S)
            res.setdefault(v, []).append(
                W.timed(lambda: L.firfilt_rrrf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr()), it=20, w=10))
    print("rrrf h=64 2^27 pair %d: " % pair + "  ".join("%s %s" % (v or "32x32", " ".join("%.4f" % t for t in ts))
                                                     for v, ts in res.items()))
    sys.stdout.flush()
    del x, y
setenv(None)
