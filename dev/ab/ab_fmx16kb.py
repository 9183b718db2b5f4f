"""firfilt crcf with 65..256 taps: 16x16x32 tiles (LQ_FMX16KB=<workgroups per
CU>) against the 32x32x16 kernel, same process and buffers (dev tool):
normwise agreement with a float64 convolution on streamed / ragged inputs and
matching Inf/NaN masks, then alternated timings on 2^27 samples.  The LQ_FMX16KB switch lived
only in the A/B build (the working tree before the commit that made the
16x16 kernel the product path); the product build has no switch."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
rs = np.random.default_rng(6)


def setenv(v):
    if v is None:
        os.environ.pop("LQ_FMX16KB", None)
    else:
        os.environ["LQ_FMX16KB"] = v


def run(h, v, x, calls):
    setenv(v)
    q = W.LQ.FirFilt("crcf", h)
    q.set_stream(W.S)
    y = torch.empty_like(x)
    o = 0
    for m in calls:
        L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr() + 8 * o, m, y.data_ptr() + 8 * o)
        o += m
    torch.cuda.synchronize()
    return y


ok = True
VS = (None, "3", "4")
for hl in (65, 128, 129, 192, 256):
    h = rs.standard_normal(hl).astype(np.float32)
    for name, n, calls in [("two calls", 3 << 20, [(3 << 19) + 2048 * 5 + 17, (3 << 19) - 2048 * 5 - 17]),
                           ("small", 5000, [1234, 3766])]:
        x = W.cbuf(n, seed=hl)
        xn = x.view(-1, 2).cpu().numpy().astype(np.float64)
        ref = np.convolve(xn[:, 0] + 1j * xn[:, 1], h.astype(np.float64))[:n]
        for v in VS:
            y = run(h, v, x, calls).view(-1, 2).cpu().numpy().astype(np.float64)
            err = np.linalg.norm(y[:, 0] + 1j * y[:, 1] - ref) / np.linalg.norm(ref)
            good = err < 2e-6
            ok &= bool(good)
            print("h=%d %-9s LQ_FMX16KB=%-4s nrm err %.2e %s" % (hl, name, v, err, "ok" if good else "FAIL"))
        del x
    n = 1 << 22
    x = W.cbuf(n, seed=3)
    x[2 * 123457] = float("inf")
    x[2 * 3000000 + 1] = float("nan")
    ya = run(h, None, x, [n])
    for v in VS[1:]:
        yb = run(h, v, x, [n])
        fa, fb = torch.isfinite(ya), torch.isfinite(yb)
        same = torch.equal(fa, fb)
        d = (ya[fa] - yb[fa]).abs().max().item() / ya[fa].abs().max().item()
        ok &= same and d < 1e-5
        print("h=%d inf/nan LQ_FMX16KB=%s finite mask equal %s, max rel diff %.2e" % (hl, v, same, d))
    del x, ya, yb
sys.stdout.flush()
setenv(None)
if not ok:
    sys.exit(1)

n = 1 << 27
x = W.cbuf(n, seed=1)
y = torch.empty_like(x)
for hl in (128, 192, 256):
    h = rs.standard_normal(hl).astype(np.float32)
    res = {}
    for rep in range(3):
        for v in VS:
            setenv(v)
            q = W.LQ.FirFilt("crcf", h)
            q.set_stream(W.S)
            res.setdefault(v, []).append(
                W.timed(lambda: L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr()), it=20, w=10))
    print("h=%d 2^27: " % hl + "  ".join("%s %s" % (v or "32x32", " ".join("%.4f" % t for t in ts))
                                        for v, ts in res.items()))
    sys.stdout.flush()
setenv(None)
