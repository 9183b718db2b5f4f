"""firfilt crcf / cccf h=64: the 16x16x32 matrix-core kernel against the
32x32x16 one it replaced, same process and buffers (dev tool, r05w / r05x):
normwise agreement with a float64 convolution on streamed / ragged /
non-finite inputs, then alternated timings.  LQ_FMX16=<10 workgroups per CU
+ chunks in flight> selected the 16x16 kernel in the A/B build (the tree
before commit 7f72544, which made it the product path without a switch), so
every setting below now runs the same kernel."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
rs = np.random.default_rng(5)
hr = rs.standard_normal(64).astype(np.float32)
hc = (rs.standard_normal(64) + 1j * rs.standard_normal(64)).astype(np.complex64)


def setenv(v):
    if v is None:
        os.environ.pop("LQ_FMX16", None)
    else:
        os.environ["LQ_FMX16"] = v


def mk(kind):
    q = W.LQ.FirFilt(kind, hr if kind == "crcf" else hc)
    q.set_stream(W.S)
    return q


def run(kind, v, x, calls):
    setenv(v)
    q = mk(kind)
    y = torch.empty_like(x)
    fn = L.firfilt_crcf_execute_block_dev if kind == "crcf" else L.firfilt_cccf_execute_block_dev
    o = 0
    for m in calls:
        fn(q.q, x.data_ptr() + 8 * o, m, y.data_ptr() + 8 * o)
        o += m
    torch.cuda.synchronize()
    return y


ok = True
for kind in ("crcf", "cccf"):
    h = (hr if kind == "crcf" else hc).astype(np.complex128)
    for name, n, calls in [("two calls", 3 << 20, [(3 << 19) + 2048 * 5 + 17, (3 << 19) - 2048 * 5 - 17]),
                           ("ragged", 2048 * 700 + 777, [2048 * 700 + 777]),
                           ("small", 5000, [1234, 3766])]:
        x = W.cbuf(n, seed=9)
        xn = x.view(-1, 2).cpu().numpy().astype(np.float64)
        xc = xn[:, 0] + 1j * xn[:, 1]
        ref = np.convolve(xc, h)[:n]
        for v in (None, "31", "32", "41", "42"):
            y = run(kind, v, x, calls).view(-1, 2).cpu().numpy().astype(np.float64)
            yc = y[:, 0] + 1j * y[:, 1]
            err = np.linalg.norm(yc - ref) / np.linalg.norm(ref)
            good = err < 2e-6
            ok &= bool(good)
            print("%s %-10s LQ_FMX16=%-4s nrm err %.2e %s" % (kind, name, v, err, "ok" if good else "FAIL"))
        del x
    # non-finite samples: both paths keep the exact-path outputs
    n = 1 << 22
    x = W.cbuf(n, seed=3)
    x[2 * 123457] = float("inf")
    x[2 * 3000000 + 1] = float("nan")
    ya = run(kind, None, x, [n])
    for v in ("31", "32", "41", "42"):
        yb = run(kind, v, x, [n])
        fa, fb = torch.isfinite(ya), torch.isfinite(yb)
        same = torch.equal(fa, fb)
        d = (ya[fa] - yb[fa]).abs().max().item() / ya[fa].abs().max().item()
        ok &= same and d < 1e-5
        print("%s inf/nan LQ_FMX16=%s finite mask equal %s, max rel diff %.2e" % (kind, v, same, d))
    del x, ya, yb
sys.stdout.flush()
setenv(None)
if not ok:
    sys.exit(1)

for kind, n in (("crcf", 1 << 28), ("cccf", 1 << 27)):
    fn = L.firfilt_crcf_execute_block_dev if kind == "crcf" else L.firfilt_cccf_execute_block_dev
    for pair in range(2):
        x = W.cbuf(n, seed=pair + 1)
        y = torch.empty_like(x)
        res = {}
        for rep in range(3):
            for v in ((None, "31", "32", "41", "42", "51") if kind == "crcf" else (None, "31", "32")):
                setenv(v)
                q = mk(kind)
                res.setdefault(v, []).append(W.timed(lambda: fn(q.q, x.data_ptr(), n, y.data_ptr()), it=20, w=10))
        print("%s 2^%d pair %d: " % (kind, n.bit_length() - 1, pair) +
              "  ".join("%s %s" % (v or "shipped", " ".join("%.4f" % t for t in ts)) for v, ts in res.items()))
        sys.stdout.flush()
        del x, y
setenv(None)
