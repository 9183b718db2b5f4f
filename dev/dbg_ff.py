"""fftfilt mismatch map against the oracle for the library named by LQ_LIB_PATH (dev tool)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "liquid-dsp_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import liquidmi as LQ
import oracle_lib as O
T = {"rrrf": O.RRRF, "crcf": O.CRCF, "cccf": O.CCCF}
for t in ("rrrf", "crcf"):
    for hlen, n, nb in ((512, 2048, 12), (512, 1 << 16, 3)):
        r = np.random.default_rng(hlen)
        h = r.uniform(-0.5, 0.5, hlen).astype(np.float32)
        x = r.uniform(-0.5, 0.5, n * nb).astype(np.float32)
        if t != "rrrf":
            x = (x + 1j * r.uniform(-0.5, 0.5, n * nb)).astype(np.complex64)
        g, o = LQ.FftFilt(h, n, t=t), O.FftFilt(T[t], h, n)
        y = np.concatenate([g.execute(x[b * n:(b + 1) * n]) for b in range(nb)])
        ref = o.execute_stream(x)
        e = np.abs(y - ref) / np.max(np.abs(ref))
        bad = np.nonzero(e > 1e-5)[0]
        print(t, hlen, n, "maxerr %.3g" % e.max(), "nbad", len(bad), "first", bad[:8], "per-call", [int(np.sum((bad >= b * n) & (bad < (b + 1) * n))) for b in range(nb)][:12], flush=True)
