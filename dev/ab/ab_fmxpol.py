"""firfilt crcf h=64, 2^28 samples: cache-policy bits of the 16x16 kernel's
chunk loads / output stores (LQ_FMX_POL = load aux + 4 x store aux, A/B
build, r05zk; the product build has no switch), alternated in one process on
two buffer pairs (dev tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
h = np.random.default_rng(1).standard_normal(64).astype(np.float32)
n = 1 << 28
VS = ("0", "2", "3", "8", "10")
for pair in range(2):
    x = W.cbuf(n, seed=pair + 1)
    y = torch.empty_like(x)
    ref = None
    res = {}
    for rep in range(3):
        for v in VS:
            os.environ["LQ_FMX_POL"] = v
            q = W.LQ.FirFilt("crcf", h)
            q.set_stream(W.S)
            res.setdefault(v, []).append(
                W.timed(lambda: L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr()), it=20, w=10))
            if rep == 0:
                if ref is None:
                    ref = y.clone()
                elif not torch.equal(ref, y):
                    print("MISMATCH", v)
    print("pair %d: " % pair + "  ".join("pol %s %s" % (v, " ".join("%.4f" % t for t in ts)) for v, ts in res.items()))
    sys.stdout.flush()
    del x, y, ref
os.environ.pop("LQ_FMX_POL", None)
