"""spgramcf estimate_psd nfft = 1024, window 512, 2^26 inputs: the fused kernel
with the zero half of each window neither loaded nor weighted (HALF) against
the full form (LQ_SPG_FULL=1 in the A/B build, r05zr; the product build
has no switch), same process (dev tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
n = 1 << 26
x = W.cbuf(n)
out = {}
res = {}
for rep in range(3):
    for v in (False, True):
        if v:
            os.environ["LQ_SPG_FULL"] = "1"
        else:
            os.environ.pop("LQ_SPG_FULL", None)
        psd = torch.empty(1024, device="cuda")
        sg = W.LQ.Spgram(1024, default=True)
        L.spgramcf_set_stream(sg.q, W.S)
        res.setdefault(v, []).append(W.timed(lambda: L.spgramcf_estimate_psd_dev(sg.q, x.data_ptr(), n, psd.data_ptr()),
                                             it=5, w=2))
        out[v] = psd.cpu().numpy().copy()
os.environ.pop("LQ_SPG_FULL", None)
print("half %s  full %s  max |diff| dB %.3g" % (" ".join("%.4f" % t for t in res[False]),
                                                 " ".join("%.4f" % t for t in res[True]),
                                                 float(np.max(np.abs(out[False] - out[True])))))
