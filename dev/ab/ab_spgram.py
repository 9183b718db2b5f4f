"""spgramcf estimate_psd kernel time, nfft = 1024 on 2^26 samples (dev A/B
tool; the library comes from LQ_LIB_PATH as in dev/ab/ab.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
n = 1 << 26
x = W.cbuf(n)
psd = torch.empty(1024, device="cuda")
sg = W.LQ.Spgram(1024, default=True)
L.spgramcf_set_stream(sg.q, W.S)
ms = W.timed(lambda: L.spgramcf_estimate_psd_dev(sg.q, x.data_ptr(), n, psd.data_ptr()), it=10, w=3)
print(os.environ.get("LQ_LIB_PATH", "default"), round(ms, 4), "ms", round(8 * n / (ms * 1e-3) / 8e12, 3))
