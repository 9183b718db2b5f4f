"""firfilt_crcf kernel time at several filter lengths (dev A/B tool; the
library comes from LQ_LIB_PATH as in dev/ab/ab.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
n = 1 << 27
x = W.cbuf(n)
y = torch.empty_like(x)
out = {}
for hl in [int(v) for v in (sys.argv[1:] or ["64", "128", "192", "256"])]:
    h = (torch.rand(hl) - 0.5).numpy().astype("float32")
    q = W.LQ.FirFilt("crcf", h)
    q.set_stream(W.S)
    out[hl] = round(W.timed(lambda: L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr())), 4)
print(os.environ.get("LQ_LIB_PATH", "default"), out)
