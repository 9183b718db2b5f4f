"""msresamp_crcf r = 0.3 on 2^26 inputs: the decimating chain run in chunks of
2^LG output groups (LQ_MS_CHUNK_LG, A/B build) -- whole-call (LG 30) vs
Infinity-Cache-sized chunks (dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
n = 1 << 26
x = W.cbuf(n)
y = torch.empty(2 * n, device="cuda")
res = {}
for rep in range(3):
    for lg in ("30", "24", "23", "22", "21"):
        os.environ["LQ_MS_CHUNK_LG"] = lg
        ms_ = W.LQ.MsResamp(0.3, 60.0)
        ms_.set_stream(W.S)
        res.setdefault(lg, []).append(W.timed(lambda: ms_.execute_block_dev(x.data_ptr(), n, y.data_ptr())))
        ms_.destroy()
print("  ".join("LG %s %s" % (k, " ".join("%.4f" % t for t in v)) for k, v in res.items()))
