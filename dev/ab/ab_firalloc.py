"""firfilt_crcf h=64 on 2^28 samples with several freshly allocated buffer
pairs in one process (dev tool): does the kernel time depend on where the
buffers land?"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
n = 1 << 28
h = (torch.rand(64) - 0.5).numpy()
q = W.LQ.FirFilt("crcf", h)
q.set_stream(W.S)
keep = []
for i in range(5):
    x = W.cbuf(n, seed=i + 1)
    y = torch.empty_like(x)
    ms = W.timed(lambda: L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr()), it=20, w=10)
    print("pair %d x %#x y %#x: %.4f ms" % (i, x.data_ptr(), y.data_ptr(), ms))
    sys.stdout.flush()
    keep.append((x, y))
    if len(keep) > 2:
        keep.pop(0)
