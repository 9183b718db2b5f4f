"""firpfbch2_crcf analyzer kernel time for given (M, m) on 2^27 input samples
(dev A/B tool; LQ_PFB2_TWO_PASS=1 selects the two-pass path)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
n = 1 << 27
x = W.cbuf(n)
out = {}
for arg in (sys.argv[1:] or ["4096:4"]):
    M, m = (int(v) for v in arg.split(":"))
    nb = n // (M // 2)
    y = torch.empty(2 * nb * M, device="cuda")
    a2 = W.LQ.FirPfbch2(W.LQ.LIQUID_ANALYZER, M, m, 60.0)
    a2.set_stream(W.S)
    ms = W.timed(lambda: L.firpfbch2_crcf_execute_block_dev(a2.q, x.data_ptr(), nb, y.data_ptr()))
    out[arg] = (round(ms, 4), round(24 * n / (ms * 1e-3) / 8e12, 3))
print("two-pass" if os.environ.get("LQ_PFB2_TWO_PASS") else "default", out)
