"""firpfbch_crcf synthesizer kernel time for given (M, m) on 2^27 samples
(dev A/B tool; the library comes from LQ_LIB_PATH as in dev/ab/ab.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
n = 1 << 27
X = W.cbuf(n)
y = torch.empty_like(X)
out = {}
for arg in (sys.argv[1:] or ["4096:4"]):
    M, m = (int(v) for v in arg.split(":"))
    nb = n // M
    q = W.LQ.FirPfbch(W.LQ.LIQUID_SYNTHESIZER, M, m=m, As=60.0)
    q.set_stream(W.S)
    ms = W.timed(lambda: L.firpfbch_crcf_execute_block_dev(q.q, X.data_ptr(), nb, y.data_ptr()))
    out[arg] = (round(ms, 4), round(16 * n / (ms * 1e-3) / 8e12, 3))
print(os.environ.get("LQ_LIB_PATH", "default"), out)
