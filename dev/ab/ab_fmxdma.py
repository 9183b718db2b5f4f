"""firfilt_crcf h=64: the LDS-DMA staged matrix-core kernel (LQ_FMX_DMA=1)
against the shipped one, same process and buffers (dev tool): bitwise
parity on streamed / ragged / non-finite inputs, then alternated timings over
three freshly allocated 2^28-sample buffer pairs."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
torch.manual_seed(3)
h = (torch.rand(64) - 0.5).numpy()


def run(dma, x, n, calls):
    if dma:
        os.environ["LQ_FMX_DMA"] = "1"
    else:
        os.environ.pop("LQ_FMX_DMA", None)
    q = W.LQ.FirFilt("crcf", h)
    q.set_stream(W.S)
    y = torch.empty_like(x)
    o = 0
    for m in calls:
        L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr() + 8 * o, m, y.data_ptr() + 8 * o)
        o += m
    torch.cuda.synchronize()
    return y


ok = True
for name, n, calls, bad in [("2^28 two calls", 1 << 28, [(1 << 27) + 2048 * 7, (1 << 27) - 2048 * 7], None),
                            ("ragged", 3 * 2048 * 512 + 776, [1000000, 3 * 2048 * 512 + 776 - 1000000], None),
                            ("small", 5000, [5000], None),
                            ("inf + nan", 1 << 22, [1 << 21, 1 << 21], (123457, 3000000))]:
    x = W.cbuf(n, seed=7)
    if bad:
        x[2 * bad[0]] = float("inf")
        x[2 * bad[1] + 1] = float("nan")
    ya = run(False, x, n, calls)
    yb = run(True, x, n, calls)
    same = torch.equal(ya.view(torch.int32), yb.view(torch.int32))
    ok &= same
    print("parity %-16s bitwise %s" % (name, same))
    del x, ya, yb
sys.stdout.flush()
if not ok:
    sys.exit(1)

n = 1 << 28
for pair in range(3):
    x = W.cbuf(n, seed=pair + 1)
    y = torch.empty_like(x)
    res = {False: [], True: []}
    for rep in range(3):
        for dma in (False, True):
            if dma:
                os.environ["LQ_FMX_DMA"] = "1"
            else:
                os.environ.pop("LQ_FMX_DMA", None)
            q = W.LQ.FirFilt("crcf", h)
            q.set_stream(W.S)
            res[dma].append(W.timed(lambda: L.firfilt_crcf_execute_block_dev(q.q, x.data_ptr(), n, y.data_ptr()),
                                    it=20, w=10))
    print("pair %d x %#x: shipped %s  dma %s" % (pair, x.data_ptr(), " ".join("%.4f" % v for v in res[False]),
                                                 " ".join("%.4f" % v for v in res[True])))
    sys.stdout.flush()
    del x, y
