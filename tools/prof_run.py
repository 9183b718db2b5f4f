#!/usr/bin/env python3
"""Short driver for profiling: the two headline kernels, a few launches each,
device-resident synthetic data (same shapes as bench.py)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
import torch  # noqa: E402

import liquidmi as LQ  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=3)
p.add_argument("--what", default="both", choices=["both", "all", "pfb2", "fir", "resamp", "fftfilt", "rs165", "ms33"])
a = p.parse_args()
s = torch.cuda.Stream()
if a.what in ("both", "all", "pfb2"):
    n = 1 << 27
    x = torch.rand(2 * n, device="cuda") - 0.5
    y = torch.empty(4 * n, device="cuda")
    q = LQ.FirPfbch2(0, 1024, 4, 60.0)
    q.set_stream(s.cuda_stream)
    for _ in range(a.iters):
        q.execute_block_dev(x.data_ptr(), n // 512, y.data_ptr())
    q.synchronize()
    q.destroy()
    del x, y
if a.what in ("both", "all", "fir"):
    n = 1 << 28
    x = torch.rand(2 * n, device="cuda") - 0.5
    y = torch.empty(2 * n, device="cuda")
    f = LQ.FirFilt("crcf", (torch.rand(64) - 0.5).numpy())
    f.set_stream(s.cuda_stream)
    for _ in range(a.iters):
        f.execute_block_dev(x.data_ptr(), n, y.data_ptr())
    f.synchronize()
    f.destroy()
if a.what in ("all", "resamp"):
    n = 1 << 25
    x = torch.rand(2 * n, device="cuda") - 0.5
    y = torch.empty(2 * (int(n * 1.037) + 4096), device="cuda")
    r = LQ.Resamp(1.037, 7, 0.25, 60.0, 64)
    r.set_stream(s.cuda_stream)
    r.num_output(n)
    for _ in range(a.iters):
        r.execute_block_dev(x.data_ptr(), n, y.data_ptr())
    r.synchronize()
    r.destroy()
if a.what == "rs165":   # the resampler alone at msresamp r = 3.3's arbitrary rate
    n = 1 << 24
    x = torch.rand(2 * n, device="cuda") - 0.5
    y = torch.empty(2 * (int(n * 1.65) + 4096), device="cuda")
    r = LQ.Resamp(1.65, 7, 0.4, 60.0, 64)
    r.set_stream(s.cuda_stream)
    for _ in range(a.iters):
        r.execute_block_dev(x.data_ptr(), n, y.data_ptr())
    r.synchronize()
    r.destroy()
if a.what == "ms33":   # msresamp r = 3.3: the resampler + half-band chain
    n = 1 << 24
    x = torch.rand(2 * n, device="cuda") - 0.5
    y = torch.empty(2 * (int(n * 3.3) + 4096), device="cuda")
    r = LQ.MsResamp(3.3, 60.0)
    r.set_stream(s.cuda_stream)
    for _ in range(a.iters):
        r.execute_block_dev(x.data_ptr(), n, y.data_ptr())
    r.synchronize()
    r.destroy()
if a.what in ("all", "fftfilt"):
    n = 1 << 26
    x = torch.rand(2 * n, device="cuda") - 0.5
    y = torch.empty(2 * n, device="cuda")
    ff = LQ.FftFilt((torch.rand(512) - 0.5).numpy(), 2048)
    ff.set_stream(s.cuda_stream)
    for _ in range(a.iters):
        ff.execute_block_dev(x.data_ptr(), n, y.data_ptr())
    torch.cuda.synchronize()
    ff.destroy()
torch.cuda.synchronize()
print("done")
