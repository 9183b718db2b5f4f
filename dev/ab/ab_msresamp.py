"""msresamp interpolating / decimating chains and their resampler stage alone,
device resident (dev tool): kernel time per call from HIP events on the
objects' stream, 20 warm-up + 30 timed calls.
    python dev/ab/ab_msresamp.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
import liquidmi as LQ  # noqa: E402

STREAM = torch.cuda.Stream()
S = STREAM.cuda_stream


def timed(fn, it=30, w=20):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(STREAM)
    for _ in range(it):
        fn()
    e1.record(STREAM)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    n = 1 << 26
    x = torch.rand(2 * n, device="cuda") - 0.5
    y = torch.empty(2 * 4 * n, device="cuda")
    for rate in (0.3, 3.3, 10.5):
        q = LQ.MsResamp(rate, 60.0)
        q.set_stream(S)
        nin = n if rate < 1 else n // 4
        nout = q.num_output(nin)
        ms = timed(lambda: q.execute_block_dev(x.data_ptr(), nin, y.data_ptr()))
        gb = (8 * nin + 8 * nout) / (ms * 1e-3) / 1e9
        print(json.dumps({"workload": "msresamp_crcf r=%g" % rate, "ms": round(ms, 4), "frac": round(gb / 8000, 3)}))
        q.destroy()
    for rate in (1.65, 0.6, 1.037):
        q = LQ.Resamp(rate, 7, 0.4, 60.0, 64)
        q.set_stream(S)
        nin = n // 4 if rate > 1 else n // 2
        nout = q.num_output(nin)
        ms = timed(lambda: q.execute_block_dev(x.data_ptr(), nin, y.data_ptr()))
        gb = (8 * nin + 8 * nout) / (ms * 1e-3) / 1e9
        print(json.dumps({"workload": "resamp_crcf r=%g" % rate, "ms": round(ms, 4), "frac": round(gb / 8000, 3)}))
        q.destroy()


if __name__ == "__main__":
    main()
