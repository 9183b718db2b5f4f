"""msresamp_crcf r=0.3 (2^26 inputs, device resident): ms per call (A/B of the
chained decimator's chunking, r06ms: the LQ_MS_CHUNK knob it read was a
temporary build of host/resamp2.c, removed after the run)."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
import bench_widened as B  # noqa: E402
import liquidmi as LQ  # noqa: E402
n = 1 << 26
x = B.cbuf(n)
y = torch.empty(2 * n, device="cuda")
for rate in (0.3, 0.2):
    m = LQ.MsResamp(rate, 60.0)
    m.set_stream(B.S)
    best = min(B.timed(lambda: m.execute_block_dev(x.data_ptr(), n, y.data_ptr())) for _ in range(3))
    print("chunk", os.environ.get("LQ_MS_CHUNK", "off"), "rate", rate, "ms %.4f" % best, flush=True)
    m.destroy()
