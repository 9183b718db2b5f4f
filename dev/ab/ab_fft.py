"""FFT plan API batch timing for the large sizes (dev A/B tool): ms per call
from HIP events, 20 warm-up + 30 timed calls; LQ_FFT_CHUNK_MB selects the
four-step chunk size."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tools"))
import bench_widened as W  # noqa: E402

L = W.LQ.lib()
out = {}
for N in (4096, 8192, 16384, 65536, 1 << 20):
    B = (1 << 26) // N
    Z = W.cbuf(B * N)
    pl = L.fft_create_plan(N, None, None, 1, 0)
    L.fft_set_stream(pl, W.S)
    ms = W.timed(lambda: L.fft_execute_batch_dev(pl, Z.data_ptr(), Z.data_ptr(), B))
    out[N] = (round(ms, 4), round(16 * B * N / (ms * 1e-3) / 8e12, 3))
    L.fft_destroy_plan(pl)
print(os.environ.get("LQ_FFT_CHUNK_MB", "0"), json.dumps(out))
