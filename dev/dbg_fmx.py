"""Where a firfilt long-stream run departs from the oracle (dev tool): the
test_firfilt_crcf_matrix_core_path_long_stream case for (type, hlen) from
argv, the library from LQ_LIB_PATH; prints the mismatching index ranges."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
import test_gpu_parity as T  # noqa: E402

t, hlen = sys.argv[1], int(sys.argv[2])
r = T.rng(100 + hlen)
h = T.coefs(r, t, hlen)
n0, n1, n2 = 6000, (3 << 20) + 12345, 777
x = T.samples(r, t, n0 + n1 + n2)
esz = x.itemsize
g = T.LQ.FirFilt(t, h)
s = (0.7 - 0.2j) if t == "cccf" else 0.7
g.set_scale(s)
bx = T.LQ.DeviceBuffer.from_array(x)
by = T.LQ.DeviceBuffer(x.nbytes)
g.execute_block_dev(bx.p, n0, by.p)
g.execute_block_dev(bx.p + n0 * esz, n1, by.p + n0 * esz)
g.execute_block_dev(bx.p + (n0 + n1) * esz, n2, by.p + (n0 + n1) * esz)
g.synchronize()
y = by.to_array(x.dtype, len(x))
o = T.O.FirFilt(T.TYPES[t], h)
o.set_scale(s)
ref = o.execute_block(x)
err = np.abs(y - ref) / np.max(np.abs(ref))
bad = np.nonzero(err > 1e-4)[0]
print(os.environ.get("LQ_LIB_PATH", "main"), t, hlen, "nrm", T.G.nrm_err(y, ref), "bad", len(bad))
if len(bad):
    # contiguous runs of bad indices
    runs, st = [], bad[0]
    for a, b in zip(bad[:-1], bad[1:]):
        if b != a + 1:
            runs.append((st, a))
            st = b
    runs.append((st, bad[-1]))
    print("runs", len(runs), [(int(a), int(b), int(b - a + 1)) for a, b in runs[:12]])
    i = bad[0]
    print("first", i, y[i], ref[i], "chunk(2048)", (i - n0) // 2048, "offset", (i - n0) % 2048)
