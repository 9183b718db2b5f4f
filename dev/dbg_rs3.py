import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "liquid-dsp_amd")
import numpy as np
import liquidmi as LQ, oracle_lib as O
r = np.random.default_rng(1)
for rate, n, calls in [(30.0, 64, None), (30.0, 200, None), (30.0, 64, [16, 48]), (20.0, 100, None), (10.3, 300, None)]:
    rate = float(np.float32(rate))
    x = (r.uniform(-0.5, 0.5, n) + 1j * r.uniform(-0.5, 0.5, n)).astype(np.complex64)
    g = LQ.Resamp(rate, 7, 0.25, 60.0, 64)
    o = O.Resamp(rate, 7, 0.25, 60.0, 64)
    if calls:
        ys = []; a = 0
        for c in calls:
            ys.append(g.execute_block(x[a:a + c])); a += c
        y = np.concatenate(ys)
    else:
        y = g.execute_block(x)
    ref = o.execute_block(x)
    bad = np.nonzero(np.abs(y - ref) > 1e-5 * np.max(np.abs(ref)))[0] if len(y) == len(ref) else None
    print(rate, n, calls, len(y), len(ref), None if bad is None else (len(bad), bad[:20], bad[-5:] if len(bad) else []))
