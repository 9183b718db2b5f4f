"""firpfbch2 analyzer mismatch map against the oracle (dev tool): per-block and per-bin error for one call."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "liquid-dsp_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import liquidmi as LQ
import oracle_lib as O
M, m = int(sys.argv[1]) if len(sys.argv) > 1 else 2048, int(sys.argv[2]) if len(sys.argv) > 2 else 4
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 64
r = np.random.default_rng(5)
x = (r.uniform(-0.5, 0.5, nb * M // 2) + 1j * r.uniform(-0.5, 0.5, nb * M // 2)).astype(np.complex64)
cuts = [int(c) for c in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, nb]
g = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, m, 60.0)
y = np.concatenate([g.execute_block(x[a * M // 2:b * M // 2]) for a, b in zip(cuts[:-1], cuts[1:])]).reshape(nb, M)
ref = O.FirPfbch2(O.ANALYZER, M, m, 60.0).execute_block(x).reshape(nb, M)
e = np.abs(y - ref) / np.max(np.abs(ref))
print("max err %.3g" % e.max())
bad = e > 1e-4
print("bad blocks:", np.nonzero(bad.any(axis=1))[0][:40].tolist(), "of", nb)
print("bad bins per bad block:", bad.sum(axis=1)[bad.any(axis=1)][:20].tolist())
b0 = int(np.argmax(e.max(axis=1)))
idx = np.nonzero(bad[b0])[0]
print("block", b0, "bad bins first:", idx[:20].tolist(), "count", len(idx))
# is the block a permutation / scaling of the reference?
yy, rr = y[b0], ref[b0]
print("norm ratio %.4f" % (np.linalg.norm(yy) / np.linalg.norm(rr)))
X = np.fft.fft(yy) ; XR = np.fft.fft(rr)
print("spectral (X domain) bad count:", int(np.sum(np.abs(X - XR) > 1e-3 * np.abs(XR).max())))
d = np.abs(X - XR) > 1e-3 * np.abs(XR).max()
print("X-domain bad idx first:", np.nonzero(d)[0][:20].tolist())
