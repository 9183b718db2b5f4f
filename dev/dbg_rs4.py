import sys, os, faulthandler
faulthandler.enable()
sys.path.insert(0, "liquid-dsp_amd"); sys.path.insert(0, "tests")
import numpy as np
import liquidmi as LQ
import oracle_lib as O
import golden_io as G
rate = float(np.float32(1.037))
r = np.random.default_rng(1)
x = (r.uniform(-0.5, 0.5, 300000) + 1j * r.uniform(-0.5, 0.5, 300000)).astype(np.complex64)
g = LQ.Resamp(rate, 7, 0.25, 60.0, 64)
print("created", flush=True)
ys = []
cuts = [0, 3, 5, 6, 250, 251, 777, 1000, 1001, 71_003, 71_004, 140_000, 213_457, 300_000]
for a, b in zip(cuts[:-1], cuts[1:]):
    print("call", a, b, flush=True)
    ys.append(g.execute_block(x[a:b]))
    print(" ->", len(ys[-1]), flush=True)
y = np.concatenate(ys)
ref = O.Resamp(rate, 7, 0.25, 60.0, 64).execute_block(x)
print(len(y), len(ref), G.nrm_err(y, ref) if len(y) == len(ref) else None, flush=True)
