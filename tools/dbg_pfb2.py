import sys, numpy as np
sys.path.insert(0,'liquid-dsp_amd'); sys.path.insert(0,'tests')
import liquidmi as LQ, oracle_lib as O, golden_io as G
for (M,m) in [(2,1),(8,2),(1024,4),(1024,2)]:
    r = np.random.default_rng(M+m)
    nb = 64
    x = (r.uniform(-.5,.5,nb*M//2)+1j*r.uniform(-.5,.5,nb*M//2)).astype(np.complex64)
    g = LQ.FirPfbch2(0, M, m, 60.0); o = O.FirPfbch2(0, M, m, 60.0)
    y = g.execute_block(x); ref = o.execute_block(x)
    err = np.abs(y-ref).reshape(nb, M).max(axis=1)/np.abs(ref).max()
    print(M, m, "whole-call err per block (first 8):", err[:8], "max", err.max(), flush=True)
    g2 = LQ.FirPfbch2(0, M, m, 60.0)
    cuts=[0,1,4,5,30,nb]; step=M//2
    y2 = np.concatenate([g2.execute_block(x[a*step:b*step]) for a,b in zip(cuts[:-1],cuts[1:])])
    err2 = np.abs(y2-ref).reshape(nb, M).max(axis=1)/np.abs(ref).max()
    print(M, m, "cut-call err per block:", np.round(np.log10(err2+1e-12),1), flush=True)
