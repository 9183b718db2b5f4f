"""Full-size parity at the BASELINE configurations (`-m gpu`).

configs[3] (firpfbch2_crcf analyzer M=1024 m=4, 2^27 samples) and the
headline firfilt_crcf h=64 stream at 2^28 samples, each compared with the
CPU oracle over the WHOLE stream -- not a slice.  The oracle runs split
across host processes with the lqshard plans (tests/parallel_oracle.py);
its own sharding is exact (tests/test_multirank.py), so this is the oracle
of the single stream.  Bound: normwise 1e-5 (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

import liquidmi as LQ
import lqshard
import parallel_oracle as PO

pytestmark = pytest.mark.gpu


def _stream(n, seed):
    r = np.random.default_rng(seed)
    x = np.empty(n, np.complex64)
    step = 1 << 24
    for a in range(0, n, step):
        b = min(n, a + step)
        x[a:b] = (r.uniform(-0.5, 0.5, b - a) + 1j * r.uniform(-0.5, 0.5, b - a)).astype(np.complex64)
    return x


def test_firpfbch2_config4_full_stream_vs_oracle():
    M, m, n = 1024, 4, 1 << 27
    x = _stream(n, 404)
    dx = LQ.DeviceBuffer.from_array(x)
    nb = n // (M // 2)
    dy = LQ.DeviceBuffer(nb * M * 8)
    q = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, m, 60.0)
    q.execute_block_dev(dx.p, nb, dy.p)
    q.synchronize()
    dx.free()
    y = dy.to_array(np.complex64, nb * M)
    dy.free()
    err, nonfin = PO.compare("firpfbch2", x, y, (M, m), lqshard.firpfbch2_plan(nb, PO.workers(), M, m))
    assert nonfin == 0
    assert err < 1e-5, err


def test_firfilt_h64_2p28_full_stream_vs_oracle():
    n = 1 << 28
    x = _stream(n, 101)
    h = np.random.default_rng(5).uniform(-0.5, 0.5, 64).astype(np.float32)
    dx = LQ.DeviceBuffer.from_array(x)
    dy = LQ.DeviceBuffer(n * 8)
    q = LQ.FirFilt("crcf", h)
    q.execute_block_dev(dx.p, n, dy.p)
    q.synchronize()
    dx.free()
    y = dy.to_array(np.complex64, n)
    dy.free()
    err, nonfin = PO.compare("firfilt", x, y, (h,), lqshard.firfilt_plan(n, PO.workers(), len(h)))
    assert nonfin == 0
    assert err < 1e-5, err
