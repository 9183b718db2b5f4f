"""Edge cases of the firfilt kernels against the oracle (`-m gpu`).

The matrix-core kernel (k_firfilt_mx.hip, 33..64 taps) computes with a
three-term bf16 split; the VALU kernel pads taps with zeros to 16/32/64*k.
Neither may change what the reference computes (firfilt.c:322-338, a plain
float32 dot product over the true taps): these tests sweep the input scale
from 2^-120 to 2^120 and inject +Inf / -Inf / NaN samples, and require
  * the same finite / +Inf / -Inf / NaN pattern as the oracle, sample for
    sample (so a bad sample reaches exactly the outputs t..t+h-1 it reaches
    in the reference, none before it), and
  * normwise 1e-5 on the finite outputs (the suite's parity bound).
"""
import numpy as np
import pytest

import liquidmi as LQ
import oracle_lib as O

pytestmark = pytest.mark.gpu

TYPES = {"rrrf": O.RRRF, "crcf": O.CRCF, "cccf": O.CCCF}
NRM = 1e-5


def _data(t, n, h_len, seed, scale):
    r = np.random.default_rng(seed)
    if t == "rrrf":
        x = (r.uniform(-0.5, 0.5, n) * scale).astype(np.float32)
    else:
        x = ((r.uniform(-0.5, 0.5, n) + 1j * r.uniform(-0.5, 0.5, n)) * scale).astype(np.complex64)
    if t == "cccf":
        h = (r.uniform(-0.5, 0.5, h_len) + 1j * r.uniform(-0.5, 0.5, h_len)).astype(np.complex64)
    else:
        h = r.uniform(-0.5, 0.5, h_len).astype(np.float32)
    return h, x


def _pattern(a):
    a = np.asarray(a)
    parts = [a.real, a.imag] if np.iscomplexobj(a) else [a]
    return np.stack([np.where(np.isnan(p), 3, np.where(np.isposinf(p), 1, np.where(np.isneginf(p), 2, 0)))
                     for p in parts])


def _check(got, ref):
    assert np.array_equal(_pattern(got), _pattern(ref)), "non-finite pattern differs from the oracle"
    fin = np.isfinite(ref)
    if fin.any():
        d = np.max(np.abs(got[fin].astype(np.complex128) - ref[fin].astype(np.complex128)))
        assert d <= NRM * np.max(np.abs(ref[fin])) or d == 0.0


def _run(t, h, x, dev):
    g = LQ.FirFilt(t, h)
    if not dev:
        return g.execute_block(x)
    bx = LQ.DeviceBuffer.from_array(x)
    by = LQ.DeviceBuffer(x.nbytes)
    g.execute_block_dev(bx.p, len(x), by.p)
    g.synchronize()
    return by.to_array(x.dtype, len(x))


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("h_len", [64, 45, 20, 100, 200])
@pytest.mark.parametrize("e", [-120, -60, -40, 40, 60, 120])
def test_firfilt_input_scale_sweep(t, h_len, e):
    h, x = _data(t, 50001, h_len, 7 + h_len, 2.0 ** e)
    ref = O.FirFilt(TYPES[t], h).execute_block(x)
    _check(_run(t, h, x, dev=True), ref)


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("h_len", [64, 45, 20, 100, 200])
def test_firfilt_nonfinite_samples(t, h_len):
    h, x = _data(t, 70001, h_len, 11 + h_len, 1.0)
    # isolated +Inf, -Inf and NaN, one in the first chunk's halo region, one
    # on a 2048/4096-sample chunk seam, one deep inside; plus a second call
    x[5] = np.inf
    x[4096 - 1] = -np.inf
    x[33333] = np.nan
    if t != "rrrf":
        x[50000] = complex(1.0, np.inf)
    ref = O.FirFilt(TYPES[t], h).execute_block(x)
    _check(_run(t, h, x, dev=True), ref)
    _check(_run(t, h, x, dev=False), ref)
    # outputs strictly before the first bad sample stay finite
    assert np.all(np.isfinite(_run(t, h, x, dev=True)[:5]))


def test_firfilt_extreme_taps_stay_exact():
    # taps outside [2^-50, 2^50] keep the filter off the matrix cores
    r = np.random.default_rng(3)
    h = r.uniform(-0.5, 0.5, 64).astype(np.float32)
    h[7] = 2.0 ** -70
    h[9] = np.float32(2.0 ** 60)
    x = ((r.uniform(-0.5, 0.5, 30000) + 1j * r.uniform(-0.5, 0.5, 30000)) * 2.0 ** -20).astype(np.complex64)
    ref = O.FirFilt(O.CRCF, h).execute_block(x)
    _check(_run("crcf", h, x, dev=True), ref)


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("h_len,n", [(2050, 2049), (4000, 4096), (6001, 8000)])
def test_fftfilt_long_filters(t, h_len, n):
    # the reference accepts any h_len with n >= h_len - 1 (fftfilt.c:78-83);
    # past the 4096-point transform's reach the object runs the convolution
    # directly -- same output, same scale semantics
    r = np.random.default_rng(h_len)
    h = (r.uniform(-0.5, 0.5, h_len) + (1j * r.uniform(-0.5, 0.5, h_len) if t == "cccf" else 0)).astype(
        np.complex64 if t == "cccf" else np.float32)
    nb = 5
    if t == "rrrf":
        x = r.uniform(-0.5, 0.5, nb * n).astype(np.float32)
    else:
        x = (r.uniform(-0.5, 0.5, nb * n) + 1j * r.uniform(-0.5, 0.5, nb * n)).astype(np.complex64)
    s = 0.5   # the oracle's fftfilt scale is real (fftfilt.c:182-187 with a real s)
    g = LQ.FftFilt(h, n, t=t)
    g.set_scale(s)
    o = O.FftFilt(TYPES[t], h, n)
    o.set_scale(s)
    got = np.concatenate([g.execute(x[i * n:(i + 1) * n]) for i in range(nb)])
    ref = np.concatenate([o.execute(x[i * n:(i + 1) * n]) for i in range(nb)])
    assert np.max(np.abs(got - ref)) <= 1e-5 * np.max(np.abs(ref))


def test_fftfilt_longest_filter_and_limit():
    """fftfilt hands filters past its 4096-point transforms to the direct FIR
    kernel, which holds a tile plus the history in LDS: the longest filter it
    can take runs (vs the oracle), one tap more is refused at create time
    with a message and exit(1) -- the reference's error convention
    (fftfilt.c:74-83) -- instead of failing at the first execute."""
    import ctypes as C
    import subprocess
    import sys
    f = LQ.lib().lqk_firfilt_max_history
    f.restype, f.argtypes = C.c_uint, [C.c_int]
    L = int(f(1))
    assert L >= 8192
    r = np.random.default_rng(L)
    h = r.uniform(-0.5, 0.5, L).astype(np.float32)
    n = L
    x = (r.uniform(-0.5, 0.5, 2 * n) + 1j * r.uniform(-0.5, 0.5, 2 * n)).astype(np.complex64)
    g, o = LQ.FftFilt(h, n), O.FftFilt(O.CRCF, h, n)
    got = np.concatenate([g.execute(x[:n]), g.execute(x[n:])])
    ref = np.concatenate([o.execute(x[:n]), o.execute(x[n:])])
    assert np.max(np.abs(got - ref)) <= 1e-5 * np.max(np.abs(ref))
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import liquidmi as LQ; "
            "LQ.FftFilt(np.ones(%d, np.float32), %d); print('created')") % (
                LQ.os.path.dirname(LQ.__file__), L + 65, L + 65)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 1, (p.returncode, p.stdout, p.stderr)
    assert "exceeds the GPU kernel limit" in p.stderr
    assert "created" not in p.stdout
