"""The host path's expanded-tap dot product (host/lq_small.c lq_host_taps /
lq_host_tdot: the per-call firfilt execute and dotprod execute on the host),
checked on CPU against a float64 numpy sum.  Taps in natural order (dotprod,
src/dotprod/src/dotprod.c:42-167: y = sum h[i] x[i]) and reversed (firfilt,
src/filter/src/firfilt.c:322-338: the window's last n samples, oldest first,
against the reversed taps).  No GPU call: the two routines are plain host code.
"""
import ctypes as C

import numpy as np
import pytest

import liquidmi as LQ

KINDS = {"rrrf": 0, "crcf": 1, "cccf": 2}  # LQ_RRRF, LQ_CRCF, LQ_CCCF (host/lq_host.h)


def _lib():
    L = C.CDLL(LQ.LIB_PATH)
    L.lq_host_taps.restype = C.c_void_p
    L.lq_host_taps.argtypes = [C.c_int, C.c_void_p, C.c_uint, C.c_int]
    L.lq_host_tdot.restype = None
    L.lq_host_tdot.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint, C.c_void_p]
    return L


@pytest.mark.parametrize("kind", sorted(KINDS))
@pytest.mark.parametrize("rev", [0, 1])
def test_host_tdot_matches_float64(kind, rev):
    L = _lib()
    libc = C.CDLL(None)
    rng = np.random.default_rng(7 + KINDS[kind] + 3 * rev)
    for n in list(range(0, 41)) + [63, 64, 65, 127, 128, 129, 255, 1000]:
        if kind == "cccf":
            h = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        else:
            h = rng.standard_normal(n).astype(np.float32)
        # one sample into a larger array: the 16-byte and 32-byte load forms
        # (lq_host_tdot picks by the samples' alignment) both run
        off = n % 2
        if kind == "rrrf":
            x = rng.standard_normal(n + 1).astype(np.float32)[off:off + n]
        else:
            x = (rng.standard_normal(n + 1) + 1j * rng.standard_normal(n + 1)).astype(np.complex64)[off:off + n]
        g = L.lq_host_taps(KINDS[kind], h.ctypes.data, n, rev)
        y = np.zeros(1, np.float32 if kind == "rrrf" else np.complex64)
        L.lq_host_tdot(KINDS[kind], g, x.ctypes.data, n, y.ctypes.data)
        libc.free(C.c_void_p(g))
        hh = h[::-1] if rev else h
        ref = np.sum(hh.astype(np.complex128) * x.astype(np.complex128))
        scale = max(1.0, float(np.sum(np.abs(hh) * np.abs(x))))
        assert abs(complex(y[0]) - ref) <= 1e-5 * scale, (kind, rev, n, y[0], ref)
