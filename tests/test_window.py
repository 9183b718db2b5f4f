"""windowf / windowcf (include/liquid.h:296-349) -- a host container, no GPU.

Pinned by the reference's own known answers (src/buffer/tests/
window_autotest.c:29-140, the test0..test8 vectors) and by a random sequence
of push / write / recreate / clear checked against a model of the
documented semantics (window.c:45-214: the last len samples, oldest first,
zeros initially).
"""
import ctypes as C

import numpy as np
import pytest

import liquidmi as LQ


def _lib():
    L = LQ.lib()
    for t, ct in (("windowf", C.c_float), ("windowcf", LQ.cfloat)):
        getattr(L, t + "_create").restype = C.c_void_p
        getattr(L, t + "_create").argtypes = [C.c_uint]
        getattr(L, t + "_recreate").restype = C.c_void_p
        getattr(L, t + "_recreate").argtypes = [C.c_void_p, C.c_uint]
        for fn in ("_destroy", "_clear", "_print", "_debug_print"):
            getattr(L, t + fn).argtypes = [C.c_void_p]
        getattr(L, t + "_read").argtypes = [C.c_void_p, C.c_void_p]
        getattr(L, t + "_index").argtypes = [C.c_void_p, C.c_uint, C.c_void_p]
        getattr(L, t + "_push").argtypes = [C.c_void_p, ct]
        getattr(L, t + "_write").argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
    return L


def _read(L, t, w, n):
    p = C.c_void_p()
    getattr(L, t + "_read")(w, C.byref(p))
    dt = np.float32 if t == "windowf" else np.complex64
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), shape=(n * (1 if t == "windowf" else 2),)) \
        .view(dt).copy()


def test_windowf_reference_autotest():
    L = _lib()
    v = np.array([9, 8, 7, 6, 5, 4, 3, 2, 1, 0], np.float32)
    w = L.windowf_create(10)
    assert np.array_equal(_read(L, "windowf", w, 10), np.zeros(10))
    for _ in range(4):
        L.windowf_push(w, 1.0)
    assert np.array_equal(_read(L, "windowf", w, 10), [0, 0, 0, 0, 0, 0, 1, 1, 1, 1])
    L.windowf_write(w, v.ctypes.data, 4)
    assert np.array_equal(_read(L, "windowf", w, 10), [0, 0, 1, 1, 1, 1, 9, 8, 7, 6])
    for _ in range(4):
        L.windowf_push(w, 3.0)
    test3 = [1, 1, 9, 8, 7, 6, 3, 3, 3, 3]
    assert np.array_equal(_read(L, "windowf", w, 10), test3)
    x = C.c_float()
    for i in range(10):
        L.windowf_index(w, i, C.byref(x))
        assert x.value == test3[i]
    for _ in range(4):
        L.windowf_push(w, 5.0)
    assert np.array_equal(_read(L, "windowf", w, 10), [7, 6, 3, 3, 3, 3, 5, 5, 5, 5])
    w = L.windowf_recreate(w, 6)
    assert np.array_equal(_read(L, "windowf", w, 6), [3, 3, 5, 5, 5, 5])
    L.windowf_push(w, 6.0)
    L.windowf_push(w, 7.0)
    assert np.array_equal(_read(L, "windowf", w, 6), [5, 5, 5, 5, 6, 7])
    w = L.windowf_recreate(w, 10)
    assert np.array_equal(_read(L, "windowf", w, 10), [0, 0, 0, 0, 5, 5, 5, 5, 6, 7])
    L.windowf_clear(w)
    assert np.array_equal(_read(L, "windowf", w, 10), np.zeros(10))
    L.windowf_destroy(w)


@pytest.mark.parametrize("t", ["windowf", "windowcf"])
@pytest.mark.parametrize("n", [1, 2, 7, 64, 1000])
def test_window_random_ops_vs_model(t, n):
    L = _lib()
    r = np.random.default_rng(n)
    dt = np.float32 if t == "windowf" else np.complex64
    model = np.zeros(n, dt)
    w = getattr(L, t + "_create")(n)
    for step in range(400):
        op = r.integers(0, 10)
        if op < 5:
            v = dt(r.normal()) if t == "windowf" else dt(complex(r.normal(), r.normal()))
            getattr(L, t + "_push")(w, float(v) if t == "windowf" else LQ.cfloat(v.real, v.imag))
            model = np.concatenate([model[1:], [v]])
        elif op < 8:
            k = int(r.integers(0, 3 * n + 2))
            a = (r.normal(size=k) + (1j * r.normal(size=k) if t == "windowcf" else 0)).astype(dt)
            getattr(L, t + "_write")(w, a.ctypes.data, k)
            model = np.concatenate([model, a])[-n:]
        elif op == 8:
            n2 = int(r.integers(1, 2 * n + 2))
            w = getattr(L, t + "_recreate")(w, n2)
            model = np.concatenate([np.zeros(max(0, n2 - n), dt), model[-min(n, n2):]])
            n = n2
        else:
            getattr(L, t + "_clear")(w)
            model = np.zeros(n, dt)
        assert np.array_equal(_read(L, t, w, n), model), (step, op)
    getattr(L, t + "_destroy")(w)
