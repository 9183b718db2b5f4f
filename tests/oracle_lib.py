"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "_build", "liboracle.so")

RRRF, CRCF, CCCF = 0, 1, 2
ANALYZER, SYNTHESIZER = 0, 1

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def _declare(L):
    vp, u, f, i = C.c_void_p, C.c_uint, C.c_float, C.c_int
    ul = C.c_ulong
    sig = {
        "orc_firdes_kaiser": (None, [u, f, f, f, vp]),
        "orc_kaiser_beta_As": (f, [f]),
        "orc_dotprod_rrrf_run4": (None, [vp, vp, u, vp]),
        "orc_dotprod_crcf_run4": (None, [vp, vp, u, vp]),
        "orc_dotprod_cccf_run4": (None, [vp, vp, u, vp]),
        "orc_dotprod_rrrf_batch": (None, [vp, vp, u, ul, vp]),
        "orc_dotprod_crcf_batch": (None, [vp, vp, u, ul, vp]),
        "orc_dotprod_cccf_batch": (None, [vp, vp, u, ul, vp]),
        "orc_fft": (None, [u, vp, vp, i]),
        "orc_firfilt_create": (vp, [i, vp, u]),
        "orc_firfilt_destroy": (None, [vp]),
        "orc_firfilt_reset": (None, [vp]),
        "orc_firfilt_set_scale": (None, [vp, f, f]),
        "orc_firfilt_push": (None, [vp, vp]),
        "orc_firfilt_execute": (None, [vp, vp]),
        "orc_firfilt_execute_block": (None, [vp, vp, u, vp]),
        "orc_firdecim_create": (vp, [i, u, vp, u]),
        "orc_firdecim_create_kaiser": (vp, [u, u, f]),
        "orc_firdecim_destroy": (None, [vp]),
        "orc_firdecim_execute_block": (None, [vp, vp, u, vp]),
        "orc_firpfb_create": (vp, [i, u, vp, u]),
        "orc_firpfb_destroy": (None, [vp]),
        "orc_firpfb_push": (None, [vp, vp]),
        "orc_firpfb_execute": (None, [vp, u, vp]),
        "orc_firpfb_set_scale": (None, [vp, f]),
        "orc_firinterp_create": (vp, [i, u, vp, u]),
        "orc_firinterp_create_kaiser": (vp, [u, u, f]),
        "orc_firinterp_destroy": (None, [vp]),
        "orc_firinterp_execute_block": (None, [vp, vp, u, vp]),
        "orc_spgram_create": (vp, [i, u, vp, u]),
        "orc_spgram_destroy": (None, [vp]),
        "orc_spgram_reset": (None, [vp]),
        "orc_spgram_write": (None, [vp, vp, u]),
        "orc_spgram_execute": (None, [vp, vp]),
        "orc_spgram_execute_psd": (None, [vp, vp]),
        "orc_spgram_accumulate_psd": (None, [vp, vp, f, u]),
        "orc_spgram_write_accumulation": (None, [vp, vp]),
        "orc_spgram_estimate_psd": (None, [vp, vp, u, vp]),
        "orc_resamp2_create": (vp, [i, u, f, f]),
        "orc_resamp2_destroy": (None, [vp]),
        "orc_resamp2_clear": (None, [vp]),
        "orc_resamp2_run": (None, [vp, i, vp, u, vp, vp]),
        "orc_msresamp2_create": (vp, [i, i, u, f, f, f]),
        "orc_msresamp2_destroy": (None, [vp]),
        "orc_msresamp2_reset": (None, [vp]),
        "orc_msresamp2_execute": (None, [vp, vp, vp]),
        "orc_msresamp_create": (vp, [f, f]),
        "orc_msresamp_destroy": (None, [vp]),
        "orc_msresamp_reset": (None, [vp]),
        "orc_msresamp_execute": (None, [vp, vp, u, vp, C.POINTER(C.c_uint)]),
        "orc_resamp_create": (vp, [f, u, f, f, u]),
        "orc_resamp_destroy": (None, [vp]),
        "orc_resamp_reset": (None, [vp]),
        "orc_resamp_set_rate": (None, [vp, f]),
        "orc_resamp_adjust_rate": (None, [vp, f]),
        "orc_resamp_execute_block": (None, [vp, vp, u, vp, C.POINTER(C.c_uint)]),
        "orc_resamp_schedule": (ul, [f, u, ul, vp, vp, vp, ul]),
        "orc_fftfilt_create": (vp, [i, vp, u, u]),
        "orc_fftfilt_destroy": (None, [vp]),
        "orc_fftfilt_set_scale": (None, [vp, f]),
        "orc_fftfilt_execute": (None, [vp, vp, vp]),
        "orc_firpfbch_create": (vp, [i, u, u, vp]),
        "orc_firpfbch_create_kaiser": (vp, [i, u, u, f]),
        "orc_firpfbch_destroy": (None, [vp]),
        "orc_firpfbch_analyzer_execute": (None, [vp, vp, vp]),
        "orc_firpfbch_synthesizer_execute": (None, [vp, vp, vp]),
        "orc_firpfbch2_create": (vp, [i, u, u, vp]),
        "orc_firpfbch2_create_kaiser": (vp, [i, u, u, f]),
        "orc_firpfbch2_destroy": (None, [vp]),
        "orc_firpfbch2_reset": (None, [vp]),
        "orc_firpfbch2_execute": (None, [vp, vp, vp]),
        "orc_firpfbch2_execute_block": (None, [vp, vp, u, vp]),
        "orc_firpfbch2_prototype": (None, [i, u, u, f, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _arr(a, typ):
    dt = np.float32 if typ == RRRF else np.complex64
    return np.ascontiguousarray(a, dtype=dt)


def _coef(h, typ):
    return np.ascontiguousarray(h, dtype=np.complex64 if typ == CCCF else np.float32)


# --------------------------------------------------------------------------- design
def firdes_kaiser(n, fc, As, mu=0.0):
    h = np.zeros(n, np.float32)
    lib().orc_firdes_kaiser(n, fc, As, mu, ptr(h))
    return h


def firpfbch2_prototype(typ, M, m, As):
    h = np.zeros(2 * M * m + 1, np.float32)
    lib().orc_firpfbch2_prototype(typ, M, m, As, ptr(h))
    return h


# --------------------------------------------------------------------------- dotprod
def dotprod(typ, h, x):
    h = _coef(h, typ)
    x = _arr(x, typ)
    y = np.zeros(1, np.float32 if typ == RRRF else np.complex64)
    fn = {RRRF: "orc_dotprod_rrrf_run4", CRCF: "orc_dotprod_crcf_run4", CCCF: "orc_dotprod_cccf_run4"}[typ]
    getattr(lib(), fn)(ptr(h), ptr(x), len(h), ptr(y))
    return y[0]


def dotprod_batch(typ, h, X):
    h = _coef(h, typ)
    X = _arr(X, typ)
    n = len(h)
    nvec = X.size // n
    Y = np.zeros(nvec, np.float32 if typ == RRRF else np.complex64)
    fn = {RRRF: "orc_dotprod_rrrf_batch", CRCF: "orc_dotprod_crcf_batch", CCCF: "orc_dotprod_cccf_batch"}[typ]
    getattr(lib(), fn)(ptr(h), ptr(X), n, nvec, ptr(Y))
    return Y


def fft(x, direction=+1):
    x = np.ascontiguousarray(x, np.complex64)
    y = np.zeros_like(x)
    lib().orc_fft(len(x), ptr(x), ptr(y), direction)
    return y


# --------------------------------------------------------------------------- objects
class _Obj:
    _destroy = None

    def __del__(self):
        if getattr(self, "q", None):
            getattr(lib(), self._destroy)(self.q)
            self.q = None


class FirFilt(_Obj):
    _destroy = "orc_firfilt_destroy"

    def __init__(self, typ, h):
        self.typ = typ
        h = _coef(h, typ)
        self.q = lib().orc_firfilt_create(typ, ptr(h), len(h))

    def set_scale(self, s):
        s = complex(s)
        lib().orc_firfilt_set_scale(self.q, s.real, s.imag)

    def reset(self):
        lib().orc_firfilt_reset(self.q)

    def push(self, v):
        a = _arr([v], self.typ)
        lib().orc_firfilt_push(self.q, ptr(a))

    def execute(self):
        y = _arr([0], self.typ)
        lib().orc_firfilt_execute(self.q, ptr(y))
        return y[0]

    def execute_block(self, x):
        x = _arr(x, self.typ)
        y = np.zeros_like(x)
        lib().orc_firfilt_execute_block(self.q, ptr(x), len(x), ptr(y))
        return y


class FirDecim(_Obj):
    _destroy = "orc_firdecim_destroy"

    def __init__(self, typ, M, h=None, m=None, As=None):
        self.typ, self.M = typ, M
        if h is None and typ != CRCF:   # firdecim.c:88-122 design, first 2Mm taps, any type
            h = firdes_kaiser(2 * M * m + 1, 0.5 / M, As, 0.0)[:2 * M * m]
        if h is None:
            self.q = lib().orc_firdecim_create_kaiser(M, m, As)
        else:
            h = _coef(h, typ)
            self.q = lib().orc_firdecim_create(typ, M, ptr(h), len(h))

    def execute_block(self, x):
        x = _arr(x, self.typ)
        n = len(x) // self.M
        y = np.zeros(n, x.dtype)
        lib().orc_firdecim_execute_block(self.q, ptr(x), n, ptr(y))
        return y


class FirPfb(_Obj):
    _destroy = "orc_firpfb_destroy"

    def __init__(self, typ, M, h):
        self.typ = typ
        h = _coef(h, typ)
        self.q = lib().orc_firpfb_create(typ, M, ptr(h), len(h))

    def push(self, v):
        a = _arr([v], self.typ)
        lib().orc_firpfb_push(self.q, ptr(a))

    def set_scale(self, s):
        lib().orc_firpfb_set_scale(self.q, s)

    def execute(self, i):
        y = _arr([0], self.typ)
        lib().orc_firpfb_execute(self.q, i, ptr(y))
        return y[0]


class FirInterp(_Obj):
    _destroy = "orc_firinterp_destroy"

    def __init__(self, typ, M, h=None, m=None, As=None):
        self.typ, self.M = typ, M
        if h is None and typ != CRCF:   # firinterp.c:92-120 design, first 2Mm taps, any type
            h = firdes_kaiser(2 * M * m + 1, 0.5 / M, As, 0.0)[:2 * M * m]
        if h is None:
            self.q = lib().orc_firinterp_create_kaiser(M, m, As)
        else:
            h = _coef(h, typ)
            self.q = lib().orc_firinterp_create(typ, M, ptr(h), len(h))

    def execute_block(self, x):
        x = _arr(x, self.typ)
        y = np.zeros(len(x) * self.M, x.dtype)
        lib().orc_firinterp_execute_block(self.q, ptr(x), len(x), ptr(y))
        return y


class Resamp(_Obj):
    _destroy = "orc_resamp_destroy"

    def __init__(self, rate, m=7, fc=0.25, As=60.0, npfb=64):
        self.rate = rate
        self.q = lib().orc_resamp_create(rate, m, fc, As, npfb)

    def reset(self):
        lib().orc_resamp_reset(self.q)

    def set_rate(self, r):
        self.rate = r
        lib().orc_resamp_set_rate(self.q, r)

    def adjust_rate(self, d):
        lib().orc_resamp_adjust_rate(self.q, d)
        self.rate = min(0.5, max(-0.5, self.rate + d))

    def execute_block(self, x):
        x = _arr(x, CRCF)
        cap = int(np.ceil(len(x) * self.rate)) + 16
        y = np.zeros(cap, np.complex64)
        ny = C.c_uint(0)
        lib().orc_resamp_execute_block(self.q, ptr(x), len(x), ptr(y), C.byref(ny))
        return y[: ny.value]


class Resamp2(_Obj):
    """resamp2 (resamp2.c:46-360); ctaps: complex taps (cccf)."""
    _destroy = "orc_resamp2_destroy"
    NIN = {0: 1, 1: 2, 2: 2, 3: 2, 4: 1}
    NOUT = {0: 1, 1: 2, 2: 2, 3: 1, 4: 2}

    def __init__(self, m, f0, As, ctaps=False):
        self.q = lib().orc_resamp2_create(int(ctaps), m, f0, As)

    def clear(self):
        lib().orc_resamp2_clear(self.q)

    def run(self, mode, x):
        x = _arr(x, CRCF)
        n = len(x) // self.NIN[mode]
        y0 = np.zeros(n * self.NOUT[mode], np.complex64)
        y1 = np.zeros(n, np.complex64)
        lib().orc_resamp2_run(self.q, mode, ptr(x), n, ptr(y0), ptr(y1))
        return (y0, y1) if mode == 0 else y0


class MsResamp2(_Obj):
    _destroy = "orc_msresamp2_destroy"

    def __init__(self, typ, ns, fc, f0, As, ctaps=False):
        self.typ, self.M = typ, 1 << ns
        self.q = lib().orc_msresamp2_create(int(ctaps), typ, ns, fc, f0, As)

    def execute_block(self, x):
        x = _arr(x, CRCF)
        if self.typ == 0:
            y = np.zeros(len(x) * self.M, np.complex64)
            for i in range(len(x)):
                lib().orc_msresamp2_execute(self.q, ptr(x[i:i + 1]), ptr(y[i * self.M:]))
        else:
            n = len(x) // self.M
            y = np.zeros(n, np.complex64)
            for i in range(n):
                lib().orc_msresamp2_execute(self.q, ptr(x[i * self.M:(i + 1) * self.M]), ptr(y[i:]))
        return y


class MsResamp(_Obj):
    _destroy = "orc_msresamp_destroy"

    def __init__(self, rate, As):
        self.rate = rate
        self.q = lib().orc_msresamp_create(rate, As)

    def reset(self):
        lib().orc_msresamp_reset(self.q)

    def execute(self, x):
        x = _arr(x, CRCF)
        y = np.zeros(int(np.ceil(len(x) * self.rate)) + 64, np.complex64)
        ny = C.c_uint(0)
        lib().orc_msresamp_execute(self.q, ptr(x), len(x), ptr(y), C.byref(ny))
        return y[:ny.value]


def resamp_schedule(rate, npfb, nx):
    cap = int(np.ceil(nx * rate)) + 16
    b = np.zeros(cap, np.int32)
    mu = np.zeros(cap, np.float32)
    idx = np.zeros(cap, np.uint32)
    k = lib().orc_resamp_schedule(rate, npfb, nx, ptr(b), ptr(mu), ptr(idx), cap)
    return b[:k], mu[:k], idx[:k]


class FftFilt(_Obj):
    _destroy = "orc_fftfilt_destroy"

    def __init__(self, typ, h, n):
        self.typ, self.n = typ, n
        h = _coef(h, typ)
        self.q = lib().orc_fftfilt_create(typ, ptr(h), len(h), n)

    def set_scale(self, s):
        lib().orc_fftfilt_set_scale(self.q, s)

    def execute(self, x):
        x = _arr(x, self.typ)
        assert len(x) == self.n
        y = np.zeros_like(x)
        lib().orc_fftfilt_execute(self.q, ptr(x), ptr(y))
        return y

    def execute_stream(self, x):
        x = _arr(x, self.typ)
        nb = len(x) // self.n
        return np.concatenate([self.execute(x[b * self.n:(b + 1) * self.n]) for b in range(nb)]) \
            if nb else np.zeros(0, x.dtype)


class FirPfbch(_Obj):
    _destroy = "orc_firpfbch_destroy"

    def __init__(self, typ, M, p=None, h=None, m=None, As=None):
        self.typ, self.M = typ, M
        if h is None:
            self.q = lib().orc_firpfbch_create_kaiser(typ, M, m, As)
        else:
            h = np.ascontiguousarray(h, np.float32)
            self.q = lib().orc_firpfbch_create(typ, M, p, ptr(h))

    def execute(self, x):
        x = _arr(x, CRCF)
        y = np.zeros(self.M, np.complex64)
        fn = "orc_firpfbch_analyzer_execute" if self.typ == ANALYZER else "orc_firpfbch_synthesizer_execute"
        getattr(lib(), fn)(self.q, ptr(x), ptr(y))
        return y


class FirPfbch2(_Obj):
    _destroy = "orc_firpfbch2_destroy"

    def __init__(self, typ, M, m, As=None, h=None):
        self.typ, self.M, self.m = typ, M, m
        if h is None:
            self.q = lib().orc_firpfbch2_create_kaiser(typ, M, m, As)
        else:
            h = np.ascontiguousarray(h, np.float32)
            self.q = lib().orc_firpfbch2_create(typ, M, m, ptr(h))

    def reset(self):
        lib().orc_firpfbch2_reset(self.q)

    def execute(self, x):
        x = _arr(x, CRCF)
        out = self.M if self.typ == ANALYZER else self.M // 2
        y = np.zeros(out, np.complex64)
        lib().orc_firpfbch2_execute(self.q, ptr(x), ptr(y))
        return y

    def execute_block(self, x):
        x = _arr(x, CRCF)
        step = self.M // 2 if self.typ == ANALYZER else self.M
        out = self.M if self.typ == ANALYZER else self.M // 2
        nb = len(x) // step
        y = np.zeros(nb * out, np.complex64)
        lib().orc_firpfbch2_execute_block(self.q, ptr(x), nb, ptr(y))
        return y


class Spgram(_Obj):
    """spgram.c:41-286; real_in: spgramf"""
    _destroy = "orc_spgram_destroy"

    def __init__(self, nfft, window, real_in=False):
        self.nfft, self.real_in = nfft, real_in
        w = np.ascontiguousarray(window, np.float32)
        self.q = lib().orc_spgram_create(int(real_in), nfft, ptr(w), len(w))

    def _x(self, x):
        return np.ascontiguousarray(x, np.float32 if self.real_in else np.complex64)

    def write(self, x):
        x = self._x(x)
        lib().orc_spgram_write(self.q, ptr(x), len(x))

    def execute(self):
        X = np.zeros(self.nfft, np.complex64)
        lib().orc_spgram_execute(self.q, ptr(X))
        return X

    def execute_psd(self):
        X = np.zeros(self.nfft, np.float32)
        lib().orc_spgram_execute_psd(self.q, ptr(X))
        return X

    def accumulate_psd(self, x, alpha):
        x = self._x(x)
        lib().orc_spgram_accumulate_psd(self.q, ptr(x), alpha, len(x))

    def write_accumulation(self):
        X = np.zeros(self.nfft, np.float32)
        lib().orc_spgram_write_accumulation(self.q, ptr(X))
        return X

    def estimate_psd(self, x):
        x = self._x(x)
        X = np.zeros(self.nfft, np.float32)
        lib().orc_spgram_estimate_psd(self.q, ptr(x), len(x), ptr(X))
        return X
