"""ctypes mirror of the liquid_mi355x C-ABI (include/liquid_mi355x.h).

This is the host-side Python view of the drop-in library used by the test
suite and bench.py.  Object names, argument meaning and error behaviour follow
liquid-dsp's liquid.h (firfilt_crcf_create / _execute_block / _destroy ...);
the library itself is C + HIP and runs every sample on the GPU.  Loading the
library never touches the GPU; the first object constructor does, and exits
with a message if no HIP device exists (no CPU fallback).

When torch is imported in the same process, import it BEFORE this module so
that the library binds torch's HIP runtime (one runtime per process).
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# LQ_LIB_PATH: an alternative build of the same library (dev/ab/ab.sh A/B runs)
LIB_PATH = os.environ.get("LQ_LIB_PATH") or os.path.join(HERE, "lib", "libliquid_mi355x.so")
HEADER = os.path.join(ROOT, "include", "liquid_mi355x.h")

LIQUID_ANALYZER, LIQUID_SYNTHESIZER = 0, 1
RRRF, CRCF, CCCF = "rrrf", "crcf", "cccf"

_lib = None


class cfloat(C.Structure):
    """liquid_float_complex passed by value (two packed floats)."""
    _fields_ = [("re", C.c_float), ("im", C.c_float)]


def build():
    subprocess.check_call(["make", "-s", "-j8", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def set_small_calls(host):
    """Small-call mode (include/liquid_mi355x.h): True computes single-sample
    calls on the host (host/lq_small.c), False (the default) on the GPU."""
    lib().liquid_mi355x_set_small_calls(1 if host else 0)


def get_small_calls():
    return bool(lib().liquid_mi355x_get_small_calls())


def header_functions():
    """Every function the public header declares (macros expanded by cpp)."""
    out = subprocess.check_output(["gcc", "-E", "-P", "-I", os.path.join(ROOT, "include"), HEADER],
                                  text=True)
    names = set()
    for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", out):
        name = m.group(1)
        if name in ("if", "while", "for", "sizeof", "return") or name.startswith("__"):
            continue
        names.add(name)
    # drop typedef'd struct tags and type names that precede '('
    return sorted(n for n in names if not n.endswith("_s") and n not in ("_Complex",))


vp, u, f, i, ull = C.c_void_p, C.c_uint, C.c_float, C.c_int, C.c_ulonglong
FIRDES_DESIGNS = ("rcos", "rrcos", "rkaiser", "arkaiser", "hM3", "gmsktx", "gmskrx", "fexp", "rfexp", "fsech",
                  "rfsech", "farcsech", "rfarcsech")


def _declare(L):
    sig = {}
    for t in (RRRF, CRCF, CCCF):
        tc = cfloat if t == CCCF else f
        sig.update({
            "dotprod_%s_run" % t: (None, [vp, vp, u, vp]),
            "dotprod_%s_run4" % t: (None, [vp, vp, u, vp]),
            "dotprod_%s_create" % t: (vp, [vp, u]),
            "dotprod_%s_recreate" % t: (vp, [vp, vp, u]),
            "dotprod_%s_destroy" % t: (None, [vp]),
            "dotprod_%s_print" % t: (None, [vp]),
            "dotprod_%s_execute" % t: (None, [vp, vp, vp]),
            "dotprod_%s_execute_batch" % t: (None, [vp, vp, ull, vp]),
            "dotprod_%s_execute_batch_dev" % t: (None, [vp, vp, ull, vp]),
            "dotprod_%s_set_stream" % t: (None, [vp, vp]),
            "dotprod_%s_get_stream" % t: (vp, [vp]),
            "firfilt_%s_create" % t: (vp, [vp, u]),
            "firfilt_%s_create_kaiser" % t: (vp, [u, f, f, f]),
            "firfilt_%s_create_rect" % t: (vp, [u]),
            "firfilt_%s_recreate" % t: (vp, [vp, vp, u]),
            "firfilt_%s_destroy" % t: (None, [vp]),
            "firfilt_%s_reset" % t: (None, [vp]),
            "firfilt_%s_print" % t: (None, [vp]),
            "firfilt_%s_set_scale" % t: (None, [vp, tc]),
            "firfilt_%s_push" % t: (None, [vp, f if t == RRRF else cfloat]),
            "firfilt_%s_execute" % t: (None, [vp, vp]),
            "firfilt_%s_execute_block" % t: (None, [vp, vp, u, vp]),
            "firfilt_%s_get_length" % t: (u, [vp]),
            "firfilt_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp]),
            "firfilt_%s_set_stream" % t: (None, [vp, vp]),
            "firfilt_%s_get_stream" % t: (vp, [vp]),
            "firfilt_%s_synchronize" % t: (None, [vp]),
        })
    for t in (RRRF, CRCF, CCCF):
        ti = f if t == RRRF else cfloat          # sample passed by value
        tc = cfloat if t == CCCF else f          # coefficient / scale by value
        sig.update({
            "firfilt_%s_freqresponse" % t: (None, [vp, f, vp]),
            "firfilt_%s_groupdelay" % t: (f, [vp, f]),
            "firdecim_%s_create" % t: (vp, [u, vp, u]),
            "firdecim_%s_create_kaiser" % t: (vp, [u, u, f]),
            "firdecim_%s_destroy" % t: (None, [vp]),
            "firdecim_%s_print" % t: (None, [vp]),
            "firdecim_%s_clear" % t: (None, [vp]),
            "firdecim_%s_execute" % t: (None, [vp, vp, vp]),
            "firdecim_%s_execute_block" % t: (None, [vp, vp, u, vp]),
            "firdecim_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp]),
            "firdecim_%s_set_stream" % t: (None, [vp, vp]),
            "firinterp_%s_create" % t: (vp, [u, vp, u]),
            "firinterp_%s_create_kaiser" % t: (vp, [u, u, f]),
            "firinterp_%s_destroy" % t: (None, [vp]),
            "firinterp_%s_print" % t: (None, [vp]),
            "firinterp_%s_reset" % t: (None, [vp]),
            "firinterp_%s_execute" % t: (None, [vp, ti, vp]),
            "firinterp_%s_execute_block" % t: (None, [vp, vp, u, vp]),
            "firinterp_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp]),
            "firinterp_%s_set_stream" % t: (None, [vp, vp]),
            "resamp_%s_create" % t: (vp, [f, u, f, f, u]),
            "resamp_%s_create_default" % t: (vp, [f]),
            "resamp_%s_destroy" % t: (None, [vp]),
            "resamp_%s_print" % t: (None, [vp]),
            "resamp_%s_reset" % t: (None, [vp]),
            "resamp_%s_get_delay" % t: (u, [vp]),
            "resamp_%s_set_rate" % t: (None, [vp, f]),
            "resamp_%s_adjust_rate" % t: (None, [vp, f]),
            "resamp_%s_execute" % t: (None, [vp, ti, vp, vp]),
            "resamp_%s_execute_block" % t: (None, [vp, vp, u, vp, vp]),
            "resamp_%s_num_output" % t: (ull, [vp, ull]),
            "resamp_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp, vp]),
            "resamp_%s_set_stream" % t: (None, [vp, vp]),
            "resamp_%s_synchronize" % t: (None, [vp]),
            "fftfilt_%s_create" % t: (vp, [vp, u, u]),
            "fftfilt_%s_destroy" % t: (None, [vp]),
            "fftfilt_%s_reset" % t: (None, [vp]),
            "fftfilt_%s_print" % t: (None, [vp]),
            "fftfilt_%s_set_scale" % t: (None, [vp, tc]),
            "fftfilt_%s_execute" % t: (None, [vp, vp, vp]),
            "fftfilt_%s_get_length" % t: (u, [vp]),
            "fftfilt_%s_execute_block" % t: (None, [vp, vp, ull, vp]),
            "fftfilt_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp]),
            "fftfilt_%s_set_stream" % t: (None, [vp, vp]),
            "firpfb_%s_create" % t: (vp, [u, vp, u]),
            "firpfb_%s_create_kaiser" % t: (vp, [u, u, f, f]),
            "firpfb_%s_recreate" % t: (vp, [vp, u, vp, u]),
            "firpfb_%s_destroy" % t: (None, [vp]),
            "firpfb_%s_print" % t: (None, [vp]),
            "firpfb_%s_set_scale" % t: (None, [vp, tc]),
            "firpfb_%s_reset" % t: (None, [vp]),
            "firpfb_%s_push" % t: (None, [vp, ti]),
            "firpfb_%s_execute" % t: (None, [vp, u, vp]),
            "firpfb_%s_execute_block" % t: (None, [vp, vp, ull, vp]),
            "firpfb_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp]),
            "firpfb_%s_set_stream" % t: (None, [vp, vp]),
            "firpfb_%s_create_rnyquist" % t: (vp, [i, u, u, u, f]),
            "firpfb_%s_create_drnyquist" % t: (vp, [i, u, u, u, f]),
            "firfilt_%s_create_rnyquist" % t: (vp, [i, u, u, f, f]),
            "firdecim_%s_create_prototype" % t: (vp, [i, u, u, f, f]),
            "firinterp_%s_create_prototype" % t: (vp, [i, u, u, f, f]),
        })
    for t in (RRRF, CRCF, CCCF):
        ti = f if t == RRRF else cfloat
        sig.update({
            "resamp2_%s_create" % t: (vp, [u, f, f]),
            "resamp2_%s_recreate" % t: (vp, [vp, u, f, f]),
            "resamp2_%s_destroy" % t: (None, [vp]),
            "resamp2_%s_print" % t: (None, [vp]),
            "resamp2_%s_clear" % t: (None, [vp]),
            "resamp2_%s_get_delay" % t: (u, [vp]),
            "resamp2_%s_filter_execute" % t: (None, [vp, ti, vp, vp]),
            "resamp2_%s_analyzer_execute" % t: (None, [vp, vp, vp]),
            "resamp2_%s_synthesizer_execute" % t: (None, [vp, vp, vp]),
            "resamp2_%s_decim_execute" % t: (None, [vp, vp, vp]),
            "resamp2_%s_interp_execute" % t: (None, [vp, ti, vp]),
            "resamp2_%s_execute_block" % t: (None, [vp, i, vp, ull, vp, vp]),
            "resamp2_%s_execute_block_dev" % t: (None, [vp, i, vp, ull, vp, vp]),
            "resamp2_%s_set_stream" % t: (None, [vp, vp]),
            "resamp2_%s_synchronize" % t: (None, [vp]),
            "msresamp2_%s_create" % t: (vp, [i, u, f, f, f]),
            "msresamp2_%s_destroy" % t: (None, [vp]),
            "msresamp2_%s_print" % t: (None, [vp]),
            "msresamp2_%s_reset" % t: (None, [vp]),
            "msresamp2_%s_get_delay" % t: (f, [vp]),
            "msresamp2_%s_execute" % t: (None, [vp, vp, vp]),
            "msresamp2_%s_execute_block" % t: (None, [vp, vp, ull, vp]),
            "msresamp2_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp]),
            "msresamp2_%s_set_stream" % t: (None, [vp, vp]),
            "msresamp2_%s_synchronize" % t: (None, [vp]),
            "msresamp_%s_create" % t: (vp, [f, f]),
            "msresamp_%s_destroy" % t: (None, [vp]),
            "msresamp_%s_print" % t: (None, [vp]),
            "msresamp_%s_reset" % t: (None, [vp]),
            "msresamp_%s_get_delay" % t: (f, [vp]),
            "msresamp_%s_execute" % t: (None, [vp, vp, u, vp, vp]),
            "msresamp_%s_num_output" % t: (ull, [vp, ull]),
            "msresamp_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp, vp]),
            "msresamp_%s_set_stream" % t: (None, [vp, vp]),
            "msresamp_%s_synchronize" % t: (None, [vp]),
        })
    for t, ti in (("spgramcf", cfloat), ("spgramf", f)):
        sig.update({
            t + "_create": (vp, [u, vp, u]),
            t + "_create_kaiser": (vp, [u, u, f]),
            t + "_create_default": (vp, [u]),
            t + "_destroy": (None, [vp]),
            t + "_reset": (None, [vp]),
            t + "_push": (None, [vp, ti]),
            t + "_write": (None, [vp, vp, u]),
            t + "_execute": (None, [vp, vp]),
            t + "_execute_psd": (None, [vp, vp]),
            t + "_accumulate_psd": (None, [vp, vp, f, u]),
            t + "_write_accumulation": (None, [vp, vp]),
            t + "_estimate_psd": (None, [vp, vp, u, vp]),
            t + "_accumulate_psd_dev": (None, [vp, vp, f, ull]),
            t + "_estimate_psd_dev": (None, [vp, vp, ull, vp]),
            t + "_set_stream": (None, [vp, vp]),
            t + "_synchronize": (None, [vp]),
        })
    for t in (CRCF, CCCF):
        sig.update({
            "firpfbch_%s_create" % t: (vp, [i, u, u, vp]),
            "firpfbch_%s_create_kaiser" % t: (vp, [i, u, u, f]),
            "firpfbch_%s_create_rnyquist" % t: (vp, [i, u, u, f, i]),
            "firpfbch_%s_destroy" % t: (None, [vp]),
            "firpfbch_%s_reset" % t: (None, [vp]),
            "firpfbch_%s_print" % t: (None, [vp]),
            "firpfbch_%s_analyzer_execute" % t: (None, [vp, vp, vp]),
            "firpfbch_%s_synthesizer_execute" % t: (None, [vp, vp, vp]),
            "firpfbch_%s_execute_block" % t: (None, [vp, vp, ull, vp]),
            "firpfbch_%s_execute_block_dev" % t: (None, [vp, vp, ull, vp]),
            "firpfbch_%s_set_stream" % t: (None, [vp, vp]),
        })
    for d in FIRDES_DESIGNS:
        sig["liquid_firdes_" + d] = (None, [u, u, f, f, vp])
    sig.update({
        "liquid_firdes_kaiser": (None, [u, f, f, f, vp]),
        "kaiser_beta_As": (f, [f]),
        "liquid_libversion_number": (i, []),
        "liquid_mi355x_malloc": (vp, [ull]),
        "liquid_mi355x_free": (None, [vp]),
        "liquid_mi355x_memcpy_h2d": (None, [vp, vp, ull]),
        "liquid_mi355x_memcpy_d2h": (None, [vp, vp, ull]),
        "liquid_mi355x_device_synchronize": (None, []),
        "kaiser": (f, [u, u, f, f]),
        "hann": (f, [u, u]),
        "blackmanharris": (f, [u, u]),
        "liquid_rcostaper_windowf": (f, [u, u, u]),
        "liquid_kbd": (f, [u, u, f]),
        "liquid_kbd_window": (None, [u, f, vp]),
        "fft_create_plan": (vp, [u, vp, vp, i, i]),
        "fft_create_plan_r2r_1d": (vp, [u, vp, vp, i, i]),
        "fft_destroy_plan": (None, [vp]),
        "fft_print_plan": (None, [vp]),
        "fft_execute": (None, [vp]),
        "fft_run": (None, [u, vp, vp, i, i]),
        "fft_r2r_1d_run": (None, [u, vp, vp, i, i]),
        "fft_shift": (None, [vp, u]),
        "liquid_nextpow2": (u, [u]),
        "fft_execute_batch": (None, [vp, vp, vp, ull]),
        "fft_execute_batch_dev": (None, [vp, vp, vp, ull]),
        "fft_set_stream": (None, [vp, vp]),
        "liquid_firdes_prototype": (None, [i, u, u, f, f, vp]),
        "liquid_getopt_str2firfilt": (i, [C.c_char_p]),
        "estimate_req_filter_len": (u, [f, f]),
        "estimate_req_filter_As": (f, [f, u]),
        "estimate_req_filter_df": (f, [f, u]),
        "rkaiser_approximate_rho": (f, [u, f]),
        "firdespm_run": (None, [u, u, vp, vp, vp, vp, i, vp]),
        "liquid_filter_autocorr": (f, [vp, u, i]),
        "liquid_filter_isi": (None, [vp, u, u, vp, vp]),
        "liquid_Qf": (f, [f]),
        "firpfbch2_crcf_create": (vp, [i, u, u, vp]),
        "firpfbch2_crcf_create_kaiser": (vp, [i, u, u, f]),
        "firpfbch2_crcf_destroy": (None, [vp]),
        "firpfbch2_crcf_reset": (None, [vp]),
        "firpfbch2_crcf_execute": (None, [vp, vp, vp]),
        "firpfbch2_crcf_execute_block": (None, [vp, vp, ull, vp]),
        "firpfbch2_crcf_execute_block_dev": (None, [vp, vp, ull, vp]),
        "firpfbch2_crcf_set_stream": (None, [vp, vp]),
        "firpfbch2_crcf_get_stream": (vp, [vp]),
        "firpfbch2_crcf_synchronize": (None, [vp]),
    })
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


# ------------------------------------------------------------------ filter design (liquid.h:1413-1668)
FIRFILT_TYPES = ["kaiser", "pm", "rcos", "fexp", "fsech", "farcsech", "arkaiser", "rkaiser", "rrc", "hM3",
                 "gmsktx", "gmskrx", "rfexp", "rfsech", "rfarcsech"]
LIQUID_FIRFILT = {n: k + 1 for k, n in enumerate(FIRFILT_TYPES)}


def firdes_prototype(ftype, k, m, beta, dt=0.0):
    """liquid_firdes_prototype: 2km+1 taps (ftype: name or LIQUID_FIRFILT_* code)."""
    code = LIQUID_FIRFILT[ftype] if isinstance(ftype, str) else int(ftype)
    h = np.zeros(2 * k * m + 1, np.float32)
    lib().liquid_firdes_prototype(code, k, m, beta, dt, ptr(h))
    return h


def firdes(design, k, m, beta, dt=0.0):
    """liquid_firdes_<design>(k, m, beta, dt): e.g. design = "rkaiser", "rcos", "gmskrx"."""
    h = np.zeros(2 * k * m + 1, np.float32)
    getattr(lib(), "liquid_firdes_" + design)(k, m, beta, dt, ptr(h))
    return h


def firdespm(n, bands, des, weights=None, wtype=None):
    """firdespm_run, band-pass designs."""
    bands = np.ascontiguousarray(bands, np.float32)
    des = np.ascontiguousarray(des, np.float32)
    w = None if weights is None else np.ascontiguousarray(weights, np.float32)
    wt = None if wtype is None else np.ascontiguousarray(wtype, np.int32)
    h = np.zeros(n, np.float32)
    lib().firdespm_run(n, len(des), ptr(bands), ptr(des), None if w is None else ptr(w),
                       None if wt is None else ptr(wt), 0, ptr(h))
    return h


def filter_isi(h, k, m):
    h = np.ascontiguousarray(h, np.float32)
    rms, mx = C.c_float(), C.c_float()
    lib().liquid_filter_isi(ptr(h), k, m, C.byref(rms), C.byref(mx))
    return rms.value, mx.value


def _samples(x, t):
    return np.ascontiguousarray(x, dtype=np.float32 if t == RRRF else np.complex64)


def _coefs(h, t):
    return np.ascontiguousarray(h, dtype=np.complex64 if t == CCCF else np.float32)


# ------------------------------------------------------------------ device buffers
class DeviceBuffer:
    """Device allocation made through the library (liquid_mi355x_malloc)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.p = lib().liquid_mi355x_malloc(self.nbytes)

    @classmethod
    def from_array(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        lib().liquid_mi355x_memcpy_h2d(b.p, ptr(a), a.nbytes)
        return b

    def to_array(self, dtype, count):
        a = np.empty(count, dtype)
        lib().liquid_mi355x_memcpy_d2h(ptr(a), self.p, a.nbytes)
        return a

    def free(self):
        if self.p:
            lib().liquid_mi355x_free(self.p)
            self.p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def firdes_kaiser(n, fc, As, mu=0.0):
    h = np.zeros(n, np.float32)
    lib().liquid_firdes_kaiser(n, fc, As, mu, ptr(h))
    return h


# ------------------------------------------------------------------ objects
class _Obj:
    prefix = None

    def _fn(self, name):
        return getattr(lib(), self.prefix + name)

    def destroy(self):
        if getattr(self, "q", None):
            self._fn("_destroy")(self.q)
            self.q = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    def set_stream(self, s):
        self._fn("_set_stream")(self.q, s)

    @classmethod
    def construct(cls, ctor, args, t=CRCF, **attrs):
        """Object from another constructor of the family, e.g.
        FirFilt.construct("_create_rnyquist", (type, k, m, beta, mu), t=CRCF)."""
        o = cls.__new__(cls)
        o.t = t
        o.prefix = cls.family % t
        o.__dict__.update(attrs)
        o.q = getattr(lib(), o.prefix + ctor)(*args)
        if not o.q:
            raise RuntimeError(o.prefix + ctor + " failed")
        return o


class FirFilt(_Obj):
    family = "firfilt_%s"

    def freqresponse(self, fc):
        H = cfloat(0.0, 0.0)
        self._fn("_freqresponse")(self.q, fc, C.byref(H))
        return complex(H.re, H.im) if hasattr(H, "re") else complex(H.real, H.imag)

    def groupdelay(self, fc):
        return float(self._fn("_groupdelay")(self.q, fc))

    def __init__(self, t, h=None, kaiser=None):
        self.t = t
        self.prefix = "firfilt_%s" % t
        if kaiser is not None:
            self.q = self._fn("_create_kaiser")(*kaiser)
        else:
            self._h = _coefs(h, t)
            self.q = self._fn("_create")(ptr(self._h), len(self._h))

    def set_scale(self, s):
        if self.t == CCCF:
            s = complex(s)
            self._fn("_set_scale")(self.q, cfloat(s.real, s.imag))
        else:
            self._fn("_set_scale")(self.q, float(s))

    def reset(self):
        self._fn("_reset")(self.q)

    def push(self, v):
        if self.t == RRRF:
            self._fn("_push")(self.q, float(v))
        else:
            v = complex(v)
            self._fn("_push")(self.q, cfloat(v.real, v.imag))

    def execute(self):
        y = _samples([0], self.t)
        self._fn("_execute")(self.q, ptr(y))
        return y[0]

    def execute_block(self, x):
        x = _samples(x, self.t)
        y = np.zeros_like(x)
        self._fn("_execute_block")(self.q, ptr(x), len(x), ptr(y))
        return y

    def execute_block_dev(self, dx, n, dy):
        self._fn("_execute_block_dev")(self.q, dx, n, dy)

    def synchronize(self):
        self._fn("_synchronize")(self.q)

    def get_length(self):
        return self._fn("_get_length")(self.q)


class DotProd(_Obj):
    def __init__(self, t, h):
        self.t = t
        self.prefix = "dotprod_%s" % t
        self._h = _coefs(h, t)
        self.n = len(self._h)
        self.q = self._fn("_create")(ptr(self._h), self.n)

    def execute(self, x):
        x = _samples(x, self.t)
        y = _samples([0], self.t)
        self._fn("_execute")(self.q, ptr(x), ptr(y))
        return y[0]

    def execute_batch(self, X):
        X = _samples(X, self.t)
        nvec = X.size // self.n
        Y = np.zeros(nvec, X.dtype)
        self._fn("_execute_batch")(self.q, ptr(X), nvec, ptr(Y))
        return Y

    def execute_batch_dev(self, dX, nvec, dY):
        self._fn("_execute_batch_dev")(self.q, dX, nvec, dY)


def dotprod_run(t, h, x):
    h = _coefs(h, t)
    x = _samples(x, t)
    y = _samples([0], t)
    getattr(lib(), "dotprod_%s_run" % t)(ptr(h), ptr(x), len(h), ptr(y))
    return y[0]


def _by_value(v, t):
    if t == RRRF:
        return float(np.real(v))
    v = complex(v)
    return cfloat(v.real, v.imag)


def _out_dtype(t):
    return np.float32 if t == RRRF else np.complex64


class FirDecim(_Obj):
    family = "firdecim_%s"

    def __init__(self, M, h=None, m=None, As=None, t=CRCF):
        self.M, self.t = M, t
        self.prefix = "firdecim_%s" % t
        if h is None:
            self.q = self._fn("_create_kaiser")(M, m, As)
        else:
            self._h = _coefs(h, t)
            self.q = self._fn("_create")(M, ptr(self._h), len(self._h))

    def execute_block(self, x):
        x = _samples(x, self.t)
        n = len(x) // self.M
        y = np.zeros(n, _out_dtype(self.t))
        self._fn("_execute_block")(self.q, ptr(x), n, ptr(y))
        return y

    def execute(self, x):
        x = _samples(x, self.t)
        y = np.zeros(1, _out_dtype(self.t))
        self._fn("_execute")(self.q, ptr(x), ptr(y))
        return y[0]

    def clear(self):
        self._fn("_clear")(self.q)


class FirInterp(_Obj):
    family = "firinterp_%s"

    def __init__(self, M, h=None, m=None, As=None, t=CRCF):
        self.M, self.t = M, t
        self.prefix = "firinterp_%s" % t
        if h is None:
            self.q = self._fn("_create_kaiser")(M, m, As)
        else:
            self._h = _coefs(h, t)
            self.q = self._fn("_create")(M, ptr(self._h), len(self._h))

    def execute_block(self, x):
        x = _samples(x, self.t)
        y = np.zeros(len(x) * self.M, _out_dtype(self.t))
        self._fn("_execute_block")(self.q, ptr(x), len(x), ptr(y))
        return y

    def execute(self, v):
        y = np.zeros(self.M, _out_dtype(self.t))
        self._fn("_execute")(self.q, _by_value(v, self.t), ptr(y))
        return y

    def reset(self):
        self._fn("_reset")(self.q)


class FftFilt(_Obj):
    family = "fftfilt_%s"

    def __init__(self, h, n, t=CRCF):
        self.n, self.t = n, t
        self.prefix = "fftfilt_%s" % t
        self._h = _coefs(h, t)
        self.q = self._fn("_create")(ptr(self._h), len(self._h), n)

    def set_scale(self, s):
        self._fn("_set_scale")(self.q, _by_value(s, CCCF) if self.t == CCCF else float(np.real(s)))

    def reset(self):
        self._fn("_reset")(self.q)

    def execute(self, x):
        x = _samples(x, self.t)
        assert len(x) == self.n
        y = np.zeros_like(x)
        self._fn("_execute")(self.q, ptr(x), ptr(y))
        return y

    def execute_block(self, x):
        x = _samples(x, self.t)
        y = np.zeros_like(x)
        self._fn("_execute_block")(self.q, ptr(x), len(x), ptr(y))
        return y

    def execute_block_dev(self, dx, n, dy):
        self._fn("_execute_block_dev")(self.q, dx, n, dy)


class FirPfbch(_Obj):
    family = "firpfbch_%s"

    def __init__(self, typ, M, p=None, h=None, m=None, As=None, t=CRCF, rnyquist=None):
        self.typ, self.M, self.t = typ, M, t
        self.prefix = self.family % t
        if rnyquist is not None:               # (m, beta, ftype)
            self.q = self._fn("_create_rnyquist")(typ, M, rnyquist[0], rnyquist[1], rnyquist[2])
        elif h is None:
            self.q = self._fn("_create_kaiser")(typ, M, m, As)
        else:
            self._h = _coefs(h, t)
            self.q = self._fn("_create")(typ, M, p, ptr(self._h))

    def execute(self, x):
        x = _samples(x, CRCF)
        y = np.zeros(self.M, np.complex64)
        fn = "_analyzer_execute" if self.typ == LIQUID_ANALYZER else "_synthesizer_execute"
        self._fn(fn)(self.q, ptr(x), ptr(y))
        return y

    def execute_block(self, x):
        x = _samples(x, CRCF)
        nb = len(x) // self.M
        y = np.zeros(nb * self.M, np.complex64)
        self._fn("_execute_block")(self.q, ptr(x), nb, ptr(y))
        return y


class FirPfbch2(_Obj):
    prefix = "firpfbch2_crcf"

    def __init__(self, typ, M, m, As=None, h=None):
        self.typ, self.M, self.m = typ, M, m
        if h is None:
            self.q = self._fn("_create_kaiser")(typ, M, m, As)
        else:
            self._h = _coefs(h, CRCF)
            self.q = self._fn("_create")(typ, M, m, ptr(self._h))
        self.nin = M // 2 if typ == LIQUID_ANALYZER else M
        self.nout = M if typ == LIQUID_ANALYZER else M // 2

    def reset(self):
        self._fn("_reset")(self.q)

    def execute(self, x):
        x = _samples(x, CRCF)
        y = np.zeros(self.nout, np.complex64)
        self._fn("_execute")(self.q, ptr(x), ptr(y))
        return y

    def execute_block(self, x):
        x = _samples(x, CRCF)
        nb = len(x) // self.nin
        y = np.zeros(nb * self.nout, np.complex64)
        self._fn("_execute_block")(self.q, ptr(x), nb, ptr(y))
        return y

    def execute_block_dev(self, dx, nblocks, dy):
        self._fn("_execute_block_dev")(self.q, dx, nblocks, dy)

    def synchronize(self):
        self._fn("_synchronize")(self.q)

    def get_stream(self):
        return self._fn("_get_stream")(self.q)


class FirPfb(_Obj):
    family = "firpfb_%s"

    def __init__(self, M, h=None, m=None, fc=None, As=None, t=CRCF):
        self.M, self.t = M, t
        self.prefix = "firpfb_%s" % t
        if h is None:
            self.q = self._fn("_create_kaiser")(M, m, fc, As)
        else:
            self._h = _coefs(h, t)
            self.q = self._fn("_create")(M, ptr(self._h), len(self._h))

    def set_scale(self, s):
        self._fn("_set_scale")(self.q, _by_value(s, CCCF) if self.t == CCCF else float(np.real(s)))

    def reset(self):
        self._fn("_reset")(self.q)

    def push(self, v):
        self._fn("_push")(self.q, _by_value(v, self.t))

    def execute(self, i):
        y = np.zeros(1, _out_dtype(self.t))
        self._fn("_execute")(self.q, i, ptr(y))
        return y[0]

    def execute_block(self, x):
        """push each x[t] and evaluate every bank: returns (len(x), M)"""
        x = _samples(x, self.t)
        y = np.zeros(len(x) * self.M, _out_dtype(self.t))
        self._fn("_execute_block")(self.q, ptr(x), len(x), ptr(y))
        return y.reshape(len(x), self.M)


class Resamp(_Obj):
    family = "resamp_%s"

    def __init__(self, rate, m=None, fc=None, As=None, npfb=None, t=CRCF):
        self.t = t
        self.prefix = "resamp_%s" % t
        if m is None:
            self.q = self._fn("_create_default")(rate)
        else:
            self.q = self._fn("_create")(rate, m, fc, As, npfb)

    def reset(self):
        self._fn("_reset")(self.q)

    def set_rate(self, r):
        self._fn("_set_rate")(self.q, float(r))

    def adjust_rate(self, d):
        self._fn("_adjust_rate")(self.q, float(d))

    def get_delay(self):
        return self._fn("_get_delay")(self.q)

    def num_output(self, nx):
        return int(self._fn("_num_output")(self.q, nx))

    def execute(self, v):
        y = np.zeros(max(1, self.num_output(1)), _out_dtype(self.t))
        nw = C.c_uint(0)
        self._fn("_execute")(self.q, _by_value(v, self.t), ptr(y), C.byref(nw))
        return y[:nw.value].copy()

    def execute_block(self, x):
        x = _samples(x, self.t)
        y = np.zeros(max(1, self.num_output(len(x))), _out_dtype(self.t))
        ny = C.c_uint(0)
        self._fn("_execute_block")(self.q, ptr(x), len(x), ptr(y), C.byref(ny))
        return y[:ny.value]

    def execute_block_dev(self, dx, nx, dy):
        ny = C.c_ulonglong(0)
        self._fn("_execute_block_dev")(self.q, dx, nx, dy, C.byref(ny))
        return ny.value

    def synchronize(self):
        self._fn("_synchronize")(self.q)


# ------------------------------------------------------------------ half-band / multi-stage resamplers
RESAMP2_FILTER, RESAMP2_ANALYZER, RESAMP2_SYNTHESIZER, RESAMP2_DECIM, RESAMP2_INTERP = range(5)
LIQUID_RESAMP_INTERP, LIQUID_RESAMP_DECIM = 0, 1


class Resamp2(_Obj):
    family = "resamp2_%s"
    NIN = {0: 1, 1: 2, 2: 2, 3: 2, 4: 1}
    NOUT = {0: 1, 1: 2, 2: 2, 3: 1, 4: 2}

    def __init__(self, m, f0, As, t=CRCF):
        self.t = t
        self.prefix = self.family % t
        self.q = self._fn("_create")(m, f0, As)

    def clear(self):
        self._fn("_clear")(self.q)

    def get_delay(self):
        return self._fn("_get_delay")(self.q)

    def run(self, mode, x):
        """n consecutive calls of one mode (execute_block extension)."""
        x = _samples(x, self.t)
        n = len(x) // self.NIN[mode]
        y0 = np.zeros(n * self.NOUT[mode], _out_dtype(self.t))
        y1 = np.zeros(n, _out_dtype(self.t))
        self._fn("_execute_block")(self.q, mode, ptr(x), n, ptr(y0), ptr(y1))
        return (y0, y1) if mode == RESAMP2_FILTER else y0

    def call(self, mode, x):
        """one call of the original per-call API"""
        if mode == RESAMP2_FILTER:
            y0, y1 = np.zeros(1, _out_dtype(self.t)), np.zeros(1, _out_dtype(self.t))
            self._fn("_filter_execute")(self.q, _by_value(x, self.t), ptr(y0), ptr(y1))
            return y0[0], y1[0]
        if mode == RESAMP2_INTERP:
            y = np.zeros(2, _out_dtype(self.t))
            self._fn("_interp_execute")(self.q, _by_value(x, self.t), ptr(y))
            return y
        x = _samples(x, self.t)
        y = np.zeros(self.NOUT[mode], _out_dtype(self.t))
        fn = {RESAMP2_ANALYZER: "_analyzer_execute", RESAMP2_SYNTHESIZER: "_synthesizer_execute",
              RESAMP2_DECIM: "_decim_execute"}[mode]
        self._fn(fn)(self.q, ptr(x), ptr(y))
        return y


class MsResamp2(_Obj):
    family = "msresamp2_%s"

    def __init__(self, typ, ns, fc, f0, As, t=CRCF):
        self.t, self.typ, self.M = t, typ, 1 << ns
        self.prefix = self.family % t
        self.q = self._fn("_create")(typ, ns, fc, f0, As)

    def execute_block(self, x):
        x = _samples(x, self.t)
        n = len(x) if self.typ == LIQUID_RESAMP_INTERP else len(x) // self.M
        y = np.zeros(n * self.M if self.typ == LIQUID_RESAMP_INTERP else n, _out_dtype(self.t))
        self._fn("_execute_block")(self.q, ptr(x), n, ptr(y))
        return y

    def execute(self, x):
        x = _samples(x, self.t)
        y = np.zeros(self.M if self.typ == LIQUID_RESAMP_INTERP else 1, _out_dtype(self.t))
        self._fn("_execute")(self.q, ptr(x), ptr(y))
        return y

    def get_delay(self):
        return self._fn("_get_delay")(self.q)


class MsResamp(_Obj):
    family = "msresamp_%s"

    def __init__(self, rate, As, t=CRCF):
        self.t = t
        self.prefix = self.family % t
        self.q = self._fn("_create")(rate, As)

    def reset(self):
        self._fn("_reset")(self.q)

    def num_output(self, nx):
        return int(self._fn("_num_output")(self.q, nx))

    def execute(self, x):
        x = _samples(x, self.t)
        y = np.zeros(max(1, self.num_output(len(x))), _out_dtype(self.t))
        ny = C.c_uint(0)
        self._fn("_execute")(self.q, ptr(x), len(x), ptr(y), C.byref(ny))
        return y[:ny.value]

    def execute_block_dev(self, dx, nx, dy):
        ny = C.c_ulonglong(0)
        self._fn("_execute_block_dev")(self.q, dx, nx, dy, C.byref(ny))
        return ny.value

    def get_delay(self):
        return self._fn("_get_delay")(self.q)

    def synchronize(self):
        self._fn("_synchronize")(self.q)


# ------------------------------------------------------------------ FFT plan API (liquid.h:1113-1216)
def fft_run(x, direction=+1):
    x = np.ascontiguousarray(x, np.complex64)
    y = np.zeros_like(x)
    lib().fft_run(len(x), ptr(x), ptr(y), direction, 0)
    return y


def fft_r2r(x, typ):
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros_like(x)
    lib().fft_r2r_1d_run(len(x), ptr(x), ptr(y), typ, 0)
    return y


def fft_batch(X, direction=+1):
    """fft_execute_batch over the rows of X (host arrays)."""
    X = np.ascontiguousarray(X, np.complex64)
    b, n = X.shape
    Y = np.zeros_like(X)
    p = lib().fft_create_plan(n, None, None, direction, 0)
    try:
        lib().fft_execute_batch(p, ptr(X), ptr(Y), b)
    finally:
        lib().fft_destroy_plan(p)
    return Y


def fft_shift(x):
    x = np.array(x, np.complex64)
    lib().fft_shift(ptr(x), len(x))
    return x



# ------------------------------------------------------------------ spectral periodogram (liquid.h:1220-1290)
class Spgram(_Obj):
    def __init__(self, nfft, window=None, real_in=False, default=False, kaiser=None):
        self.nfft, self.real_in = nfft, real_in
        self.prefix = "spgramf" if real_in else "spgramcf"
        if default:
            self.q = self._fn("_create_default")(nfft)
        elif kaiser is not None:               # (window_len, beta)
            self.q = self._fn("_create_kaiser")(nfft, kaiser[0], kaiser[1])
        else:
            self._w = np.ascontiguousarray(window, np.float32)
            self.q = self._fn("_create")(nfft, ptr(self._w), len(self._w))

    def _x(self, x):
        return np.ascontiguousarray(x, np.float32 if self.real_in else np.complex64)

    def reset(self):
        self._fn("_reset")(self.q)

    def push(self, v):
        self._fn("_push")(self.q, float(np.real(v)) if self.real_in else _by_value(v, CRCF))

    def write(self, x):
        x = self._x(x)
        self._fn("_write")(self.q, ptr(x), len(x))

    def execute(self):
        X = np.zeros(self.nfft, np.complex64)
        self._fn("_execute")(self.q, ptr(X))
        return X

    def execute_psd(self):
        X = np.zeros(self.nfft, np.float32)
        self._fn("_execute_psd")(self.q, ptr(X))
        return X

    def accumulate_psd(self, x, alpha):
        x = self._x(x)
        self._fn("_accumulate_psd")(self.q, ptr(x), alpha, len(x))

    def write_accumulation(self):
        X = np.zeros(self.nfft, np.float32)
        self._fn("_write_accumulation")(self.q, ptr(X))
        return X

    def estimate_psd(self, x):
        x = self._x(x)
        X = np.zeros(self.nfft, np.float32)
        self._fn("_estimate_psd")(self.q, ptr(x), len(x), ptr(X))
        return X
