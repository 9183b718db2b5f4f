"""Loader for the committed golden fixtures (tests/golden/*.json)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)["data"]


def arr(v):
    """JSON list -> float32 (real) or complex64 ([re, im] pairs) array."""
    if isinstance(v, list) and v and isinstance(v[0], list):
        a = np.asarray(v, dtype=np.float64)
        return (a[:, 0] + 1j * a[:, 1]).astype(np.complex64)
    if isinstance(v, list) and len(v) == 2 and isinstance(v[0], float) and False:
        pass
    return np.asarray(v, dtype=np.float32)


def scalar(v):
    if isinstance(v, list):
        return complex(v[0], v[1])
    return float(v)


def nrm_err(y, ref):
    """Normwise error max|y-ref| / max|ref| (the parity metric)."""
    y = np.asarray(y)
    ref = np.asarray(ref)
    den = np.max(np.abs(ref)) if ref.size else 1.0
    return float(np.max(np.abs(y.astype(np.complex128) - ref.astype(np.complex128))) / (den if den > 0 else 1.0)) \
        if ref.size else 0.0


# ------------------------------------------------------------ reference property tests
# (shared by the oracle and GPU suites: the same checks the reference's autotests make)
def liquid_kaiser(n, N, beta, mu=0.0):
    """kaiser(), src/math/src/math.c:289-312 (float64)."""
    from scipy.special import i0
    t = n - (N - 1) / 2.0 + mu
    r = 2.0 * t / N
    return i0(beta * np.sqrt(np.clip(1 - r * r, 0.0, None))) / i0(beta)


def resamp2_analysis_case():
    """src/filter/tests/resamp2_crcf_autotest.c:27-58: two tones through the
    analyzer; returns (x, check(y0, y1) -> max error, tol)."""
    m, n, f0, f1 = 5, 37, 0.0739, -0.1387
    i = np.arange(2 * n + 2 * m + 1)
    x = np.where(i < 2 * n, np.exp(1j * f0 * i) + np.exp(1j * (np.pi + f1) * i), 0).astype(np.complex64)

    def check(y0, y1):
        k = np.arange(m, n - m)
        d0 = y0[k + m] - np.exp(1j * 2 * f0 * (k + 0.5))
        d1 = y1[k + m] - np.exp(1j * 2 * f1 * (k + 0.5))
        return \
            max(np.max(np.abs(d0.real)), np.max(np.abs(d0.imag)), np.max(np.abs(d1.real)),
                np.max(np.abs(d1.imag))), 1e-3
    return m, n, x[:2 * n], check


def resamp2_synthesis_case():
    """src/filter/tests/resamp2_crcf_autotest.c:81-113"""
    m, n, f0, f1 = 5, 37, 0.0739, -0.1387
    i = np.arange(n)
    x = np.empty(2 * n, np.complex64)
    x[0::2] = np.exp(1j * f0 * i)
    x[1::2] = np.exp(1j * f1 * i)

    def check(y):
        k = np.arange(m, n - 2 * m)
        ref = np.exp(1j * 0.5 * f0 * k) + np.exp(1j * (np.pi + 0.5 * f1) * k)
        d = y[k + 2 * m] - ref
        return max(np.max(np.abs(d.real)), np.max(np.abs(d.imag))), 3e-3
    return m, n, x, check


def msresamp_spectral_case():
    """src/filter/tests/msresamp_crcf_autotest.c:25-100: Kaiser-windowed tone at
    0.2 r; returns (r, As, x, check(y) -> list of failed conditions)."""
    m, r, As, n, fx = 13, 0.127115323, 60.0, 1200, 0.0254230646
    nx = n + m
    i = np.arange(nx)
    w = np.where(i < n, liquid_kaiser(i, n, 10.0), 0.0)
    x = (np.exp(1j * 2 * np.pi * fx * i) * w).astype(np.complex64)
    wsum = float(np.sum(w))

    def check(y):
        ny = len(y)
        fy = fx / r
        nfft = 1 << int(np.ceil(np.log2(ny)))
        Y = np.fft.fftshift(np.fft.fft(np.concatenate([y, np.zeros(nfft - ny)])))
        Y = Y / (r * wsum)
        f = np.arange(nfft) / nfft - 0.5
        mag = 20 * np.log10(np.abs(Y) + 1e-30)
        k = int(np.argmax(mag))
        side = np.max(mag[np.abs(f - fy) > 0.07])
        bad = []
        if abs(ny / nx - r) > 0.01: bad.append("rate %g" % (ny / nx))
        if abs(mag[k]) > 0.25: bad.append("peak %g dB" % mag[k])
        if abs(f[k] - fy) > 0.01: bad.append("peak freq %g" % f[k])
        if side >= -As: bad.append("sidelobe %g dB" % side)
        return bad
    return r, As, x, check


def firpfbch2_downconverter(x, h, M, m, nblocks, firfilt, channels=None):
    """The firpfbch2 analyzer restated as a bank of M "traditional" down-
    converters -- the reference's own methodology for pinning a channelizer
    to a filter it already pins: firpfbch_crcf_analyzer_autotest.c:30-146
    (mixer + firfilt, tol 1e-4) and, for firpfbch2 itself,
    sandbox/firpfbch2_analysis_equivalence_test.c:182-215 (mix channel k
    down by e^{-j2pi kt/M}, filter with the prototype, sample after every M/2
    inputs).  Any taps work ("these coefficients can be random", :39-41).

    With h the 2Mm prototype taps (firpfbch2.c:99-109 uses exactly those)
    and t_b = (b+1)M/2 - 1 the last input of block b, the closed form
     gives
        Y_b[k] = (1/M) e^{+j2pi k (offset_b + t_b)/M} y_k[t_b],
        y_k = firfilt(h, x[t] e^{-j2pi kt/M}),  offset_b = (b mod 2) M/2,
    the phase term being the commutator's rotation of the bins.
    `firfilt(h, z)` is the pinned FIR filter to use (complex64 in and out).
    `channels` restricts the bank to a subset of k (the reference loops over
    all of them; any subset is the same identity): returns (nblocks,
    len(channels)) in that order, else (nblocks, M).
    """
    L = 2 * M * m
    ks = list(range(M)) if channels is None else list(channels)
    t = (np.arange(nblocks) + 1) * (M // 2) - 1
    off = (np.arange(nblocks) % 2) * (M // 2)
    n = np.arange(len(x))
    Y = np.zeros((nblocks, len(ks)), np.complex128)
    for c, k in enumerate(ks):
        z = (x.astype(np.complex128) * np.exp(-2j * np.pi * ((k * n) % M) / M)).astype(np.complex64)
        y = np.asarray(firfilt(np.asarray(h[:L], np.float32), z))
        Y[:, c] = np.exp(2j * np.pi * ((k * (off + t)) % M) / M) * y[t] / M
    return Y


def firpfbch_downconverter(x, h, M, nsym, firfilt, channels=None):
    """src/multichannel/tests/firpfbch_crcf_analyzer_autotest.c:88-115: the
    critically sampled analyzer as M "traditional" down-converters -- channel
    k mixed down by e^{-j 2 pi k j / M}, filtered by the full prototype h
    (the pinned `firfilt`), sampled after every M inputs:
        Y1[n][k] = firfilt(h, x[j] e^{-j2pi kj/M})[(n+1) M - 1]
    (the reference compares this with the analyzer output at tol 1e-4,
    no scaling).  The mixer phase is reduced exactly (k j mod M)."""
    ks = list(range(M)) if channels is None else list(channels)
    t = (np.arange(nsym) + 1) * M - 1
    n = np.arange(len(x))
    Y = np.zeros((nsym, len(ks)), np.complex128)
    for c, k in enumerate(ks):
        z = (x.astype(np.complex128) * np.exp(-2j * np.pi * ((k * n) % M) / M)).astype(np.complex64)
        Y[:, c] = np.asarray(firfilt(np.asarray(h, np.float32), z))[t]
    return Y


def resamp_autotest_case():
    """src/filter/tests/resamp_crcf_autotest.c:29-136 (autotest_resamp_crcf),
    restated: r = 1.27115323, m = 13, bw = 0.45, As = 60, npfb = 64, a
    Kaiser-windowed (beta 10) tone at fx = 0.254230646 over n = 400 samples
    plus m zeros, pushed one sample per execute().  Returns (r, m, bw, As,
    npfb, x, check); check(y) lists the failed conditions of :106-109 --
    rate within 0.01, peak 0 +- 0.25 dB, peak at fy = fx / r +- 0.01, every
    bin further than 0.07 from fy below -As."""
    m, r, bw, As, npfb, n, fx = 13, 1.27115323, 0.45, 60.0, 64, 400, 0.254230646
    r32 = float(np.float32(r))
    nx = n + m
    i = np.arange(nx)
    w = np.where(i < n, liquid_kaiser(i, n, 10.0), 0.0).astype(np.float32)
    x = (np.exp(1j * 2 * np.pi * fx * i) * w).astype(np.complex64)
    wsum = float(np.sum(w, dtype=np.float32))

    def check(y):
        y = np.asarray(y, np.complex128)
        ny = len(y)
        r_actual = ny / nx
        fy = fx / r32
        nfft = 1 << int(np.ceil(np.log2(ny)))
        Y = np.fft.fftshift(np.fft.fft(np.concatenate([y, np.zeros(nfft - ny)])))
        Y = Y / (r32 * wsum)
        f = np.arange(nfft) / nfft - 0.5
        mag = 20 * np.log10(np.abs(Y) + 1e-30)
        k = int(np.argmax(mag))
        side = float(np.max(mag[np.abs(f - fy) > 0.07]))
        bad = []
        if abs(r_actual - r32) > 0.01: bad.append("rate %g" % r_actual)
        if abs(mag[k]) > 0.25: bad.append("peak %g dB" % mag[k])
        if abs(f[k] - fy) > 0.01: bad.append("peak freq %g (want %g)" % (f[k], fy))
        if not side < -As: bad.append("sidelobe %g dB" % side)
        return bad
    return r32, m, bw, As, npfb, x, check
