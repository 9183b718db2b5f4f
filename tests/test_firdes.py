"""Prototype filter design (host, create time): liquid_firdes_prototype and the
designs behind the *_create_rnyquist / *_create_prototype constructors.

Pinned by
  * the reference's own golden coefficient arrays (tests/golden/firdes.json,
    extracted by gen_golden.py from src/filter/tests/firdes_autotest.c and
    firdespm_autotest.c, with those tests' tolerances);
  * the reference's rkaiser ISI test (firdes_autotest.c:99-125: < -30 dB);
  * float64 numpy restatements of the closed-form designs (fnyquist.c:41-345
    frequency-sampled flipped-Nyquist families, gmsk.c:37-70 transmit pulse);
  * (root-)Nyquist properties for the iterative designs (rkaiser, hM3, PM).
No GPU: these run in the CPU suite against the built library.
"""
import json
import os

import numpy as np
import pytest
from scipy.special import erfc

import liquidmi as LQ

HERE = os.path.dirname(os.path.abspath(__file__))
FD = json.load(open(os.path.join(HERE, "golden", "firdes.json")))["data"]


@pytest.mark.parametrize("name", sorted(FD))
def test_firdes_golden(name):
    c = FD[name]
    if c["design"] == "firdespm":
        h = LQ.firdespm(c["n"], c["bands"], c["des"], c["weights"])
        ref = np.asarray(c["h"], np.float64)
    else:
        h = LQ.firdes(c["design"], c["k"], c["m"], c["beta"], c["dt"])
        ref = np.zeros(len(h))
        ref[:len(c["h"])] = c["h"]          # the reference's array initialiser may omit a trailing 0
    assert np.max(np.abs(h - ref)) < c["tol"]


def test_rkaiser_isi_reference_case():
    # firdes_autotest.c:99-125
    k, m, beta = 2, 3, 0.3
    h = LQ.firdes("rkaiser", k, m, beta)
    rms, mx = LQ.filter_isi(h, k, m)
    assert 20 * np.log10(mx) < -30 and 20 * np.log10(rms) < -30


@pytest.mark.parametrize("ftype", ["arkaiser", "rkaiser", "rrc", "hM3", "rfexp", "rfsech", "rfarcsech"])
@pytest.mark.parametrize("k,m,beta", [(2, 4, 0.25), (4, 7, 0.5), (8, 3, 0.35)])
def test_root_nyquist_designs(ftype, k, m, beta):
    h = LQ.firdes_prototype(ftype, k, m, beta)
    rms, _ = LQ.filter_isi(h, k, m)
    assert 20 * np.log10(rms) < -35
    assert abs(np.sum(h.astype(np.float64) ** 2) - k) < 0.05 * k     # unit symbol energy (h'h = k)
    assert np.max(np.abs(h - h[::-1])) < 1e-5 * np.max(np.abs(h))      # linear phase


@pytest.mark.parametrize("ftype,tol", [("kaiser", 1e-6), ("rcos", 1e-6), ("pm", 5e-3), ("fexp", 2e-2),
                                        ("fsech", 2e-2), ("farcsech", 2e-2)])
@pytest.mark.parametrize("k,m,beta", [(2, 5, 0.3), (4, 6, 0.5)])
def test_nyquist_designs_zero_crossings(ftype, tol, k, m, beta):
    h = LQ.firdes_prototype(ftype, k, m, beta).astype(np.float64)
    c = k * m
    zc = np.delete(h[c % k::k], c // k)
    assert np.max(np.abs(zc)) < tol * abs(h[c])


def _fnyquist_np(family, root, k, m, beta):
    # fnyquist.c:41-100 and :144-345 in float64
    n = 2 * k * m + 1
    f = np.arange(n) / n
    f = np.abs(np.where(f > 0.5, f - 1.0, f))
    f0, f1, f2 = 0.5 * (1 - beta) / k, 0.5 / k, 0.5 * (1 + beta) / k
    B = 0.5 / k
    H = np.zeros(n)
    H[f < f0] = 1.0
    band = (f > f0) & (f < f2)
    lo, hi = band & (f < f1), band & ~(f < f1)
    if family == "exp":
        g = np.log(2.0) / (beta * B)
        H[lo] = np.exp(g * (B * (1 - beta) - f[lo]))
        H[hi] = 1 - np.exp(g * (f[hi] - (1 + beta) * B))
    elif family == "sech":
        g = np.log(np.sqrt(3.0) + 2.0) / (beta * B)
        H[lo] = 1 / np.cosh(g * (f[lo] - B * (1 - beta)))
        H[hi] = 1 - 1 / np.cosh(g * (B * (1 + beta) - f[hi]))
    else:
        g = np.log(np.sqrt(3.0) + 2.0) / (beta * B)
        z = 1.0 / (2.0 * beta * B)
        asech = lambda v: np.log(np.sqrt(1 / v - 1) * np.sqrt(1 / v + 1) + 1 / v)
        H[lo] = 1 - (z / g) * asech(z * (B * (1 + beta) - f[lo]))
        H[hi] = (z / g) * asech(z * (f[hi] - B * (1 - beta)))
    if root:
        H = np.sqrt(H)
    t = np.fft.ifft(H) * n                      # fft_run(..., LIQUID_FFT_BACKWARD): unnormalised
    return np.real(t[(np.arange(n) + k * m + 1) % n]) * k / n


@pytest.mark.parametrize("design,family,root", [("fexp", "exp", 0), ("rfexp", "exp", 1), ("fsech", "sech", 0),
                                                ("rfsech", "sech", 1), ("farcsech", "arcsech", 0),
                                                ("rfarcsech", "arcsech", 1)])
@pytest.mark.parametrize("k,m,beta", [(2, 3, 0.3), (5, 4, 0.7)])
def test_fnyquist_vs_numpy(design, family, root, k, m, beta):
    h = LQ.firdes(design, k, m, beta)
    ref = _fnyquist_np(family, root, k, m, beta)
    assert np.max(np.abs(h - ref)) < 1e-5 * np.max(np.abs(ref))


@pytest.mark.parametrize("k,m,bt", [(4, 3, 0.3), (2, 5, 0.5)])
def test_gmsktx_vs_numpy(k, m, bt):
    # gmsk.c:37-70: Gaussian-filtered rectangular pulse, area k*pi/2
    t = np.arange(2 * k * m + 1) / k - m
    c0 = 1 / np.sqrt(np.log(2.0))
    Q = lambda z: 0.5 * erfc(z / np.sqrt(2.0))
    ref = Q(2 * np.pi * bt * (t - 0.5) * c0) - Q(2 * np.pi * bt * (t + 0.5) * c0)
    ref *= np.pi / (2 * np.sum(ref)) * k
    h = LQ.firdes("gmsktx", k, m, bt)
    assert np.max(np.abs(h - ref)) < 1e-5 * np.max(np.abs(ref))


def test_gmskrx_equalises_gmsktx():
    # the receive filter flattens the transmit pulse's spectrum in band:
    # the cascade is close to a Nyquist pulse at the symbol instants
    k, m, bt = 4, 5, 0.3
    ht = LQ.firdes("gmsktx", k, m, bt).astype(np.float64)
    hr = LQ.firdes("gmskrx", k, m, bt).astype(np.float64)
    g = np.convolve(ht, hr)
    c = int(np.argmax(np.abs(g)))
    isi = np.delete(g[c % k::k], c // k)
    assert np.max(np.abs(isi)) < 0.1 * abs(g[c])


def test_getopt_and_estimates():
    L = LQ.lib()
    for code, name in enumerate(["kaiser", "pm", "rcos", "fexp", "fsech", "farcsech", "arkaiser", "rkaiser",
                                 "rrcos", "hM3", "gmsktx", "gmskrx", "rfexp", "rfsech", "rfarcsech"], start=1):
        assert L.liquid_getopt_str2firfilt(name.encode()) == code
    assert L.liquid_getopt_str2firfilt(b"nope") == 0
    # firdes.c:52-160: the As/df searches invert the Kaiser length estimate
    for df, N in [(0.05, 64), (0.1, 33), (0.02, 301)]:
        As = L.estimate_req_filter_As(df, N)
        assert abs((As - 7.95) / (14.26 * df) - N) < 0.01 * N
        d2 = L.estimate_req_filter_df(As, N)
        assert abs(d2 - df) < 1e-3 * max(df, 0.01)
    assert L.estimate_req_filter_len(0.1, 60.0) == int((60.0 - 7.95) / (14.26 * 0.1))
    assert abs(L.liquid_Qf(0.0) - 0.5) < 1e-7 and abs(L.liquid_Qf(1.0) - 0.1586553) < 1e-6
