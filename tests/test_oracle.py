"""Pin the CPU oracle (oracle/oracle.c) to the reference's own golden vectors and
property tests.  CPU only; these run in the build container.

Golden data: tests/golden/*.json (extracted from the reference's test files by
tests/golden/gen_golden.py).  Tolerances are the reference's own (written next
to each case in the fixture).  Objects without shipped golden data (firpfbch,
firpfbch2, resamp) are pinned by the reference's own property tests
(src/multichannel/tests/firpfbch_crcf_analyzer_autotest.c,
src/multichannel/tests/firpfbch2_crcf_autotest.c,
src/filter/tests/resamp_crcf_autotest.c) plus float64 numpy restatements of
the closed forms in SURVEY Appendix B.
"""
import numpy as np
import pytest

import golden_io as G
import oracle_lib as O

TYPES = {"rrrf": O.RRRF, "crcf": O.CRCF, "cccf": O.CCCF}


# ----------------------------------------------------------------------------- golden
@pytest.mark.parametrize("case", G.load("firfilt"), ids=lambda c: c["name"])
def test_firfilt_golden(case):
    # runner: src/filter/tests/firfilt_runtest.c:68-95 (push + execute, tol 1e-3)
    typ = TYPES[case["type"]]
    h, x, y = G.arr(case["h"]), G.arr(case["x"]), G.arr(case["y"])
    q = O.FirFilt(typ, h)
    out = []
    for v in x:
        q.push(v)
        out.append(q.execute())
    out = np.asarray(out)
    assert np.max(np.abs(out - y)) < case["tol"]
    q2 = O.FirFilt(typ, h)
    assert np.max(np.abs(q2.execute_block(x) - y)) < case["tol"]


@pytest.mark.parametrize("case", G.load("firdecim"), ids=lambda c: c["name"])
def test_firdecim_golden(case):
    # runner: src/filter/tests/firdecim_runtest.c:78-93
    typ = TYPES[case["type"]]
    h, x, y = G.arr(case["h"]), G.arr(case["x"]), G.arr(case["y"])
    q = O.FirDecim(typ, case["M"], h)
    out = q.execute_block(x[: len(y) * case["M"]])
    assert np.max(np.abs(out - y)) < case["tol"]


def _nextpow2(x):
    n = 0
    x -= 1
    while x > 0:
        x >>= 1
        n += 1
    return n


@pytest.mark.parametrize("case", G.load("fftfilt"), ids=lambda c: c["name"])
def test_fftfilt_golden(case):
    # runner: src/filter/tests/fftfilt_runtest.c:83-120 (block n = 2^nextpow2(h-1))
    typ = TYPES[case["type"]]
    h, x, y = G.arr(case["h"]), G.arr(case["x"]), G.arr(case["y"])
    n = 1 << _nextpow2(len(h) - 1)
    nb = -(-len(x) // n)
    xp = np.zeros(nb * n, x.dtype)
    xp[: len(x)] = x
    q = O.FftFilt(typ, h, n)
    out = q.execute_stream(xp)
    assert np.max(np.abs(out[: len(y)] - y)) < case["tol"]


@pytest.mark.parametrize("case", G.load("fft"), ids=lambda c: "n%d" % c["n"])
def test_fft_golden(case):
    # runner: src/fft/tests/fft_runtest.c:30-67 (tol 2e-4 on |error|)
    x, y = G.arr(case["x"]), G.arr(case["y"])
    Y = O.fft(x, +1)
    assert np.max(np.abs(Y - y)) < case["tol"]
    z = O.fft(Y, -1) / len(x)
    assert np.max(np.abs(z - x)) < case["tol"]


KA = G.load("known_answers")


@pytest.mark.parametrize("name", [k for k in KA if k.startswith("autotest_dotprod") and "basic" not in k])
def test_dotprod_known_answer(name):
    c = KA[name]
    typ = TYPES[c["type"]]
    y = O.dotprod(typ, G.arr(c["h"]), G.arr(c["x"]))
    assert abs(complex(y) - G.scalar(c["y"])) < c["tol"] * 1.5


def test_dotprod_rrrf_basic():
    c = KA["autotest_dotprod_rrrf_basic"]
    for case in c["cases"]:
        y = O.dotprod(O.RRRF, G.arr(c["h"]), G.arr(case["x"]))
        assert abs(y - case["y"]) < c["tol"]


@pytest.mark.parametrize("name", ["autotest_firinterp_rrrf_generic", "autotest_firinterp_crcf_generic"])
def test_firinterp_known_answer(name):
    c = KA[name]
    typ = TYPES[c["type"]]
    q = O.FirInterp(typ, c["M"], G.arr(c["h"]))
    y = q.execute_block(G.arr(c["x"]))
    assert np.max(np.abs(y - G.arr(c["y"]))) < c["tol"] * 4   # float32 rounding of a 1e-6 test


def test_firpfb_known_answer():
    c = KA["autotest_firpfb_impulse_response"]
    q = O.FirPfb(O.RRRF, c["M"], G.arr(c["h"]))
    for v in G.arr(c["x"]):
        q.push(v)
    out = np.array([q.execute(i) for i in range(c["M"])])
    assert np.max(np.abs(out - G.arr(c["y"]))) < c["tol"]


# ----------------------------------------------------------------------------- float64 restatements
def _rng(seed=1):
    return np.random.default_rng(seed)


def _cx(rng, n):
    return (rng.uniform(-0.5, 0.5, n) + 1j * rng.uniform(-0.5, 0.5, n)).astype(np.complex64)


def test_firfilt_matches_convolution():
    rng = _rng(2)
    h = rng.uniform(-0.5, 0.5, 64).astype(np.float32)
    x = _cx(rng, 5000)
    ref = np.convolve(x.astype(np.complex128), h.astype(np.float64))[: len(x)]
    q = O.FirFilt(O.CRCF, h)
    q.set_scale(0.75)
    y = q.execute_block(x)
    assert G.nrm_err(y, 0.75 * ref) < 1e-6


def test_kaiser_design_properties():
    h = O.firdes_kaiser(65, 0.2, 60.0, 0.0)
    assert np.allclose(h, h[::-1], atol=1e-6)                 # linear phase
    H = np.abs(np.fft.fft(h.astype(np.float64), 4096))
    f = np.arange(4096) / 4096
    assert np.max(H[(f > 0.27) & (f < 0.73)]) < 10 ** (-50 / 20) * H[0]
    assert abs(O.lib().orc_kaiser_beta_As(60.0) - 0.1102 * (60 - 8.7)) < 1e-5


def firpfbch2_closed_form(x, h, M, m, nblocks):
    """SURVEY Appendix B closed form of the firpfbch2 analyzer, float64."""
    x = x.astype(np.complex128)
    h = h.astype(np.float64)
    M2 = M // 2
    Y = np.zeros((nblocks, M), np.complex128)
    j = np.arange(M)
    for b in range(nblocks):
        off = (b % 2) * M2
        i = (j - off) % M
        c = np.where(j < M2, b // 2, (b - 1) // 2)
        base = np.where(j < M2, M2 - 1 - j, 3 * M2 - 1 - j)
        X = np.zeros(M, np.complex128)
        for n in range(2 * m):
            t = (c - n) * M + base
            v = np.where((t >= 0) & (t < len(x)), x[np.clip(t, 0, len(x) - 1)], 0)
            X += h[i + n * M] * v
        Y[b] = np.fft.ifft(X)          # (1/M) sum X e^{+j2pi jk/M}
    return Y


@pytest.mark.parametrize("M,m", [(8, 2), (64, 4), (1024, 4)])
def test_firpfbch2_analyzer_closed_form(M, m):
    rng = _rng(3)
    nblocks = 24 if M == 1024 else 64
    x = _cx(rng, nblocks * M // 2)
    q = O.FirPfbch2(O.ANALYZER, M, m, 60.0)
    y = q.execute_block(x).reshape(nblocks, M)
    h = O.firpfbch2_prototype(O.ANALYZER, M, m, 60.0)
    ref = firpfbch2_closed_form(x, h, M, m, nblocks)
    assert G.nrm_err(y, ref) < 2e-6


@pytest.mark.parametrize("M,m", [(8, 2), (16, 5), (64, 4)])
@pytest.mark.parametrize("kaiser", [False, True])
def test_firpfbch2_analyzer_equals_downconverter_bank(M, m, kaiser):
    """pins the analyzer ALONE to the golden-pinned firfilt oracle
    (test_firfilt_golden) through the reference's down-converter equivalence
    (G.firpfbch2_downconverter): random taps and the Kaiser prototype, both
    block parities, from a zero state"""
    rng = _rng(M + m)
    nblocks = 64
    x = _cx(rng, nblocks * M // 2)
    if kaiser:
        q = O.FirPfbch2(O.ANALYZER, M, m, 60.0)
        h = O.firpfbch2_prototype(O.ANALYZER, M, m, 60.0)
    else:
        h = rng.uniform(-0.5, 0.5, 2 * M * m).astype(np.float32)
        q = O.FirPfbch2(O.ANALYZER, M, m, h=h)
    y = q.execute_block(x).reshape(nblocks, M)
    ref = G.firpfbch2_downconverter(x, h, M, m, nblocks, lambda hh, z: O.FirFilt(O.CRCF, hh).execute_block(z))
    assert G.nrm_err(y, ref) < 1e-5


@pytest.mark.parametrize("M", [8, 16, 32, 64])
def test_firpfbch2_perfect_reconstruction(M):
    # src/multichannel/tests/firpfbch2_crcf_autotest.c:28-98 (m=5, As=60, tol 1e-3)
    m = 5
    n = M * 8 * m
    s, p, g = 1, 524287, 1031
    x = np.zeros(n, np.complex64)
    for i in range(n):
        s = (s * p) % g
        x[i] = np.float32(s) / np.float32(g) - np.float32(0.5)
    qa = O.FirPfbch2(O.ANALYZER, M, m, 60.0)
    qs = O.FirPfbch2(O.SYNTHESIZER, M, m, 60.0)
    y = np.zeros(n, np.complex64)
    for i in range(0, n, M // 2):
        Y = qa.execute(x[i:i + M // 2])
        y[i:i + M // 2] = qs.execute(Y)
    d = 2 * M * m - M // 2 + 1
    assert np.max(np.abs(y[:d])) < 1e-3
    assert np.max(np.abs(y[d:] - x[: n - d])) < 1e-3


def test_firpfbch_analyzer_vs_traditional():
    # src/multichannel/tests/firpfbch_crcf_analyzer_autotest.c:30-146:
    # polyphase analyzer == mixer + full-rate firfilt sampled every M
    rng = _rng(4)
    M, p, ns = 4, 5, 40
    h = rng.choice([-1.5, -0.5, 0.5, 1.5], M * p).astype(np.float32)
    x = (0.1 * np.sqrt(0.5) * (rng.choice([-1.5, -0.5, 0.5, 1.5], M * ns)
                               + 1j * rng.choice([-1.5, -0.5, 0.5, 1.5], M * ns))).astype(np.complex64)
    q = O.FirPfbch(O.ANALYZER, M, p=p, h=h)
    Y0 = np.array([q.execute(x[i * M:(i + 1) * M]) for i in range(ns)])
    Y1 = np.zeros((ns, M), np.complex128)
    for k in range(M):
        mix = x.astype(np.complex128) * np.exp(-2j * np.pi * k * np.arange(M * ns) / M)
        full = np.convolve(mix, h.astype(np.float64))[: M * ns]
        Y1[:, k] = full[M - 1::M]
    assert np.max(np.abs(Y0 - Y1)) < 1e-4


def test_fftfilt_matches_convolution():
    rng = _rng(5)
    h = rng.uniform(-0.5, 0.5, 512).astype(np.float32)
    n = 2048
    x = _cx(rng, 8 * n)
    q = O.FftFilt(O.CRCF, h, n)
    y = q.execute_stream(x)
    ref = np.convolve(x.astype(np.complex128), h.astype(np.float64))[: len(x)]
    assert G.nrm_err(y, ref) < 2e-6


def test_firdecim_firinterp_closed_forms():
    rng = _rng(6)
    x = _cx(rng, 1200)
    for M, m in [(2, 3), (5, 4)]:
        q = O.FirDecim(O.CRCF, M, m=m, As=60.0)
        y = q.execute_block(x)
        hf = O.firdes_kaiser(2 * M * m + 1, 0.5 / M, 60.0)[: 2 * M * m]
        full = np.convolve(x.astype(np.complex128), hf.astype(np.float64))[: len(x)]
        assert G.nrm_err(y, full[::M][: len(y)]) < 1e-6
        qi = O.FirInterp(O.CRCF, M, m=m, As=60.0)
        yi = qi.execute_block(x[:300])
        z = np.zeros(300 * M, np.complex128)
        z[::M] = x[:300]
        ref = np.convolve(z, hf.astype(np.float64))[: 300 * M]
        assert G.nrm_err(yi, ref) < 1e-6


def _resamp_ref(x, rate, m=7, fc=0.25, As=60.0, npfb=64):
    """float64 evaluation of the resampler on the oracle's exact schedule."""
    b, mu, idx = O.resamp_schedule(rate, npfb, len(x))
    n = 2 * m * npfb + 1
    hf = O.firdes_kaiser(n, fc / npfb, As).astype(np.float64)
    hf = hf * (npfb / np.sum(O.firdes_kaiser(n, fc / npfb, As)))
    L = 2 * m
    bank = np.array([[hf[i + k * npfb] for k in range(L)] for i in range(npfb)])   # bank[i][k] taps newest-last reversed
    xx = np.concatenate([np.zeros(L - 1, np.complex128), x.astype(np.complex128)])

    def f(i, t):                           # filter i on the window ending at input t
        w = xx[t: t + L][::-1]            # newest first
        return np.dot(bank[i], w)
    y = np.zeros(len(b), np.complex128)
    for k in range(len(b)):
        t = int(idx[k])
        if b[k] >= 0:
            y0, y1 = f(b[k], t), f(b[k] + 1, t)
        else:
            y0, y1 = f(npfb - 1, t - 1), f(0, t)
        y[k] = (1 - mu[k]) * y0 + mu[k] * y1
    return y


def test_resamp_exact_schedule_and_values():
    rng = _rng(7)
    x = _cx(rng, 3000)
    q = O.Resamp(1.037)
    y = q.execute_block(x)
    b, mu, idx = O.resamp_schedule(1.037, 64, len(x))
    assert len(y) == len(b)
    assert abs(len(y) / len(x) - 1.037) < 0.01
    assert G.nrm_err(y, _resamp_ref(x, 1.037)) < 2e-6


def test_resamp_reference_autotest():
    """autotest_resamp_crcf restated exactly (resamp_crcf_autotest.c:29-136):
    rate, peak level, peak frequency and side-lobes of the resampled
    Kaiser-windowed tone, one execute() per input"""
    r, m, bw, As, npfb, x, check = G.resamp_autotest_case()
    q = O.Resamp(r, m, bw, As, npfb)
    y = np.concatenate([q.execute_block(x[i:i + 1]) for i in range(len(x))])
    assert check(y) == []
    y2 = O.Resamp(r, m, bw, As, npfb).execute_block(x)
    np.testing.assert_array_equal(y2, y)


@pytest.mark.parametrize("M,m,chans", [
    (1024, 4, [0, 1, 255, 511, 512, 513, 1023, 77, 140, 333, 600, 700, 801, 900, 950, 1000]),
])
def test_firpfbch2_downconverter_baseline_geometry(M, m, chans):
    """sandbox/firpfbch2_analysis_equivalence_test.c:182-215 at BASELINE
    config 4's geometry (M = 1024, m = 4, Kaiser As = 60): the oracle
    analyzer against mixer + golden-pinned firfilt, on a channel subset,
    24 blocks from a zero state (both block parities)"""
    rng = _rng(1024 + 4)
    nblocks = 24
    x = _cx(rng, nblocks * M // 2)
    y = O.FirPfbch2(O.ANALYZER, M, m, 60.0).execute_block(x).reshape(nblocks, M)
    h = O.firpfbch2_prototype(O.ANALYZER, M, m, 60.0)
    ref = G.firpfbch2_downconverter(x, h, M, m, nblocks, lambda hh, z: O.FirFilt(O.CRCF, hh).execute_block(z),
                                    channels=chans)
    assert G.nrm_err(y[:, chans], ref) < 1e-5


def test_firpfbch_downconverter_baseline_geometry():
    """firpfbch_crcf_analyzer_autotest.c:30-146 at M = 1024, p = 8 (random
    taps, as the reference's "can be random" note allows), channel subset"""
    rng = _rng(88)
    M, p, ns = 1024, 8, 16
    chans = [0, 1, 2, 511, 512, 513, 1022, 1023, 100, 300, 700, 900]
    h = rng.choice([-1.5, -0.5, 0.5, 1.5], M * p).astype(np.float32)
    x = (0.1 * np.sqrt(0.5) * (rng.choice([-1.5, -0.5, 0.5, 1.5], M * ns)
                               + 1j * rng.choice([-1.5, -0.5, 0.5, 1.5], M * ns))).astype(np.complex64)
    y = O.FirPfbch(O.ANALYZER, M, p=p, h=h)
    Y0 = np.array([y.execute(x[i * M:(i + 1) * M]) for i in range(ns)])
    Y1 = G.firpfbch_downconverter(x, h, M, ns, lambda hh, z: O.FirFilt(O.CRCF, hh).execute_block(z), chans)
    assert np.max(np.abs(Y0[:, chans] - Y1)) < 1e-4


def test_resamp_spectral():
    # src/filter/tests/resamp_crcf_autotest.c: a tone survives at unit gain
    q = O.Resamp(0.9)
    n = 4000
    f0 = 0.05
    x = np.exp(2j * np.pi * f0 * np.arange(n)).astype(np.complex64)
    y = q.execute_block(x)
    t = y[200:-50]
    amp = np.abs(t)
    assert abs(np.mean(amp) - 1.0) < 0.01
    assert abs(len(y) / n - 0.9) < 0.01


# ------------------------------------------------------------ resamp2 / msresamp (reference autotests)
def test_resamp2_analysis_reference():
    m, n, x, check = G.resamp2_analysis_case()
    q = O.Resamp2(m, 0.0, 60.0)
    y = q.run(1, x)
    err, tol = check(y[0::2], y[1::2])
    assert err < tol


def test_resamp2_synthesis_reference():
    m, n, x, check = G.resamp2_synthesis_case()
    y = O.Resamp2(m, 0.0, 60.0).run(2, x)
    err, tol = check(y)
    assert err < tol


def test_resamp2_modes_closed_form():
    # every mode is a convolution with the half-band h (resamp2.c:62-99):
    # interp y[2n] = x[n-m], y[2n+1] = sum_l h[2l+1] x[n-l]; the filter mode's
    # low band is 0.5 (x[i-2m] + sum_l h[2l+1] x[i-1-2l])
    m, As = 4, 60.0
    hl = 4 * m + 1
    t = np.arange(hl) - 2 * m
    from scipy.special import i0
    beta = 0.1102 * (As - 8.7)
    h = np.sinc(t / 2.0) * G.liquid_kaiser(np.arange(hl), hl, beta)
    r = _rng(8)
    x = _cx(r, 300).astype(np.complex128)
    q = O.Resamp2(m, 0.0, As)
    y = q.run(4, x.astype(np.complex64))
    xp = np.concatenate([np.zeros(2 * m), x])
    ref = np.empty(600, complex)
    for k in range(300):
        ref[2 * k] = xp[2 * m + k - m]
        ref[2 * k + 1] = sum(h[2 * l + 1] * xp[2 * m + k - l] for l in range(2 * m))
    assert np.max(np.abs(y - ref)) < 1e-5 * np.max(np.abs(ref))
    q2 = O.Resamp2(m, 0.0, As)
    y0, y1 = q2.run(0, x.astype(np.complex64))
    xp = np.concatenate([np.zeros(4 * m), x])
    lo = np.array([0.5 * (xp[4 * m + i - 2 * m] + sum(h[2 * l + 1] * xp[4 * m + i - 1 - 2 * l] for l in range(2 * m)))
                   for i in range(300)])
    assert np.max(np.abs(y0 - lo)) < 1e-5 * np.max(np.abs(lo))


def test_msresamp_spectral_reference():
    r, As, x, check = G.msresamp_spectral_case()
    q = O.MsResamp(r, As)
    y = np.concatenate([q.execute(x[i:i + 1]) for i in range(len(x))])
    assert check(y) == []


# ------------------------------------------------------------ real-to-real transforms
R2R = G.load("fft_r2r")


def r2r_np(typ, x):
    """fft_r2r_1d.c:95-250 in float64 (un-normalised, factor 2)."""
    x = np.asarray(x, np.float64)
    n = len(x)
    i = np.arange(n)[:, None]
    k = np.arange(n)[None, :]
    if typ == 10:
        y = 0.5 * (x[0] + np.where(np.arange(n) % 2, -x[-1], x[-1]))
        y = y + (np.cos(np.pi * k[:, 1:n - 1] * i / (n - 1)) @ x[1:n - 1])
    elif typ == 11:
        y = np.cos(np.pi * (k + 0.5) * i / n) @ x
    elif typ == 12:
        y = 0.5 * x[0] + np.cos(np.pi * (i + 0.5) * k[:, 1:] / n) @ x[1:]
    elif typ == 13:
        y = np.cos(np.pi * (k + 0.5) * (i + 0.5) / n) @ x
    elif typ == 20:
        y = np.sin(np.pi * (k + 1) * (i + 1) / (n + 1)) @ x
    elif typ == 21:
        y = np.sin(np.pi * (k + 0.5) * (i + 1) / n) @ x
    elif typ == 22:
        y = np.where(np.arange(n) % 2, -0.5, 0.5) * x[-1] + np.sin(np.pi * (k[:, :n - 1] + 1) * (i + 0.5) / n) @ x[:n - 1]
    else:
        y = np.sin(np.pi * (k + 0.5) * (i + 0.5) / n) @ x
    return 2.0 * np.ravel(y)


@pytest.mark.parametrize("case", R2R, ids=lambda c: c["name"])
def test_r2r_formula_golden(case):
    assert np.max(np.abs(r2r_np(case["type"], case["x"]) - np.asarray(case["y"]))) < case["tol"]
