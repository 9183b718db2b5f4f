"""The small-call mode (the library's default; LQ_SMALL_CALLS=gpu or
liquid_mi355x_set_small_calls(0) turns it off): single-sample calls computed
on the host by host/lq_small.c, block calls on the GPU.  Same bar as the GPU path: the reference's golden vectors at their
tolerances, and normwise 1e-5 against the oracle over streams that mix
per-sample (host) and block (GPU) calls on one object, so the history
mirrors and the resampler's timing state are exercised in both directions."""
import numpy as np
import pytest

import golden_io as G
import liquidmi as LQ
import oracle_lib as O

pytestmark = pytest.mark.gpu

NRM = 1e-5
TYPES = {"rrrf": O.RRRF, "crcf": O.CRCF, "cccf": O.CCCF}


@pytest.fixture(autouse=True)
def host_small_calls():
    LQ.set_small_calls(True)
    yield
    LQ.set_small_calls(False)


def rng(seed):
    return np.random.default_rng(seed)


def cx(r, n):
    return (r.uniform(-0.5, 0.5, n) + 1j * r.uniform(-0.5, 0.5, n)).astype(np.complex64)


def samples(r, t, n):
    return r.uniform(-0.5, 0.5, n).astype(np.float32) if t == "rrrf" else cx(r, n)


def coefs(r, t, n):
    return cx(r, n) if t == "cccf" else r.uniform(-0.5, 0.5, n).astype(np.float32)


def test_mode_switch():
    assert LQ.get_small_calls()
    LQ.set_small_calls(False)
    assert not LQ.get_small_calls()
    LQ.set_small_calls(True)


@pytest.mark.parametrize("case", G.load("firfilt"), ids=lambda c: c["name"])
def test_firfilt_golden_host(case):
    h, x, y = G.arr(case["h"]), G.arr(case["x"]), G.arr(case["y"])
    q = LQ.FirFilt(case["type"], h)
    out = []
    for v in x:                       # firfilt_runtest.c:68-95: push + execute
        q.push(v)
        out.append(q.execute())
    assert np.max(np.abs(np.asarray(out) - y)) < case["tol"]


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("hlen", [1, 13, 64, 100])
def test_firfilt_mixed_vs_oracle(t, hlen):
    r = rng(hlen + 3)
    h = coefs(r, t, hlen)
    x = samples(r, t, 6000)
    g = LQ.FirFilt(t, h)
    o = O.FirFilt(TYPES[t], h)
    s = (0.7 - 0.2j) if t == "cccf" else 0.7
    g.set_scale(s)
    o.set_scale(s)
    out = []
    for a, b, per in [(0, 300, True), (300, 4000, False), (4000, 4400, True), (4400, 6000, False)]:
        if per:
            for v in x[a:b]:
                g.push(v)
                out.append(np.atleast_1d(g.execute()))
        else:
            out.append(g.execute_block(x[a:b]))
    y = np.concatenate(out)
    assert G.nrm_err(y, o.execute_block(x)) < NRM


KA = G.load("known_answers")


@pytest.mark.parametrize("name", [k for k in KA if k.startswith("autotest_dotprod") and "basic" not in k])
def test_dotprod_known_answer_host(name):
    c = KA[name]
    h, x = G.arr(c["h"]), G.arr(c["x"])
    assert abs(complex(LQ.dotprod_run(c["type"], h, x)) - G.scalar(c["y"])) < c["tol"] * 1.5
    assert abs(complex(LQ.DotProd(c["type"], h).execute(x)) - G.scalar(c["y"])) < c["tol"] * 1.5


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("n", [1, 7, 64, 1000])
def test_dotprod_vs_oracle_host(t, n):
    r = rng(n)
    h, x = coefs(r, t, n), samples(r, t, n)
    y = LQ.DotProd(t, h).execute(x)
    ref = O.dotprod(TYPES[t], h, x)
    assert abs(complex(y) - complex(ref)) <= 1e-5 * max(1.0, abs(complex(ref)))


@pytest.mark.parametrize("case", G.load("firdecim"), ids=lambda c: c["name"])
def test_firdecim_golden_host(case):
    h, x, y = G.arr(case["h"]), G.arr(case["x"]), G.arr(case["y"])
    q = LQ.FirDecim(case["M"], h, t=case["type"])
    out = np.array([q.execute(x[i * case["M"]:(i + 1) * case["M"]]) for i in range(len(y))])
    assert np.max(np.abs(out - y)) < case["tol"]


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("M,hlen", [(2, 1), (3, 21), (8, 64)])
def test_firdecim_mixed_vs_oracle(t, M, hlen):
    r = rng(M * 100 + hlen)
    h = coefs(r, t, hlen)
    nout = 900
    x = samples(r, t, nout * M)
    g = LQ.FirDecim(M, h, t=t)
    o = O.FirDecim(TYPES[t], M, h=h)
    out = []
    for a, b, per in [(0, 100, True), (100, 600, False), (600, 700, True), (700, 900, False)]:
        if per:
            out += [np.atleast_1d(g.execute(x[i * M:(i + 1) * M])) for i in range(a, b)]
        else:
            out.append(g.execute_block(x[a * M:b * M]))
    y = np.concatenate(out)
    assert G.nrm_err(y, o.execute_block(x)) < NRM


def test_firinterp_known_answer_host():
    c = KA["autotest_firinterp_crcf_generic"]
    q = LQ.FirInterp(c["M"], G.arr(c["h"]))
    y = np.concatenate([q.execute(v) for v in G.arr(c["x"])])
    assert np.max(np.abs(y - G.arr(c["y"]))) < 4e-6


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("M,hlen", [(2, 2), (4, 27), (8, 64)])
def test_firinterp_mixed_vs_oracle(t, M, hlen):
    r = rng(M * 31 + hlen)
    h = coefs(r, t, hlen)
    x = samples(r, t, 3000)
    g = LQ.FirInterp(M, h, t=t)
    o = O.FirInterp(TYPES[t], M, h=h)
    out = []
    for a, b, per in [(0, 200, True), (200, 2000, False), (2000, 2300, True), (2300, 3000, False)]:
        if per:
            out += [g.execute(v) for v in x[a:b]]
        else:
            out.append(g.execute_block(x[a:b]))
    y = np.concatenate(out)
    assert G.nrm_err(y, o.execute_block(x)) < NRM


@pytest.mark.parametrize("rate,m,npfb", [(1.037, 7, 64), (0.5, 7, 64), (3.7, 4, 32), (0.8131, 3, 37),
                                         (83.3, 7, 64), (10.3, 3, 64)])
def test_resamp_mixed_vs_oracle(rate, m, npfb):
    rate = float(np.float32(rate))
    r = rng(int(rate * 1000) + m)
    x = cx(r, 40_000)
    g = LQ.Resamp(rate, m, 0.25, 60.0, npfb)
    o = O.Resamp(rate, m, 0.25, 60.0, npfb)
    out = []
    for a, b, per in [(0, 500, True), (500, 20_000, False), (20_000, 20_700, True), (20_700, 40_000, False)]:
        if per:
            out += [g.execute(v) for v in x[a:b]]
        else:
            out.append(g.execute_block(x[a:b]))
    y = np.concatenate(out)
    ref = o.execute_block(x)
    assert len(y) == len(ref)
    assert G.nrm_err(y, ref) < NRM


def test_resamp_reference_autotest_host():
    # autotest_resamp_crcf (resamp_crcf_autotest.c:29-136): one execute() per input
    rr, m, bw, As, npfb, x, check = G.resamp_autotest_case()
    g = LQ.Resamp(rr, m, bw, As, npfb)
    y = np.concatenate([g.execute(v) for v in x])
    assert check(y) == []
    ref = O.Resamp(rr, m, bw, As, npfb).execute_block(x)
    assert len(y) == len(ref) and G.nrm_err(y, ref) < NRM


def test_resamp_set_rate_reset_host():
    r = rng(77)
    x = cx(r, 12_000)
    g = LQ.Resamp(float(np.float32(1.037)), 7, 0.25, 60.0, 64)
    o = O.Resamp(float(np.float32(1.037)), 7, 0.25, 60.0, 64)
    a = [g.execute(v) for v in x[:3000]] + [g.execute_block(x[3000:6000])]
    b = [o.execute_block(x[:6000])]
    g.set_rate(0.913)
    o.set_rate(float(np.float32(0.913)))
    a += [g.execute(v) for v in x[6000:7000]] + [g.execute_block(x[7000:])]
    b += [o.execute_block(x[6000:])]
    ya, yb = np.concatenate(a), np.concatenate(b)
    assert len(ya) == len(yb) and G.nrm_err(ya, yb) < NRM
    g.reset()
    o.reset()
    ya = np.concatenate([g.execute(v) for v in x[:2000]])
    yb = o.execute_block(x[:2000])
    assert len(ya) == len(yb) and G.nrm_err(ya, yb) < NRM


def _nextpow2(v):
    n = 0
    while (1 << n) < v:
        n += 1
    return n


@pytest.mark.parametrize("case", G.load("fftfilt"), ids=lambda c: c["name"])
def test_fftfilt_golden_host(case):
    # the golden vectors' short blocks run as host direct convolutions
    h, x, y = G.arr(case["h"]), G.arr(case["x"]), G.arr(case["y"])
    n = 1 << _nextpow2(len(h) - 1)
    nb = -(-len(x) // n)
    xp = np.zeros(nb * n, np.float32 if case["type"] == "rrrf" else np.complex64)
    xp[: len(x)] = x
    q = LQ.FftFilt(h, n, t=case["type"])
    out = np.concatenate([q.execute(xp[b * n:(b + 1) * n]) for b in range(nb)])
    assert np.max(np.abs(out[: len(y)] - y)) < case["tol"]


@pytest.mark.parametrize("t", ["rrrf", "crcf", "cccf"])
@pytest.mark.parametrize("hlen,n", [(1, 4), (23, 32), (65, 64), (512, 1024)])
def test_fftfilt_mixed_vs_oracle(t, hlen, n):
    # execute() calls of n samples (host while n h_len <= 65536, else GPU)
    # interleaved with long execute_block calls (GPU) on one object
    r = rng(hlen * 7 + n)
    h = coefs(r, t, hlen)
    nb = 60
    x = samples(r, t, n * nb)
    g, o = LQ.FftFilt(h, n, t=t), O.FftFilt(TYPES[t], h, n)
    s = (1.5 - 0.25j) if t == "cccf" else 1.5
    g.set_scale(s)
    out = []
    for a, b, per in [(0, 10, True), (10, 30, False), (30, 45, True), (45, 60, False)]:
        if per:
            out += [g.execute(x[i * n:(i + 1) * n]) for i in range(a, b)]
        else:
            out.append(g.execute_block(x[a * n:b * n]))
    y = np.concatenate(out)
    assert G.nrm_err(y, s * o.execute_stream(x)) < NRM
    g.reset()
    y2 = np.concatenate([g.execute(x[i * n:(i + 1) * n]) for i in range(4)])
    assert G.nrm_err(y2, y[:4 * n]) < NRM
