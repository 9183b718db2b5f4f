"""resamp timing plan (host side, no GPU): the periodic / direct plans the
library builds must reproduce the reference's float32 timing schedule bit for
bit -- bank index, mu and input index of every output -- against the oracle's
restatement of resamp.c:245-363 (orc_resamp_schedule).

Covers rates with a pure cycle (1.037, 0.97), a pre-period (3.7), tiny periods
(0.5, 1.5, 2.0), many outputs per input (10.3), non-power-of-two banks, and
streams several periods long so the wrap-around of the plan is exercised.
"""
import ctypes as C

import numpy as np
import pytest

import liquidmi as LM
import oracle_lib as O


def _lib_schedule(rate, npfb, nx, periodic, allow_none=False):
    L = LM.lib()
    fn = L.liquid_mi355x_resamp_schedule
    fn.restype = C.c_longlong
    fn.argtypes = [C.c_float, C.c_uint, C.c_ulonglong, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                   C.c_ulonglong, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
    cap = int(np.ceil(nx * rate)) + 16
    b = np.zeros(cap, np.int32)
    mu = np.zeros(cap, np.float32)
    idx = np.zeros(cap, np.uint32)
    pre, per = C.c_ulonglong(0), C.c_ulonglong(0)
    k = fn(rate, npfb, nx, periodic, LM.ptr(b), LM.ptr(mu), LM.ptr(idx), cap, C.byref(pre), C.byref(per))
    if allow_none and k == -1:
        return None
    assert k >= 0, "plan failed (%d)" % k
    return b[:k], mu[:k], idx[:k], pre.value, per.value


@pytest.mark.parametrize("rate,npfb,nx,pre0", [
    (1.037, 64, 3_100_000, 0),     # config 5: period 1 011 163 inputs
    (0.97, 64, 1_000_000, 0),
    (3.7, 64, 2_000_000, 864_961),  # pre-period before the cycle
    (0.5, 64, 10_000, 0),
    (1.5, 64, 10_000, 0),
    (2.0, 64, 10_000, 0),
    (10.3, 64, 900_000, 0),
    (1.037, 50, 1_500_000, 0),     # non-power-of-two bank count
    (0.8131, 37, 400_000, None),
])
def test_periodic_plan_matches_oracle_schedule(rate, npfb, nx, pre0):
    rate = float(np.float32(rate))
    b, mu, idx, pre, per = _lib_schedule(rate, npfb, nx, 1)
    if pre0 is not None:
        assert pre == pre0
    ob, omu, oidx = O.resamp_schedule(rate, npfb, nx)
    assert len(b) == len(ob)
    np.testing.assert_array_equal(b, ob)
    np.testing.assert_array_equal(mu.view(np.uint32), omu.view(np.uint32))
    np.testing.assert_array_equal(idx, oidx)


@pytest.mark.parametrize("rate", [1.037, 0.63, 4.21])
def test_direct_plan_matches_oracle_schedule(rate):
    rate = float(np.float32(rate))
    nx = 50_000
    b, mu, idx, _, _ = _lib_schedule(rate, 64, nx, 0)
    ob, omu, oidx = O.resamp_schedule(rate, 64, nx)
    np.testing.assert_array_equal(b, ob)
    np.testing.assert_array_equal(mu.view(np.uint32), omu.view(np.uint32))
    np.testing.assert_array_equal(idx, oidx)


def test_config5_output_count():
    # 32M inputs at r = 1.037 -> 34 795 945 outputs (probe of the reference)
    rate = float(np.float32(1.037))
    b, _, _, pre, per = _lib_schedule(rate, 64, 1 << 25, 1)
    assert (pre, per) == (0, 1_011_163)
    assert len(b) == 34_795_945


@pytest.mark.parametrize("rate,npfb", [(83.3, 64), (75.5, 64), (100.0, 64), (64.0, 64), (130.7, 64), (57.3, 37)])
@pytest.mark.parametrize("periodic", [0, 1])
def test_rate_above_npfb_unsigned_semantics(rate, npfb, periodic):
    """rates above npfb: resamp.c:254 compares int b with unsigned npfb, so a
    BOUNDARY update that leaves tau < 0 (b = -1) ends the loop and the
    resampler stops producing output (b stays negative); the plans and the
    oracle (which states the comparison as the reference does) agree"""
    rate = float(np.float32(rate))
    nx = 3000
    # a dying orbit has no period (b keeps decreasing): the periodic search
    # gives up and the object runs on direct plans
    got = _lib_schedule(rate, npfb, nx, periodic, allow_none=bool(periodic))
    if got is None:
        return
    b, mu, idx, _, _ = got
    ob, omu, oidx = O.resamp_schedule(rate, npfb, nx)
    assert len(b) == len(ob)
    np.testing.assert_array_equal(b, ob)
    np.testing.assert_array_equal(mu.view(np.uint32), omu.view(np.uint32))
    np.testing.assert_array_equal(idx, oidx)


def test_rate_above_npfb_stops():
    # r = 83.3, npfb = 64: del = 0.012 < 1/64; the first BOUNDARY update
    # leaves tau < 0, so input 1 ends the stream: 84 outputs, none after
    rate = float(np.float32(83.3))
    ob, _, oidx = O.resamp_schedule(rate, 64, 1000)
    assert len(ob) < 2 * rate and oidx.max() <= 1
    b, _, idx, _, _ = _lib_schedule(rate, 64, 1000, 0)
    assert len(b) == len(ob)


# ---------------------------------------------------------------- output plans (k_resamp4)
def _lib_schedule4(rate, npfb, nx, periodic):
    L = LM.lib()
    fn = L.liquid_mi355x_resamp_schedule4
    fn.restype = C.c_longlong
    fn.argtypes = [C.c_float, C.c_uint, C.c_ulonglong, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                   C.c_ulonglong, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
    cap = int(np.ceil(nx * rate)) + 16
    b = np.zeros(cap, np.int32)
    mu = np.zeros(cap, np.float32)
    idx = np.zeros(cap, np.uint32)
    pre, per = C.c_ulonglong(0), C.c_ulonglong(0)
    k = fn(rate, npfb, nx, periodic, LM.ptr(b), LM.ptr(mu), LM.ptr(idx), cap, C.byref(pre), C.byref(per))
    return k, b[:max(k, 0)], mu[:max(k, 0)], idx[:max(k, 0)], pre.value, per.value


@pytest.mark.parametrize("rate,npfb,nx", [
    (1.037, 64, 2_200_000),      # config 5: period 2^20 outputs, crossed twice
    (1.27115323, 64, 400_000),   # autotest_resamp_crcf's rate: period 2^23 outputs
    (1.5, 64, 20_000),           # period 3 outputs: the table repeats 256 outputs
    (1.9, 64, 300_000),
    (1.0001, 64, 300_000),
    (1.3, 32, 300_000),
    (1.7, 256, 300_000),
    (1.00624001, 64, 3_000_000),  # pre-period of 3 inputs: entries below pre, then the period's own phase
    (1.02353001, 64, 1_500_000),  # pre-period of 2 inputs
    (0.97, 64, 300_000),          # 1/2 < r < 1: an output every one or two inputs
    (0.51, 64, 300_000),
    (0.6, 32, 300_000),
    (0.825, 64, 300_000),         # msresamp r = 3.3's arbitrary stage
    (0.75, 128, 20_000),
    (0.99, 256, 300_000),
    (0.9999999, 64, 9_000_000),   # period 8 388 609 inputs
    (2.5, 64, 300_000),           # 2 < r < 4: up to four outputs per input
    (3.7, 64, 300_000),           # pre-period before the cycle
    (2.01, 32, 300_000),
    (3.99, 64, 300_000),
    (2.2, 256, 20_000),
    (5.5, 32, 100_000),           # r > 4 on the same class
    (10.0, 64, 50_000),
    (60.0, 64, 10_000),
    (0.45, 64, 300_000),          # 1/4 < r <= 1/2: an output every two to four inputs
    (0.3, 64, 300_000),
    (0.26, 32, 300_000),
    (0.5, 64, 100_000),
    (0.4, 256, 20_000),
])
@pytest.mark.parametrize("periodic", [1, 0])
def test_output_plan_matches_oracle_schedule(rate, npfb, nx, periodic):
    """the output plan that k_resamp4 replays (an entry every fourth output,
    then up to three straight-line steps) reproduces the reference's float32
    schedule bit for bit: bank (BOUNDARY = -1), mu and input of every output"""
    rate = float(np.float32(rate))
    if not periodic:
        nx = min(nx, 200_000)
    k, b, mu, idx, pre, per = _lib_schedule4(rate, npfb, nx, periodic)
    if periodic and k == -1:
        pytest.skip("no period within the search limit")
    assert k >= 0, "output plan not built (%d)" % k
    if periodic:
        assert per >= 256
    ob, omu, oidx = O.resamp_schedule(rate, npfb, nx)
    assert len(b) == len(ob)
    np.testing.assert_array_equal(b, ob)
    np.testing.assert_array_equal(mu.view(np.uint32), omu.view(np.uint32))
    np.testing.assert_array_equal(idx, oidx)


@pytest.mark.parametrize("rate", [0.25, 0.2, 65.0, 130.0])
def test_output_plan_only_above_quarter_up_to_npfb(rate):
    """rates up to 1/4 or above npfb (bank-index timing) keep the
    input-checkpoint plan (k_resamp3 / k_resamp)"""
    k, *_ = _lib_schedule4(float(np.float32(rate)), 64, 10_000, 0)
    assert k == -3


@pytest.mark.parametrize("rate,npfb", [(1.037, 64), (0.9999999, 64), (1.27115323, 64), (3.7, 64)])
def test_plan_memory(rate, npfb):
    """plan memory: host checkpoints every 16 inputs
    (16-byte entries, grown by doubling) over the search walk and, for the
    device, an entry per 4 outputs (output plan) or per 4 inputs (input
    plan) -- r = 0.9999999 (period 8 388 609 inputs): at most 16 MB host and
    24 MB device"""
    L = LM.lib()
    fn = L.liquid_mi355x_resamp_plan_bytes
    fn.restype = C.c_int
    fn.argtypes = [C.c_float, C.c_uint, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong),
                   C.POINTER(C.c_ulonglong)]
    h, d, P = C.c_ulonglong(0), C.c_ulonglong(0), C.c_ulonglong(0)
    ok = fn(float(np.float32(rate)), npfb, C.byref(h), C.byref(d), C.byref(P))
    assert ok == 1
    per = P.value
    # the host table covers the search walk (Brent's tortoise runs past the
    # period when the orbit does not return to its first states)
    assert h.value <= 16 << 20
    # the output plan holds the pre-period's entries too (r = 3.7: 864 961
    # inputs before the cycle, test_periodic_plan_matches_oracle_schedule above)
    rmax = max(rate, 1.0)
    span = per + {float(np.float32(3.7)): 864_961}.get(float(np.float32(rate)), 0)
    assert d.value <= 8 * (rmax * span / 4 + 1024) + 16 * (span / 4 + 1024)
    if rate == float(np.float32(0.9999999)):
        assert h.value <= 16 << 20 and d.value <= 24 << 20
