"""k_resamp4 (csrc/k_resamp4.hip): resamp_crcf / _cccf at rates 1/4 < r <= npfb
with a power-of-two bank count, against the oracle (`-m gpu`).

The kernel replays an output plan (an entry every fourth output, then up to
three straight-line steps per lane), so what these cases stress is where the
plan and the tiles meet the call: calls whose first output is not a multiple
of 4 (every lane skips 1-3 outputs from its entry), calls whose output count
is not a multiple of 4 (the ragged lane), calls shorter than one 256-output
tile, the first tiles of a call reading the history, long streams crossing
the plan's period, unaligned output pointers (8-byte stores), and the same
stream through the input-checkpoint kernel (k_resamp3, LQ_RESAMP_INPUT_PLAN=1)
for comparison.  Bar: normwise 1e-5 against the oracle, exact output counts.
"""
import os

import numpy as np
import pytest

import golden_io as G
import liquidmi as LQ
import oracle_lib as O

pytestmark = pytest.mark.gpu

NRM = 1e-5


def cx(r, n):
    return (r.uniform(-0.5, 0.5, n) + 1j * r.uniform(-0.5, 0.5, n)).astype(np.complex64)


@pytest.fixture(params=["output_plan", "input_plan"])
def plan_kind(request):
    old = os.environ.get("LQ_RESAMP_INPUT_PLAN")
    if request.param == "input_plan":
        os.environ["LQ_RESAMP_INPUT_PLAN"] = "1"
    else:
        os.environ.pop("LQ_RESAMP_INPUT_PLAN", None)
    yield request.param
    if old is None:
        os.environ.pop("LQ_RESAMP_INPUT_PLAN", None)
    else:
        os.environ["LQ_RESAMP_INPUT_PLAN"] = old


@pytest.mark.parametrize("rate,m,npfb", [(1.037, 7, 64), (1.27115323, 13, 64), (1.5, 4, 64), (1.9, 7, 32),
                                         (1.0001, 2, 64), (1.3, 16, 256), (1.7, 10, 128), (1.11, 1, 8),
                                         (1.00624001, 7, 64), (1.02353001, 5, 64),
                                         # 1/2 < r < 1 (the kernel's second rate class)
                                         (0.97, 7, 64), (0.51, 7, 64), (0.6, 13, 32), (0.825, 7, 64),
                                         (0.75, 4, 128), (0.99, 16, 256), (0.5001, 1, 8), (0.9, 12, 64),
                                         # r > 2 (the third class: more than two outputs per input)
                                         (2.5, 7, 64), (3.7, 7, 64), (2.01, 13, 32), (3.99, 4, 128),
                                         (3.3, 16, 256), (2.2, 1, 8), (5.5, 7, 32), (10.0, 7, 64),
                                         (60.0, 4, 64), (7.3, 1, 8),
                                         # 1/4 < r <= 1/2 (an output every two to four inputs)
                                         (0.3, 7, 64), (0.45, 13, 32), (0.26, 4, 128), (0.5, 7, 64),
                                         (0.33, 16, 256), (0.4, 1, 8)])
def test_resamp4_ragged_calls(plan_kind, rate, m, npfb):
    rate = float(np.float32(rate))
    r = np.random.default_rng(int(rate * 1000) + m + npfb)
    x = cx(r, 300_000)
    g = LQ.Resamp(rate, m, 0.25, 60.0, npfb)
    o = O.Resamp(rate, m, 0.25, 60.0, npfb)
    # short calls (< one tile), odd lengths (first outputs not multiples of
    # 4, ragged ends), one call of 2^16 inputs or more (periodic plan)
    cuts = [0, 3, 5, 6, 250, 251, 777, 1000, 1001, 71_003, 71_004, 140_000, 213_457, 300_000]
    ys = [g.execute_block(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    for (a, b), y in zip(zip(cuts[:-1], cuts[1:]), ys):
        assert len(y) == g_num(rate, npfb, a, b)
    y = np.concatenate(ys)
    ref = o.execute_block(x)
    assert len(y) == len(ref)
    assert G.nrm_err(y, ref) < NRM


_SCHED = {}


def g_num(rate, npfb, a, b):
    """outputs of inputs a..b-1 of a fresh stream, from the oracle's schedule"""
    key = (rate, npfb)
    if key not in _SCHED:
        _, _, idx = O.resamp_schedule(rate, npfb, 300_000)
        _SCHED[key] = idx
    idx = _SCHED[key]
    return int(np.searchsorted(idx, b) - np.searchsorted(idx, a))


@pytest.mark.parametrize("rate", [1.037, 1.00624001, 0.97])
def test_resamp4_cccf_and_long_stream(plan_kind, rate):
    # cccf runs the complex kernel (real taps, resamp.c:117-132); 3M inputs in
    # calls of 700 001 cross the plan period twice (r = 1.037: 2^20 outputs;
    # r = 1.00624001: a 3-input pre-period, then 1 389 431 inputs)
    rate = float(np.float32(rate))
    r = np.random.default_rng(99)
    x = cx(r, 3_000_000)
    g = LQ.Resamp(rate, 7, 0.25, 60.0, 64, t=LQ.CCCF)
    o = O.Resamp(rate, 7, 0.25, 60.0, 64)
    y = np.concatenate([g.execute_block(x[a:a + 700_001]) for a in range(0, len(x), 700_001)])
    ref = o.execute_block(x)
    assert len(y) == len(ref)
    assert G.nrm_err(y, ref) < NRM


@pytest.mark.parametrize("off,rate", [(0, 1.037), (8, 1.037), (0, 0.8), (8, 0.8), (0, 3.7), (8, 3.7), (0, 0.3),
                                      (8, 0.3)])
def test_resamp4_device_pointers(off, rate):
    # device-resident call; off = 8: output pointer 8 bytes past a 16-byte
    # boundary (the kernel then stores 8 bytes at a time)
    rate = float(np.float32(rate))
    n = 1_000_003
    r = np.random.default_rng(5 + off)
    x = cx(r, n)
    g = LQ.Resamp(rate, 7, 0.25, 60.0, 64)
    nout = g.num_output(n)
    dx = LQ.DeviceBuffer.from_array(x)
    dy = LQ.DeviceBuffer(nout * 8 + 64)
    ny = g.execute_block_dev(dx.p, n, dy.p + off)
    g.synchronize()
    assert ny == nout
    y = np.empty(nout + 8, np.complex64)
    LQ.lib().liquid_mi355x_memcpy_d2h(LQ.ptr(y), dy.p, y.nbytes)
    y = y.view(np.uint8)[off:off + nout * 8].view(np.complex64)
    ref = O.Resamp(rate, 7, 0.25, 60.0, 64).execute_block(x)
    assert len(ref) == nout
    assert G.nrm_err(y, ref) < NRM


@pytest.mark.parametrize("rate", [1.037, 0.83])
def test_resamp4_matches_input_plan_kernel_bitwise_count(rate):
    # both kernels on the same stream: identical output counts, and values
    # within float32 rounding of each other
    rate = float(np.float32(rate))
    r = np.random.default_rng(123)
    x = cx(r, 400_000)
    a = LQ.Resamp(rate, 7, 0.25, 60.0, 64).execute_block(x)
    os.environ["LQ_RESAMP_INPUT_PLAN"] = "1"
    try:
        b = LQ.Resamp(rate, 7, 0.25, 60.0, 64).execute_block(x)
    finally:
        os.environ.pop("LQ_RESAMP_INPUT_PLAN", None)
    assert len(a) == len(b)
    assert G.nrm_err(a, b) < 2e-6
