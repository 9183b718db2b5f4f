"""Every BASELINE.json config, exercised at its FULL size against the CPU oracle.

CONFIG_TESTS is the index: for each entry of BASELINE.json "configs" it names
the `-m gpu` test that runs that workload at full size and compares the HIP
path with the oracle over the whole output (normwise max|d| / max|ref|
<= 1e-5, the north-star tolerance; tests/test_gpu_parity.py explains why
normwise).  `test_config_index_complete` (CPU) checks that the index covers
every config and that each named test exists.

The two configs whose full-size tests live here:
  * config 2, dotprod_cccf n in {16, 64, 256, 1024} x 2^20 vectors
    (dotprod_cccf.mmx.c:295-381): the whole batch is ONE device launch over
    2^20 vectors (8.6 GB of X at n = 1024, the bench's launch geometry); X is
    generated and uploaded in 2^18-vector slices and each slice of Y is
    compared with the oracle's batch dot product of the same slice.
  * config 3, fftfilt_crcf h=512 with the reference's block n=2048 on 2^26
    samples (fftfilt.c:193-260): one device call over the whole stream,
    compared with the oracle run in 2048-sample execute() calls, split across
    host processes on lqshard.fftfilt_plan shards (warm-up: one whole block
    >= h-1 samples, so each shard's oracle state equals the single stream's).
"""
import json
import os

import numpy as np
import pytest

import golden_io as G
import liquidmi as LQ
import lqshard
import oracle_lib as O
import parallel_oracle as PO

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NRM = 1e-5

# BASELINE.json configs[i] -> the full-size -m gpu test ("file::test")
CONFIG_TESTS = {
    0: ["test_gpu_parity.py::test_firfilt_crcf_baseline_config1_vs_oracle",
        "test_gpu_fullsize.py::test_firfilt_h64_2p28_full_stream_vs_oracle"],
    1: ["test_gpu_configs.py::test_config2_dotprod_cccf_full_batch_vs_oracle"],
    2: ["test_gpu_configs.py::test_config3_fftfilt_full_stream_vs_oracle"],
    3: ["test_gpu_fullsize.py::test_firpfbch2_config4_full_stream_vs_oracle"],
    4: ["test_gpu_parity.py::test_resamp_baseline_config5_device"],
}


def test_config_index_complete():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        configs = json.load(f)["configs"]
    assert sorted(CONFIG_TESTS) == list(range(len(configs)))
    for i, tests in CONFIG_TESTS.items():
        for t in tests:
            fname, name = t.split("::")
            with open(os.path.join(ROOT, "tests", fname)) as f:
                assert ("def %s(" % name) in f.read(), (configs[i], t)


def _cx_slice(seed, count):
    r = np.random.default_rng(seed)
    a = r.random(2 * count, dtype=np.float32)
    a -= 0.5
    return a.view(np.complex64)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [16, 64, 256, 1024])
def test_config2_dotprod_cccf_full_batch_vs_oracle(n):
    nvec, sl = 1 << 20, 1 << 18
    h = _cx_slice(7 + n, n).copy()
    dX = LQ.DeviceBuffer(nvec * n * 8)
    dY = LQ.DeviceBuffer(nvec * 8)
    for s in range(nvec // sl):
        xs = _cx_slice(1000 * n + s, sl * n)
        LQ.lib().liquid_mi355x_memcpy_h2d(dX.p + s * sl * n * 8, LQ.ptr(xs), xs.nbytes)
        del xs
    q = LQ.DotProd("cccf", h)
    q.execute_batch_dev(dX.p, nvec, dY.p)          # one launch over all 2^20 vectors
    LQ.lib().liquid_mi355x_device_synchronize()
    dX.free()
    Y = dY.to_array(np.complex64, nvec)
    dY.free()
    dmax = rmax = 0.0
    for s in range(nvec // sl):
        xs = _cx_slice(1000 * n + s, sl * n)
        ref = O.dotprod_batch(O.CCCF, h, xs)
        got = Y[s * sl:(s + 1) * sl]
        assert np.all(np.isfinite(got))
        dmax = max(dmax, float(np.max(np.abs(got.astype(np.complex128) - ref))))
        rmax = max(rmax, float(np.max(np.abs(ref))))
    assert dmax / rmax < NRM, dmax / rmax


@pytest.mark.gpu
def test_config3_fftfilt_full_stream_vs_oracle():
    nblk, n = 2048, 1 << 26
    h = np.random.default_rng(33).uniform(-0.5, 0.5, 512).astype(np.float32)
    x = np.empty(n, np.complex64)
    step = 1 << 24
    for a in range(0, n, step):
        x[a:a + step] = _cx_slice(300 + a // step, step)
    dx = LQ.DeviceBuffer.from_array(x)
    dy = LQ.DeviceBuffer(n * 8)
    q = LQ.FftFilt(h, nblk)
    q.execute_block_dev(dx.p, n, dy.p)
    LQ.lib().liquid_mi355x_device_synchronize()
    dx.free()
    y = dy.to_array(np.complex64, n)
    dy.free()
    plan = lqshard.fftfilt_plan(n, PO.workers(), len(h), block=nblk)
    assert all(s.count % nblk == 0 and s.first % nblk == 0 for s in plan)
    err, nonfin = PO.compare("fftfilt", x, y, (h, nblk), plan)
    assert nonfin == 0
    assert err < NRM, err


def test_fftfilt_plan_blocks_cpu():
    """the block-aligned fftfilt shard plan reproduces the single-stream oracle
    (CPU, small): shards of whole 64-sample blocks, warm-up >= h-1"""
    r = np.random.default_rng(4)
    h = r.uniform(-0.5, 0.5, 61).astype(np.float32)   # n >= h_len - 1 (fftfilt.c:78-83)
    nb, n = 64, 64 * 40
    x = _cx_slice(5, n)
    ref = O.FftFilt(O.CRCF, h, nb).execute_stream(x)
    out = np.zeros_like(ref)
    for s in lqshard.fftfilt_plan(n, 3, len(h), block=nb):
        assert s.first % nb == 0 and s.warm >= min(s.start, len(h) - 1)
        y = O.FftFilt(O.CRCF, h, nb).execute_stream(x[s.first:s.start + s.count])
        out[s.start:s.start + s.count] = y[s.warm:]
    assert G.nrm_err(out, ref) < 1e-6
