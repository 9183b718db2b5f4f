"""Multi-GPU path on the GPU box (`-m gpu`), one device.

* Time-sharding one firpfbch2 stream (liquid-dsp_amd/lqshard.py):
  independent HIP objects, each warmed up on its shard's halo, must
  reproduce the single-stream HIP run bit for bit (firpfbch2.c:252-281: the
  block parity `flag` and the last 2mM inputs are the whole state).
* bench.py --gpus 2 started without a launcher spawns its own ranks (here
  both on the one GPU, counters over gloo) and reports n_gpus 2 with the
  same sharded-stream checksum as --gpus 1.
* Fast-path guards: an output pointer that is only 8-byte aligned must
  still give correct results (the fast analyzer stores 16 bytes at a time).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import golden_io as G
import liquidmi as LQ
import lqshard
import oracle_lib as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cx(r, n):
    return (r.uniform(-0.5, 0.5, n) + 1j * r.uniform(-0.5, 0.5, n)).astype(np.complex64)


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("M,m", [(1024, 4), (1024, 2), (64, 4)])
def test_firpfbch2_sharded_objects_bit_exact(world, M, m):
    r = np.random.default_rng(world * 100 + M + m)
    nb = 4000 if M == 1024 else 20001
    x = cx(r, nb * M // 2)
    dx = LQ.DeviceBuffer.from_array(x)
    dy = LQ.DeviceBuffer(nb * M * 8)
    q = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, m, 60.0)
    q.execute_block_dev(dx.p, nb, dy.p)
    q.synchronize()
    full = dy.to_array(np.complex64, nb * M)
    parts = []
    for sh in lqshard.firpfbch2_plan(nb, world, M, m):
        n = sh.warm + sh.count
        if not n:
            continue
        qs = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, m, 60.0)
        ys = LQ.DeviceBuffer(n * M * 8)
        qs.execute_block_dev(dx.p + sh.first * (M // 2) * 8, n, ys.p)
        qs.synchronize()
        parts.append(ys.to_array(np.complex64, n * M)[sh.warm * M:])
    assert np.array_equal(np.concatenate(parts), full)


def test_firfilt_sharded_objects_bit_exact():
    r = np.random.default_rng(5)
    h = r.uniform(-0.5, 0.5, 64).astype(np.float32)
    n = (1 << 20) + 999
    x = cx(r, n)
    full = LQ.FirFilt("crcf", h).execute_block(x)
    parts = [LQ.FirFilt("crcf", h).execute_block(x[s.first:s.start + s.count])[s.warm:]
             for s in lqshard.firfilt_plan(n, 4, len(h))]
    # shards start on other chunk boundaries: equal to float32 rounding of the
    # same sums (the matrix kernel's term order does not depend on position)
    assert G.nrm_err(np.concatenate(parts), full) < 1e-6


def _bench(gpus):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "2", "--warmup", "1",
           "--samples", str(1 << 20), "--shard-samples", str(1 << 21), "--no-firfilt", "--no-resamp",
           "--no-extra", "--no-cpu-baseline", "--no-percall", "--no-ceilings"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    # the headline record is the last JSON line (an "aux" line precedes it)
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    head = [d for d in lines if "metric" in d]
    assert len(head) == 1 and lines[-1] is head[0], out.stdout
    return head[0]


def test_bench_spawns_ranks_and_sharded_checksum_is_invariant():
    one = _bench(1)
    two = _bench(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    s1, s2 = one["firpfbch2_sharded_stream"], two["firpfbch2_sharded_stream"]
    assert s1["owned_samples"] == s2["owned_samples"] == 1 << 21
    assert s1["output_checksum"] == s2["output_checksum"]


def test_firpfbch2_output_8byte_aligned():
    r = np.random.default_rng(8)
    nb = 300
    x = cx(r, nb * 512)
    dx = LQ.DeviceBuffer.from_array(x)
    dy = LQ.DeviceBuffer(nb * 1024 * 8 + 8)
    q = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, 1024, 4, 60.0)
    q.execute_block_dev(dx.p, nb, dy.p + 8)
    q.synchronize()
    y = dy.to_array(np.complex64, nb * 1024 + 1)[1:]
    ref = O.FirPfbch2(O.ANALYZER, 1024, 4, 60.0).execute_block(x)
    assert G.nrm_err(y, ref) < 1e-5


@pytest.mark.parametrize("m", [4, 2])
def test_firpfbch2_input_8byte_aligned(m):
    """x only 8-byte aligned: the M = 1024 analyzer takes its one-load-per-row
    kernel instead of the paired 16-byte loads; calls of both parities and
    ragged lengths, compared with the oracle"""
    r = np.random.default_rng(9 + m)
    nb = 333
    x = cx(r, nb * 512)
    dx = LQ.DeviceBuffer(nb * 512 * 8 + 8)
    LQ.lib().liquid_mi355x_memcpy_h2d(dx.p + 8, LQ.ptr(x), x.nbytes)
    dy = LQ.DeviceBuffer(nb * 1024 * 8)
    q = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, 1024, m, 60.0)
    cut = 101   # odd: the second call starts on an odd block
    q.execute_block_dev(dx.p + 8, cut, dy.p)
    q.execute_block_dev(dx.p + 8 + cut * 512 * 8, nb - cut, dy.p + cut * 1024 * 8)
    q.synchronize()
    y = dy.to_array(np.complex64, nb * 1024)
    ref = O.FirPfbch2(O.ANALYZER, 1024, m, 60.0).execute_block(x)
    assert G.nrm_err(y, ref) < 1e-5
