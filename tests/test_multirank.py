"""Multi-rank path on CPU: gloo, world_size 2 (the driver runs N>1 on real GPUs).

Checks the stream-sharding plan (liquid-dsp_amd/lqshard.py) that splits one
long stream across ranks with warm-up halos and no data-path collective:
each rank runs the CPU oracle over its shard, results are gathered, and the
concatenation must equal the single-stream run bit for bit.  Also exercises
the counter reductions bench.py performs (max time, summed samples).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
    import lqshard
    import oracle_lib as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        # firpfbch2 analyzer, M = 64, m = 4: 301 blocks (odd total, ragged shards)
        M, m, nb = 64, 4, 301
        x = (rng.uniform(-.5, .5, nb * M // 2) + 1j * rng.uniform(-.5, .5, nb * M // 2)).astype(np.complex64)
        sh = lqshard.firpfbch2_plan(nb, world, M, m)[rank]
        q2 = O.FirPfbch2(O.ANALYZER, M, m, 60.0)
        seg = x[sh.first * M // 2:(sh.start + sh.count) * M // 2]
        y = q2.execute_block(seg).reshape(-1, M)[sh.warm:]
        parts = [None] * world
        dist.all_gather_object(parts, y)
        # firfilt h = 37 over 5000 samples
        h = rng.uniform(-.5, .5, 37).astype(np.float32)
        xf = (rng.uniform(-.5, .5, 5000) + 1j * rng.uniform(-.5, .5, 5000)).astype(np.complex64)
        shf = lqshard.firfilt_plan(len(xf), world, len(h))[rank]
        f = O.FirFilt(O.CRCF, h)
        yf = f.execute_block(xf[shf.first:shf.start + shf.count])[shf.warm:]
        parts_f = [None] * world
        dist.all_gather_object(parts_f, yf)
        # counters as bench.py reduces them
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        s = torch.tensor([float(sh.count)], dtype=torch.float64)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        if rank == 0:
            full = O.FirPfbch2(O.ANALYZER, M, m, 60.0).execute_block(x).reshape(-1, M)
            fullf = O.FirFilt(O.CRCF, h).execute_block(xf)
            ok = (np.array_equal(np.concatenate(parts), full) and np.array_equal(np.concatenate(parts_f), fullf)
                  and t.item() == world and s.item() == nb)
            q.put(ok)
    finally:
        dist.destroy_process_group()


def test_sharded_stream_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=10) is True


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_plans_cover_stream(world):
    sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))
    import lqshard
    for plan, n in ((lqshard.firpfbch2_plan(1001, world, 1024, 4), 1001),
                    (lqshard.firfilt_plan(12345, world, 64), 12345)):
        assert sum(s.count for s in plan) == n
        pos = 0
        for s in plan:
            assert s.start == pos and s.first >= 0
            pos += s.count
    for s in lqshard.firpfbch2_plan(1001, world, 1024, 4):
        assert s.start % 2 == 0 and s.warm % 2 == 0
