"""Full-size oracle comparisons, split across host processes (test infrastructure).

The CPU oracle (oracle/oracle.c) is single-threaded; at BASELINE sizes (2^27
firpfbch2 samples, 2^28 firfilt samples) one core would need tens of seconds.
The stream is therefore split with the same shard plans the multi-GPU path
uses (liquid-dsp_amd/lqshard.py): every worker re-creates the oracle's state
from a warm-up halo, computes its shard and compares it with the GPU output.
Input and GPU output are handed over as read-only memory-mapped files in
/dev/shm; workers are started with the "spawn" method, so none of them
inherits the parent's GPU context.  Each worker returns (max |gpu - oracle|,
max |oracle|, count of non-finite mismatches) over its shard.
"""
import multiprocessing as mp
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _paths():
    for p in (HERE, os.path.join(ROOT, "liquid-dsp_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _worker(job):
    _paths()
    import lqshard  # noqa: F401
    import oracle_lib as O
    kind, xpath, ypath, n_x, n_y, args, sh = job
    x = np.memmap(xpath, dtype=np.complex64, mode="r", shape=(n_x,))
    y = np.memmap(ypath, dtype=np.complex64, mode="r", shape=(n_y,))
    if kind == "firpfbch2":
        M, m = args
        h2 = M // 2
        q = O.FirPfbch2(O.ANALYZER, M, m, 60.0)
        ref = q.execute_block(np.asarray(x[sh["first"] * h2:(sh["start"] + sh["count"]) * h2]))
        ref = ref[sh["warm"] * M:]
        got = np.asarray(y[sh["start"] * M:(sh["start"] + sh["count"]) * M])
    elif kind == "firfilt":
        (h,) = args
        q = O.FirFilt(O.CRCF, np.asarray(h, np.float32))
        ref = q.execute_block(np.asarray(x[sh["first"]:sh["start"] + sh["count"]]))[sh["warm"]:]
        got = np.asarray(y[sh["start"]:sh["start"] + sh["count"]])
    elif kind == "fftfilt":
        h, n = args
        q = O.FftFilt(O.CRCF, np.asarray(h, np.float32), n)
        ref = q.execute_stream(np.asarray(x[sh["first"]:sh["start"] + sh["count"]]))[sh["warm"]:]
        got = np.asarray(y[sh["start"]:sh["start"] + sh["count"]])
    else:
        raise ValueError(kind)
    fin = np.isfinite(ref) & np.isfinite(got)
    d = float(np.max(np.abs(got[fin] - ref[fin]))) if fin.any() else 0.0
    r = float(np.max(np.abs(ref[fin]))) if fin.any() else 0.0
    bad = int(np.count_nonzero(np.isfinite(ref) != np.isfinite(got)))
    return d, r, bad


def workers():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def compare(kind, x, y, args, plan):
    """Run the oracle over `plan` (lqshard shards) in parallel; return the
    normwise error max|d| / max|ref| and the count of finite/non-finite
    disagreements."""
    d = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    xp, yp = os.path.join(d, "x.c64"), os.path.join(d, "y.c64")
    try:
        x.astype(np.complex64, copy=False).tofile(xp)
        y.astype(np.complex64, copy=False).tofile(yp)
        jobs = [(kind, xp, yp, len(x), len(y), args,
                 {"first": s.first, "start": s.start, "count": s.count, "warm": s.warm}) for s in plan if s.count]
        with mp.get_context("spawn").Pool(min(len(jobs), workers())) as pool:
            res = pool.map(_worker, jobs)
    finally:
        for p in (xp, yp):
            if os.path.exists(p):
                os.remove(p)
        os.rmdir(d)
    dmax = max(r[0] for r in res)
    rmax = max(r[1] for r in res)
    return dmax / rmax if rmax > 0 else dmax, sum(r[2] for r in res)
