#!/usr/bin/env python3
"""Headline benchmark: liquid-dsp's streaming channelizer / filter hot path on MI355X.

Metric (BASELINE.json): "Msamples/s: firfilt_crcf h=64 & firpfbch2_crcf M=1024;
%HBM roofline".

Workload of `value` (configs[3]): firpfbch2_crcf analyzer, M = 1024, m = 4,
Kaiser As = 60, one independent 128M-sample complex-float stream per GPU
(synthetic U(-0.5,0.5) data, resident in HBM before timing).  A step = one
firpfbch2_crcf_execute_block_dev() over the whole 128M-sample stream
(262,144 analyzer blocks, continuing the stream's state step after step).
`value` = input samples of all ranks / max-over-ranks time (Msamples/s).
The second headline workload, firfilt_crcf h=64 (configs[0] shape, 2^28
samples per GPU so the 4 GB working set is far above the 256 MB Infinity
Cache), is timed the same way and reported under "firfilt_crcf_h64".

Multi-GPU: one process per GPU.  `--gpus N` without a launcher starts N
child ranks itself (fresh interpreters, started before this process makes
any GPU call); under torch.distributed.run the env's RANK / WORLD_SIZE are
used.  Each rank binds its own GPU; the only collectives are RCCL
all-reduces of counters (max time, sample counts, checksums).  `value`:
independent 128M-sample streams, one per GPU (weak scaling).  Leg
"firpfbch2_sharded_stream": ONE 128M-sample stream split across the ranks
by liquid-dsp_amd/lqshard.py (even-block shard starts, a 16-block warm-up
halo recomputed per shard, no data exchange; strong scaling), with an
order-independent checksum of the owned outputs that must not change with N.

roofline: algorithmic bytes of the dominant kernel per launch (24 B per
input sample for the analyzer: 8 B read + 16 B written; 16 B per sample for
firfilt) / its average launch duration measured with HIP events on the
stream the kernel runs on; peak 8000 GB/s (MI355X HBM3E spec).

cpu_baseline: the CPU oracle (oracle/oracle.c, a plain-C port of the
reference firpfbch2.c analyzer, "kind": "port"; the reference itself cannot
be built in this image) timed on the host cores, rank 0 at
N=1 only: `value` = the aggregate of C processes each running its own
independent stream (C = the box's CPU share, stated in `cores`), beside the
one-core figure; bounded samples (~10 s + ~5 s).  The secondary legs carry
their own one-core oracle rates (firfilt, resamp, fftfilt, dotprod n=64).

Output: two JSON lines.  The first ("aux") holds the secondary records
(per-call legs, dotprod legs, the measured ceilings' launch shapes, the CPU
baseline detail); the LAST line is the headline record, kept short, with
firfilt_crcf_h64 as its final key.  Measured ceilings: hand-written HIP copy /
read / pattern kernels (tools/mb/bw_probe.hip) warmed up like the legs; each
roofline carries frac (of the 8 TB/s spec) beside frac_of_measured_copy and,
for the two headline kernels and fftfilt, frac_of_measured_pattern.

per_call: the reference's own per-call benchmark bodies
(src/*/bench/*_benchmark.c: push/execute one sample, one firpfbch2 block,
one dot product per call) compiled unchanged against this library by
tools/build_ref_benches.sh and timed in wall clock -- the unbatched liquid.h
API in the library's default mode (single-sample calls on the host, block
calls on the GPU); per_call_gpu: the same loops with every call forced onto
the GPU (one round trip per call).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))

import torch  # noqa: E402  (import before the library: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import liquidmi as LQ  # noqa: E402

HBM_PEAK_GBPS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--warmup-ms", type=float, default=150.0,
                   help="per-leg warm-up floor: untimed launches continue until this much wall time has passed")
    p.add_argument("--samples", type=int, default=1 << 27, help="firpfbch2 input samples per GPU")
    p.add_argument("--fir-samples", type=int, default=1 << 28, help="firfilt samples per GPU")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (rank 0, N=1)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-firfilt", action="store_true")
    p.add_argument("--rs-samples", type=int, default=1 << 25, help="resamp_crcf input samples per GPU")
    p.add_argument("--no-resamp", action="store_true")
    p.add_argument("--dp-vectors", type=int, default=1 << 20, help="dotprod_cccf vectors per GPU per n")
    p.add_argument("--ff-samples", type=int, default=1 << 26, help="fftfilt_crcf samples per GPU")
    p.add_argument("--no-extra", action="store_true", help="skip the dotprod / fftfilt legs")
    p.add_argument("--shard-samples", type=int, default=1 << 27,
                   help="length of the ONE firpfbch2 stream split across ranks (sharded leg)")
    p.add_argument("--no-shard", action="store_true", help="skip the single-stream sharded leg")
    p.add_argument("--no-percall", action="store_true", help="skip the per-call latency leg")
    p.add_argument("--no-ceilings", action="store_true", help="skip the measured HBM ceilings (probe kernels)")
    p.add_argument("--cpu-procs", type=int, default=0,
                   help="processes for the aggregate CPU baseline (0: the host CPU share, at most 16)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch (from a separate rocprofv3 --pmc run)")
    return p.parse_args()


def launch_ranks(n):
    """Start n ranks of this script as child processes (one per GPU) and
    return the worst exit code.  Runs before this process touches the GPU
    (no HIP call, no torch.cuda initialisation), so nothing is re-executed
    from a process holding a device context."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        if c != 0 and rc == 0:
            rc = c
            for q in procs:
                if q.poll() is None:
                    q.terminate()
    return rc


DEV_COLLECTIVES = True   # counters reduced over RCCL (device tensors) unless ranks share a GPU


def setup_dist():
    global DEV_COLLECTIVES
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev == 0:
        sys.exit("bench.py: no GPU visible (the library has no CPU path)")
    torch.cuda.set_device(local % ndev)
    if world > 1:
        # RCCL needs one GPU per rank; ranks sharing a GPU (a 1-GPU rehearsal
        # of --gpus N) reduce their counters over gloo instead
        DEV_COLLECTIVES = world <= ndev
        dist.init_process_group(backend="nccl" if DEV_COLLECTIVES else "gloo", init_method="env://")
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def _reduce(v, world, op, dtype=torch.float64):
    t = torch.tensor([v], dtype=dtype, device="cuda" if DEV_COLLECTIVES else "cpu")
    if world > 1:
        dist.all_reduce(t, op=op)
    return t.item()


def allreduce_max(v, world):
    return float(_reduce(v, world, dist.ReduceOp.MAX))


def allreduce_sum(v, world):
    return float(_reduce(v, world, dist.ReduceOp.SUM))


def allreduce_sum_i64(v, world):
    return int(_reduce(int(v), world, dist.ReduceOp.SUM, torch.int64))


def synth_complex(n, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    x = torch.rand(2 * n, generator=g, device="cuda", dtype=torch.float32) - 0.5
    return x


def synth_indexed(a, b, chunk=1 << 24):
    """Complex samples a..b-1 of ONE synthetic stream, as interleaved float32:
    a counter-based hash of the global float index, so any shard of the stream
    is generated identically on any rank, U[-0.5, 0.5) in steps of 2^-24."""
    out = torch.empty(2 * (b - a), dtype=torch.float32, device="cuda")
    for c0 in range(2 * a, 2 * b, chunk):
        c1 = min(2 * b, c0 + chunk)
        h = torch.arange(c0, c1, dtype=torch.int64, device="cuda")
        h = (h * 0x9E3779B1) & 0xFFFFFFFF
        h ^= h >> 15
        h = (h * 0x85EBCA77) & 0xFFFFFFFF
        h ^= h >> 13
        h = (h * 0xC2B2AE3D) & 0xFFFFFFFF
        h ^= h >> 16
        out[c0 - 2 * a:c1 - 2 * a] = (h >> 8).to(torch.float32) * (1.0 / (1 << 24)) - 0.5
        del h
    return out


WARMUP_FLOOR_MS = 150.0   # per leg: keep launching until clocks have ramped (set by --warmup-ms)


def time_steps(run_step, steps, warmup, world, stream, info=None):
    """W untimed warm-up steps, then further untimed steps until the leg has
    run for at least WARMUP_FLOOR_MS of wall time (the first launches after
    idle run 5-10 % slower while clocks ramp; the driver's --warmup 5 alone
    does not cover that), then exactly `steps` timed steps between a barrier
    + synchronize on both sides.  `info` (a dict) receives the warm-up count
    and duration."""
    t_w = time.perf_counter()
    nw = 0
    for _ in range(warmup):
        run_step()
        nw += 1
    stream.synchronize()
    while (time.perf_counter() - t_w) * 1e3 < WARMUP_FLOOR_MS:
        for _ in range(4):
            run_step()
            nw += 1
        stream.synchronize()
    warm_ms = (time.perf_counter() - t_w) * 1e3
    barrier(world)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        run_step()
    ev1.record(stream)
    barrier(world)
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if info is not None:
        info["warmup_launches"] = nw
        info["warmup_ms"] = warm_ms
    return wall, gpu_ms


def bench_firpfbch2(args, world, rank, stream):
    M, m = 1024, 4
    n = args.samples - args.samples % (M // 2)
    nblocks = n // (M // 2)
    x = synth_complex(n, 1234 + rank)
    y = torch.empty(2 * nblocks * M, dtype=torch.float32, device="cuda")
    q = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, m, 60.0)
    q.set_stream(stream.cuda_stream)

    def step():
        q.execute_block_dev(x.data_ptr(), nblocks, y.data_ptr())

    wi = {}
    wall, gpu_ms = time_steps(step, args.steps, args.warmup, world, stream, wi)
    res = {"n": n, "nblocks": nblocks, "wall": wall, "gpu_ms": gpu_ms, "warm": wi}
    q.destroy()
    del x, y
    torch.cuda.empty_cache()
    return res


def bench_firpfbch2_sharded(args, world, rank, stream):
    """ONE firpfbch2 analyzer stream of args.shard_samples samples split across
    the ranks: rank r owns blocks [start, start+count) of
    lqshard.firpfbch2_plan and runs its own object over [start-warm, start+count)
    -- a 16-block warm-up recomputed from its own slice of the stream, block
    parity preserved, no data exchange.  Checksum: sum of the int32 bit
    patterns of the owned outputs of a fresh object (exact, order-independent),
    identical for every N iff the sharded outputs equal the single-stream ones."""
    import lqshard
    M, m = 1024, 4
    nb_total = args.shard_samples // (M // 2)
    sh = lqshard.firpfbch2_plan(nb_total, world, M, m)[rank]
    nb = sh.warm + sh.count
    x = synth_indexed(sh.first * (M // 2), (sh.start + sh.count) * (M // 2))
    y = torch.empty(2 * max(nb, 1) * M, dtype=torch.float32, device="cuda")
    q = LQ.FirPfbch2(LQ.LIQUID_ANALYZER, M, m, 60.0)
    q.set_stream(stream.cuda_stream)

    def step():
        if nb:
            q.execute_block_dev(x.data_ptr(), nb, y.data_ptr())

    wi = {}
    wall, gpu_ms = time_steps(step, args.steps, args.warmup, world, stream, wi)
    q.reset()                      # checksum pass from the stream's initial state
    step()
    stream.synchronize()
    own = y[2 * sh.warm * M:2 * nb * M]
    csum = int(own.view(torch.int32).sum(dtype=torch.int64).item()) if sh.count else 0
    res = {"wall": wall, "gpu_ms": gpu_ms, "owned": sh.count * (M // 2), "halo_blocks": sh.warm,
           "total": nb_total * (M // 2), "checksum": csum, "warm": wi}
    q.destroy()
    del x, y, own
    torch.cuda.empty_cache()
    return res


def bench_firfilt(args, world, rank, stream):
    n = args.fir_samples
    x = synth_complex(n, 777 + rank)
    y = torch.empty(2 * n, dtype=torch.float32, device="cuda")
    g = torch.Generator()
    g.manual_seed(5)
    h = (torch.rand(64, generator=g) - 0.5).numpy()
    q = LQ.FirFilt("crcf", h)
    q.set_stream(stream.cuda_stream)

    def step():
        q.execute_block_dev(x.data_ptr(), n, y.data_ptr())

    wi = {}
    wall, gpu_ms = time_steps(step, args.steps, args.warmup, world, stream, wi)
    res = {"n": n, "wall": wall, "gpu_ms": gpu_ms, "warm": wi}
    q.destroy()
    del x, y
    torch.cuda.empty_cache()
    return res


def bench_dotprod(args, world, rank, stream):
    """configs[1]: dotprod_cccf n in {16,64,256,1024}, 2^20 vectors per GPU"""
    out = {}
    nvec = args.dp_vectors
    g = torch.Generator()
    g.manual_seed(11)
    # the config's 1M vectors at n = 16 / 64 are 134 MB / 537 MB: the n = 16
    # set fits the 256 MB Infinity Cache, so "n16_hbm" repeats it on 2^23
    # vectors (1 GiB) for an HBM figure
    for n, nv, key in ((16, nvec, 16), (64, nvec, 64), (256, nvec, 256), (1024, nvec, 1024),
                       (16, 8 * nvec, "16_hbm")):
        X = synth_complex(n * nv, 99 + n + rank)
        Y = torch.empty(2 * nv, dtype=torch.float32, device="cuda")
        h = ((torch.rand(n, generator=g) - 0.5) + 1j * (torch.rand(n, generator=g) - 0.5)).numpy()
        q = LQ.DotProd("cccf", h)
        q.set_stream(stream.cuda_stream)

        def step():
            q.execute_batch_dev(X.data_ptr(), nv, Y.data_ptr())

        wi = {}
        wall, gpu_ms = time_steps(step, args.steps, args.warmup, world, stream, wi)
        out[key] = {"wall": wall, "gpu_ms": gpu_ms, "n": n, "nvec": nv, "warm": wi}
        q.destroy()
        del X, Y
        torch.cuda.empty_cache()
    return {"nvec": nvec, "runs": out}


def bench_fftfilt(args, world, rank, stream):
    """configs[2]: fftfilt_crcf h=512 on 2^26 samples per GPU"""
    n = args.ff_samples
    x = synth_complex(n, 31337 + rank)
    y = torch.empty(2 * n, dtype=torch.float32, device="cuda")
    g = torch.Generator()
    g.manual_seed(17)
    h = (torch.rand(512, generator=g) - 0.5).numpy()
    q = LQ.FftFilt(h, 2048)
    q.set_stream(stream.cuda_stream)

    def step():
        q.execute_block_dev(x.data_ptr(), n, y.data_ptr())

    wi = {}
    wall, gpu_ms = time_steps(step, args.steps, args.warmup, world, stream, wi)
    q.destroy()
    del x, y
    torch.cuda.empty_cache()
    return {"n": n, "wall": wall, "gpu_ms": gpu_ms, "warm": wi}


def bench_resamp(args, world, rank, stream):
    """configs[4]: resamp_crcf r=1.037, npfb=64, m=7 on 32M samples per GPU"""
    n = args.rs_samples
    rate = 1.037
    x = synth_complex(n, 4242 + rank)
    y = torch.empty(2 * (int(n * rate) + 4096), dtype=torch.float32, device="cuda")
    # the kernels' first launches in the process (code-object loading), on
    # other objects and rates: 1.23 runs k_resamp4 as 1.037 does, 0.77 k_resamp3
    for wr in (1.23, 0.77):
        w = LQ.Resamp(wr, 7, 0.25, 60.0, 64)
        w.set_stream(stream.cuda_stream)
        w.execute_block_dev(x.data_ptr(), 1 << 15, y.data_ptr())
        stream.synchronize()
        w.destroy()
    q = LQ.Resamp(rate, 7, 0.25, 60.0, 64)
    q.set_stream(stream.cuda_stream)
    nys = []

    def step():
        nys.append(q.execute_block_dev(x.data_ptr(), n, y.data_ptr()))

    # first call of a fresh object: the timing plan (host walk of one period,
    # host/resamp.c) + upload + kernel, wall clock to the end of the stream
    t0 = time.perf_counter()
    step()
    stream.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    q.reset()                # the periodic plan from the initial state is kept
    nys.clear()
    wi = {}
    wall, gpu_ms = time_steps(step, args.steps, args.warmup, world, stream, wi)
    nout = sum(nys[-args.steps:])
    res = {"n": n, "wall": wall, "gpu_ms": gpu_ms, "nout": nout, "first_ms": first_ms, "warm": wi}
    q.destroy()
    del x, y
    torch.cuda.empty_cache()
    return res


PROBE_SO = os.path.join(ROOT, "tools", "mb", "bin", "libbwprobe.so")


def measured_ceilings(stream):
    """Hand-written HIP streaming kernels (tools/mb/bw_probe.hip), each a few
    launch shapes, every shape warmed up for the same 150 ms floor as the
    legs: the box's own rate for a plain 16-byte/lane copy, a read-only
    stream, firpfbch2's 1 read : 2 write tile pattern and firfilt's 1:1
    chunk pattern, with no arithmetic.  GB/s of algorithmic bytes, best shape."""
    import ctypes
    if not os.path.exists(PROBE_SO):
        return {"error": "tools/mb/bin/libbwprobe.so not built"}
    lib = ctypes.CDLL(PROBE_SO)
    lib.bwprobe_run.restype = ctypes.c_int
    lib.bwprobe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_int]
    src = torch.empty(1 << 29, dtype=torch.float32, device="cuda")   # 2 GiB
    dst = torch.empty(1 << 30, dtype=torch.float32, device="cuda")   # 4 GiB
    src.fill_(0.25)
    torch.cuda.synchronize()
    out, shapes = {}, {}
    # (key, probe kind, source bytes): copy / read over 1 GiB; the firpfbch2
    # pattern over the bench's 2^27 samples (1 GiB in, 2 GiB out); the firfilt
    # pattern over its 2^28 samples (2 GiB in, 2 GiB out)
    for key, kind, nbytes in (("copy", 0, 1 << 30), ("read", 1, 1 << 30), ("pfb2_pattern", 2, 1 << 30),
                              ("fir_pattern", 3, 1 << 31)):
        g, ms = ctypes.c_double(), ctypes.c_double()
        name = ctypes.create_string_buffer(512)
        rc = lib.bwprobe_run(kind, src.data_ptr(), dst.data_ptr(), nbytes, stream.cuda_stream, WARMUP_FLOOR_MS, 20,
                             ctypes.byref(g), ctypes.byref(ms), name, 512)
        if rc != 0:
            out[key] = None
            shapes[key] = "error %d" % rc
            continue
        out[key] = g.value
        shapes[key] = name.value.decode()
    del src, dst
    torch.cuda.empty_cache()
    return {"copy_GBps": out["copy"], "read_GBps": out["read"], "pfb2_pattern_GBps": out["pfb2_pattern"],
            "fir_pattern_GBps": out["fir_pattern"], "shapes": shapes}


def _cpu_pfb2_worker(seconds, seed, start_evt, out_q):
    """One independent firpfbch2 stream on one core (oracle port), for the
    aggregate CPU baseline."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np

    import oracle_lib as O
    q = O.FirPfbch2(O.ANALYZER, 1024, 4, 60.0)
    rng = np.random.default_rng(seed)
    chunk = 1 << 18
    x = (rng.uniform(-0.5, 0.5, chunk) + 1j * rng.uniform(-0.5, 0.5, chunk)).astype(np.complex64)
    start_evt.wait()
    done, t0 = 0, time.perf_counter()
    while True:
        q.execute_block(x)
        done += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    out_q.put((done, el))


def cpu_share():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var)
        if v and v.isdigit():
            n = min(n, int(v))
    return max(1, min(n, 16))


def cpu_baseline(seconds, procs):
    """Oracle firpfbch2 analyzer (M=1024, m=4): one core, then `procs`
    processes on independent streams (the reference is single-threaded; its
    multi-core figure is N streams in N processes)."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np

    import oracle_lib as O
    q = O.FirPfbch2(O.ANALYZER, 1024, 4, 60.0)
    rng = np.random.default_rng(9)
    chunk = 1 << 20
    x = (rng.uniform(-0.5, 0.5, chunk) + 1j * rng.uniform(-0.5, 0.5, chunk)).astype(np.complex64)
    done = 0
    t0 = time.perf_counter()
    while True:
        q.execute_block(x)
        done += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    single = {"value": done / el / 1e6, "unit": "Msamples/s", "cores": 1,
              "sample": "%d x 2^20 complex samples, %.1f s, 1 thread" % (done // chunk, el)}
    ctx = mp.get_context("spawn")
    evt, out_q = ctx.Event(), ctx.Queue()
    agg_s = seconds / 2
    ps = [ctx.Process(target=_cpu_pfb2_worker, args=(agg_s, 100 + i, evt, out_q)) for i in range(procs)]
    for p in ps:
        p.start()
    time.sleep(1.0)               # let every worker import and allocate before the start signal
    evt.set()
    res = [out_q.get(timeout=120 + 4 * agg_s) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    agg = sum(d for d, _ in res) / max(e for _, e in res) / 1e6
    return {"value": agg, "unit": "Msamples/s", "cores": procs, "kind": "port",
            "what": "oracle/oracle.c: plain-C port of the reference firpfbch2_crcf analyzer "
                    "(src/multichannel/src/firpfbch2.c:244-282), M=1024 m=4 As=60; the reference itself "
                    "is not buildable in this image (DESIGN.md (c))",
            "sample": "%d processes x one independent stream each, %.1f s, 2^18-sample blocks" % (procs, agg_s),
            "single_core": single,
            "reference_measured_in_survey": {"1_core": 22.9, "8_cores_8_streams": 135.0, "unit": "Msamples/s",
                                             "source": "BASELINE.md section 2"}}


def percall_baseline(force_gpu=False):
    """The reference's own per-call benchmark bodies linked against this
    library (tools/build_ref_benches.sh -> build/ref_bench/percall), wall
    clock; None when the harness was not built.  Default mode: the library's
    default (single-sample calls on the host, host/lq_small.c; block calls on
    the GPU).  force_gpu: LQ_SMALL_CALLS=gpu, every call a GPU round trip."""
    import subprocess
    exe = os.path.join(ROOT, "build", "ref_bench", "percall")
    if not os.path.exists(exe):
        return None
    names = ["firfilt_crcf_64", "dotprod_crcf_64", "dotprod_cccf_64", "firpfbch2_crcf_a1024",
             "firpfbch_crcf_a1024", "resamp_crcf_m8", "firdecim_crcf_m8_h32", "firinterp_crcf_m8_h32",
             "fftfilt_crcf_64", "windowcf_push_n64"]
    try:
        env = dict(os.environ)
        env.pop("LQ_SMALL_CALLS", None)
        if force_gpu:
            env["LQ_SMALL_CALLS"] = "gpu"
        out = subprocess.run([exe, "--runtime", "0.25"] + names, capture_output=True, text=True, timeout=240,
                             env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    # the reference's own `make bench` rates for the same bodies, one core of
    # the survey container (trials/s)
    ref = {"firfilt_crcf_64": 35.4e6, "dotprod_crcf_64": 62.7e6, "dotprod_cccf_64": 38.4e6,
           "firpfbch2_crcf_a1024": 41.5e3, "firpfbch_crcf_a1024": 31.1e3, "resamp_crcf_m8": 17.8e6,
           "firdecim_crcf_m8_h32": 22.4e6, "firinterp_crcf_m8_h32": 10.6e6, "fftfilt_crcf_64": 25.5e6}
    res = {}
    for line in out.stdout.splitlines():
        if line.startswith("{"):
            d = json.loads(line)
            name = d.pop("name")
            if name in ref and d.get("trials_per_s"):
                d["reference_trials_per_s"] = ref[name]
                d["vs_reference"] = d["trials_per_s"] / ref[name]
            res[name] = d
    if out.returncode != 0:
        res["error"] = "exit %d: %s" % (out.returncode, out.stderr[-300:])
    return res


def cpu_baselines_secondary(seconds):
    """Oracle rates for the secondary legs (configs[0], [1], [2], [4]) on one
    host core, each over a bounded sample of about `seconds` of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np

    import oracle_lib as O
    rng = np.random.default_rng(10)

    def cx(n):
        return (rng.uniform(-0.5, 0.5, n) + 1j * rng.uniform(-0.5, 0.5, n)).astype(np.complex64)

    def timed(fn, units_per_call, what, unit):
        done, t0 = 0, time.perf_counter()
        while True:
            fn()
            done += units_per_call
            el = time.perf_counter() - t0
            if el >= seconds:
                break
        return {"value": done / el / 1e6, "unit": unit, "cores": 1, "kind": "port",
                "sample": "%s, %d units (%.1f s, 1 thread)" % (what, done, el)}

    out = {}
    h64 = rng.uniform(-0.5, 0.5, 64).astype(np.float32)
    ff = O.FirFilt(O.CRCF, h64)
    x = cx(1 << 18)
    out["firfilt_crcf_h64"] = timed(lambda: ff.execute_block(x), len(x),
                                    "oracle firfilt_crcf h=64 execute_block on 2^18-sample blocks", "Msamples/s")
    rs = O.Resamp(1.037, 7, 0.25, 60.0, 64)
    out["resamp_crcf_r1037"] = timed(lambda: rs.execute_block(x), len(x),
                                     "oracle resamp_crcf r=1.037 m=7 npfb=64 on 2^18-sample blocks",
                                     "Msamples/s (input)")
    h512 = rng.uniform(-0.5, 0.5, 512).astype(np.float32)
    fq = O.FftFilt(O.CRCF, h512, 2048)
    xb = cx(2048)
    out["fftfilt_crcf_h512"] = timed(lambda: fq.execute(xb), 2048,
                                     "oracle fftfilt_crcf h=512 (n=2048, nfft=4096) execute per block",
                                     "Msamples/s")
    hd = cx(64)
    X = cx(64 * (1 << 14))
    out["dotprod_cccf_n64"] = timed(lambda: O.dotprod_batch(O.CCCF, hd, X), 1 << 14,
                                    "oracle dotprod_cccf n=64 over batches of 2^14 vectors", "M dot products/s")
    return out


def main():
    global WARMUP_FLOOR_MS
    args = parse()
    WARMUP_FLOOR_MS = args.warmup_ms
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world, rank, local = setup_dist()
    # a dedicated (non-null) stream: the library's objects launch on it and
    # the HIP events below are recorded on it
    stream = torch.cuda.Stream()

    pfb = bench_firpfbch2(args, world, rank, stream)
    t_pfb = allreduce_max(pfb["wall"], world)
    g_pfb = allreduce_max(pfb["gpu_ms"], world)
    tot_pfb = allreduce_sum(pfb["n"] * args.steps, world)

    shd = None
    if not args.no_shard:
        shd = bench_firpfbch2_sharded(args, world, rank, stream)
        t_shd = allreduce_max(shd["wall"], world)
        g_shd = allreduce_max(shd["gpu_ms"], world)
        owned_shd = allreduce_sum(shd["owned"], world)
        csum_shd = allreduce_sum_i64(shd["checksum"], world)

    fir = None
    if not args.no_firfilt:
        fir = bench_firfilt(args, world, rank, stream)
        t_fir = allreduce_max(fir["wall"], world)
        g_fir = allreduce_max(fir["gpu_ms"], world)
        tot_fir = allreduce_sum(fir["n"] * args.steps, world)

    rs = None
    if not args.no_resamp:
        rs = bench_resamp(args, world, rank, stream)
        first_rs = allreduce_max(rs["first_ms"], world)
        t_rs = allreduce_max(rs["wall"], world)
        g_rs = allreduce_max(rs["gpu_ms"], world)
        tot_rs = allreduce_sum(rs["n"] * args.steps, world)

    dp = ff = None
    if not args.no_extra:
        dp = bench_dotprod(args, world, rank, stream)
        ff = bench_fftfilt(args, world, rank, stream)
        dp_t = {n: (allreduce_max(r["wall"], world), allreduce_max(r["gpu_ms"], world)) for n, r in dp["runs"].items()}
        ff_t = (allreduce_max(ff["wall"], world), allreduce_max(ff["gpu_ms"], world))

    ceil = measured_ceilings(stream) if rank == 0 and not args.no_ceilings else None
    percall = percall_gpu = None
    if rank == 0 and world == 1 and not args.no_percall:
        percall = percall_baseline()
        percall_gpu = percall_baseline(force_gpu=True)
    cpu = cpu2 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_procs or cpu_share())
        cpu2 = cpu_baselines_secondary(args.cpu_seconds / 4)

    if rank == 0:
        tj, tsrc = {}, None
        if os.path.exists(args.traffic_json):
            with open(args.traffic_json) as f:
                tj = json.load(f)
            # the PMC bytes are not counted in this timed run: separate
            # rocprofv3 --pmc passes over the same launch shapes wrote them
            tsrc = "%s (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, separate passes%s)" % (
                os.path.relpath(args.traffic_json, ROOT), (", " + tj["measured"]) if tj.get("measured") else "")
        copy_gbps = ceil.get("copy_GBps") if ceil else None

        def roof(alg_bytes, launch_ms, traffic, pattern_key=None):
            ach = alg_bytes / (launch_ms * 1e-3) / 1e9
            r = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS,
                 "traffic": traffic, "launch_ms": launch_ms, "alg_bytes": alg_bytes}
            if copy_gbps:
                r["frac_of_measured_copy"] = ach / copy_gbps
            if pattern_key and ceil and ceil.get(pattern_key):
                r["frac_of_measured_pattern"] = ach / ceil[pattern_key]
            return r

        # ---- secondary records first, on their own stdout line, so the final
        # line (the one the driver parses from its stdout tail) stays short
        aux = {"aux": "bench.py secondary records (the headline line follows)"}
        if ceil:
            aux["measured_ceilings"] = ceil
        if dp is not None:
            legs = {}
            for key, (tw, tg) in dp_t.items():
                ms = tg / args.steps
                n, nv = dp["runs"][key]["n"], dp["runs"][key]["nvec"]
                legs["n%s" % key] = {"value": world * nv * args.steps / tw / 1e6, "unit": "M dot products/s",
                                     "vectors": nv, "working_set_MB": (8.0 * n + 8.0) * nv / 1e6,
                                     "launch_ms": ms, "achieved_GBps": (8.0 * n + 8.0) * nv / (ms * 1e-3) / 1e9,
                                     "frac": (8.0 * n + 8.0) * nv / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                                     "warmup_launches": dp["runs"][key]["warm"]["warmup_launches"]}
            aux["dotprod_cccf"] = {"workload": "dotprod_cccf batched, %d vectors/GPU (BASELINE configs[1]); n16_hbm: "
                                               "n=16 on 8x the vectors (beyond the 256 MB Infinity Cache)"
                                               % dp["nvec"], "bytes_per_unit": "8n+8 B/vector", "legs": legs}
            if cpu2 and "dotprod_cccf_n64" in cpu2:
                aux["dotprod_cccf"]["cpu_baseline"] = cpu2["dotprod_cccf_n64"]
        if percall is not None:
            aux["per_call"] = {"what": "the reference's per-call benchmark loops (src/*/bench/*_benchmark.c) linked "
                                       "against this library, default mode (single-sample calls on the host, "
                                       "host/lq_small.c; block calls on the GPU); wall clock", "runs": percall}
        if percall_gpu is not None:
            aux["per_call_gpu"] = {"what": "the same loops with LQ_SMALL_CALLS=gpu: every call one GPU round trip",
                                   "runs": percall_gpu}
        if cpu is not None:
            aux["cpu_baseline_detail"] = cpu
        print(json.dumps(aux), flush=True)

        # ---- the headline line
        launch_ms = g_pfb / args.steps
        out = {
            "metric": "Msamples/s: firfilt_crcf h=64 & firpfbch2_crcf M=1024; %HBM roofline",
            "value": tot_pfb / t_pfb / 1e6,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_pfb / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic U(-0.5,0.5) complex float32, HBM resident",
            "config": {"workload": "firpfbch2_crcf analyzer M=1024 m=4 As=60, %d samples/GPU (BASELINE configs[3])"
                                   % pfb["n"], "M": 1024, "m": 4, "samples_per_gpu": pfb["n"],
                       "blocks_per_step": pfb["nblocks"], "parallelism": "stream-per-gpu x%d" % world},
            "roofline": dict(roof(24.0 * pfb["n"], launch_ms, tj.get("firpfbch2_bytes_per_launch"), "pfb2_pattern_GBps"),
                             bytes_per_unit="24 B/input sample (8 read + 16 write)", traffic_source=tsrc),
            "measured_copy_GBps": copy_gbps,
            "measured_pfb2_pattern_GBps": ceil.get("pfb2_pattern_GBps") if ceil else None,
            "measured_fir_pattern_GBps": ceil.get("fir_pattern_GBps") if ceil else None,
            "measured_read_GBps": ceil.get("read_GBps") if ceil else None,
            "warmup_floor": {"floor_ms": WARMUP_FLOOR_MS, "launches": pfb["warm"]["warmup_launches"],
                             "ms": pfb["warm"]["warmup_ms"]},
        }
        if cpu is not None:
            out["cpu_baseline"] = {k: cpu[k] for k in ("value", "unit", "cores", "kind", "sample")}
            out["cpu_baseline"]["single_core"] = cpu["single_core"]["value"]
            out["cpu_baseline"]["what"] = ("oracle/oracle.c port of firpfbch2.c:244-282 (the reference is not "
                                           "buildable here); detail on the preceding aux line")
        if shd is not None:
            out["firpfbch2_sharded_stream"] = {
                "value": owned_shd * args.steps / t_shd / 1e6, "unit": "Msamples/s", "scaling": "strong",
                "total_samples": shd["total"], "ranks": world, "halo_blocks": shd["halo_blocks"],
                "ms_per_step": t_shd / args.steps * 1e3, "launch_ms": g_shd / args.steps,
                "owned_samples": int(owned_shd), "output_checksum": csum_shd}
        if rs is not None:
            rl_ms = g_rs / args.steps
            out["resamp_crcf_r1037"] = {"value": tot_rs / t_rs / 1e6, "unit": "Msamples/s (input)",
                                        "workload": "resamp_crcf r=1.037 m=7 npfb=64 (BASELINE configs[4])",
                                        "samples_per_gpu": rs["n"], "outputs_per_step": rs["nout"] / args.steps,
                                        "ms_per_step": t_rs / args.steps * 1e3, "first_call_ms": first_rs,
                                        "roofline": dict(roof(8.0 * rs["n"] + 8.0 * rs["nout"] / args.steps, rl_ms,
                                                              tj.get("resamp_bytes_per_launch")),
                                                         bytes_per_unit="8 B/input + 8 B/output")}
            if cpu2 and "resamp_crcf_r1037" in cpu2:
                out["resamp_crcf_r1037"]["cpu_baseline"] = cpu2["resamp_crcf_r1037"]
        if ff is not None:
            ms = ff_t[1] / args.steps
            out["fftfilt_crcf_h512"] = {"value": world * ff["n"] * args.steps / ff_t[0] / 1e6, "unit": "Msamples/s",
                                        "workload": "fftfilt_crcf h=512 overlap-save, %d samples/GPU "
                                                    "(BASELINE configs[2])" % ff["n"],
                                        "roofline": dict(roof(16.0 * ff["n"], ms, tj.get("fftfilt_bytes_per_launch"),
                                                              "fir_pattern_GBps"), bytes_per_unit="16 B/sample")}
            if cpu2 and "fftfilt_crcf_h512" in cpu2:
                out["fftfilt_crcf_h512"]["cpu_baseline"] = cpu2["fftfilt_crcf_h512"]
        if dp is not None:
            out["dotprod_cccf_frac"] = {k: round(v["frac"], 4) for k, v in aux["dotprod_cccf"]["legs"].items()}
        if fir is not None:
            # last key of the line: the second headline workload
            fl_ms = g_fir / args.steps
            out["firfilt_crcf_h64"] = {"value": tot_fir / t_fir / 1e6, "unit": "Msamples/s",
                                       "workload": "firfilt_crcf h=64 execute_block_dev, %d samples/GPU" % fir["n"],
                                       "samples_per_gpu": fir["n"], "ms_per_step": t_fir / args.steps * 1e3,
                                       "warmup_launches": fir["warm"]["warmup_launches"],
                                       "arith": "f32-accurate three-term bf16 split on v_mfma_f32_16x16x32_bf16",
                                       "roofline": dict(roof(16.0 * fir["n"], fl_ms, tj.get("firfilt_bytes_per_launch"),
                                                             "fir_pattern_GBps"), bytes_per_unit="16 B/sample",
                                                        traffic_source=tsrc)}
            if cpu2 and "firfilt_crcf_h64" in cpu2:
                out["firfilt_crcf_h64"]["cpu_baseline"] = cpu2["firfilt_crcf_h64"]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
