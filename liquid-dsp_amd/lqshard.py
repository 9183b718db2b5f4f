"""Time-sharding of one long stream across ranks (one process per GPU).

The streaming objects carry only a short history between calls:
  * firfilt        : the last h-1 inputs;
  * firpfbch2 (an.): the last 2mM - M/2 inputs and the block parity;
  * fftfilt        : the last h-1 inputs.
So a long stream splits into contiguous shards that need no data exchange:
each rank re-creates the state by running a short warm-up prefix (the halo)
through its own object and discarding those outputs, then processes its
shard.  firpfbch2 shards start on even block indices and the warm-up is a
whole, even number of blocks, so the parity of every block matches the
single-stream run.  No collective is needed on the data path; ranks only
all-reduce counters.

The planner is pure integer arithmetic (no GPU); it is used by bench.py's
sharded mode and checked against the single-stream oracle by
tests/test_multirank.py (gloo, world_size 2).
"""
from dataclasses import dataclass


@dataclass
class Shard:
    rank: int
    start: int        # first output unit owned (sample or block index)
    count: int        # units owned
    warm: int         # warm-up units processed before `start` (outputs discarded)

    @property
    def first(self):  # first unit processed (warm-up included)
        return self.start - self.warm


def _split(n_units, world, align=1):
    """Contiguous split of n_units into `world` parts, boundaries multiples of align."""
    per = -(-n_units // world)
    per = -(-per // align) * align
    out = []
    for r in range(world):
        a = min(n_units, r * per)
        b = min(n_units, a + per)
        out.append((a, b - a))
    return out


def firfilt_plan(n, world, h_len):
    """Shards of an n-sample firfilt stream; warm-up = h_len-1 samples."""
    halo = max(0, h_len - 1)
    return [Shard(r, a, c, min(halo, a)) for r, (a, c) in enumerate(_split(n, world))]


def firpfbch2_plan(nblocks, world, M, m):
    """Shards of an analyzer stream of `nblocks` blocks (M/2 inputs each).

    Every block depends on the latest 2mM inputs, i.e. on
    2mM/(M/2) = 4m blocks of input ending at its own; warm-up = 4m - 1 blocks
    rounded up to an even count so each shard starts on an even (global)
    block parity, matching the reference's `flag` sequence.
    """
    halo = 4 * m - 1
    halo += halo & 1
    return [Shard(r, a, c, min(halo, a)) for r, (a, c) in enumerate(_split(nblocks, world, align=2))]


def fftfilt_plan(n, world, h_len, block=1):
    """Shards of an fftfilt stream.  The output is the linear convolution
    (fftfilt.c:193-260 carries the last n inputs' tail), so the warm-up is
    h_len-1 samples; with `block` > 1 shard starts and the warm-up are whole
    multiples of the reference's block size n, for callers that must feed
    exactly n samples per execute() (the reference's own API)."""
    if block <= 1:
        return firfilt_plan(n, world, h_len)
    halo = -(-max(0, h_len - 1) // block) * block
    return [Shard(r, a, c, min(halo, a)) for r, (a, c) in enumerate(_split(n, world, align=block))]
