"""Static keyspace sharding shared by bench.py and the multi-rank tests.

Every (ESSID, candidate) PMK is independent, so shards never exchange data.  Weak scaling (fixed work per GPU per
step): rank r of N owns shard r of the node's workload -- its own dictionary, ESSID set or ESSID -- so no two ranks
ever derive the same (ESSID, candidate) PMK however many ranks there are, and scans its shard batch by batch.
Strong scaling and crack_files split one keyspace or dictionary chunk into N contiguous equal ranges
(dwpa_amd/csrc/crack.cpp).  The only cross-rank traffic is the bench's control plane: a barrier around the timed
region, the max elapsed time and the total PMK count.
"""
from __future__ import annotations


def weak_units(rank: int, first_step: int, steps: int, nbatches: int, offset: int = 0):
    """(shard, batch) scanned by `rank` at each step: its own shard, step s -> batch (s + offset) mod nbatches."""
    return [(rank, (s + offset) % nbatches) for s in range(first_step, first_step + steps)]


def contiguous_shard(n: int, k: int, g: int):
    """[b, e) of shard k of g over n items (same split as crack.cpp: W*k/G .. W*(k+1)/G)."""
    return n * k // g, n * (k + 1) // g


def strong_batches(n: int, rank: int, world: int, batch: int):
    """Strong scaling: rank g's contiguous range [g*n/G, (g+1)*n/G) cut into the fewest
    batches of at most `batch` candidates, all of (nearly) equal size so no launch runs a thin last wave round.
    Returns [(first, count)]."""
    b, e = contiguous_shard(n, rank, world)
    m = e - b
    if m <= 0:
        return []
    nb = -(-m // max(1, batch))
    return [(b + m * j // nb, m * (j + 1) // nb - m * j // nb) for j in range(nb)]


def reduce_timing(dist, elapsed: float, done: float):
    """max elapsed and summed PMKs over ranks (gloo tensors on the CPU)."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(done)], dtype=torch.float64)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), float(c.item())


def all_ranks(dist, ok: bool) -> bool:
    """True on every rank iff `ok` is true on every rank (gloo MIN over the ranks' flags)."""
    import torch
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item() == 1.0)
