"""CPU, world_size 2 over gloo: the N>1 path of bench.py (static shards, barrier, max/sum reductions) and the
crack_files shard split.  No GPU: the data path has no collective, only these control-plane steps."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from dwpa_amd.shard import contiguous_shard, reduce_timing, weak_units


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = weak_units(rank, 2, 8, 6)
    gathered = [None] * world
    dist.all_gather_object(gathered, ids)
    dist.barrier()
    el, tot = reduce_timing(dist, 1.0 + rank, 100 * (rank + 1))
    q.put((rank, gathered, el, tot))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shards_disjoint_and_reductions(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, gathered, el, tot in res:
        assert el == float(world)                     # max over ranks
        assert tot == 100 * world * (world + 1) / 2   # sum over ranks
        # every rank scans its own shard, so no (shard, batch) unit is scanned by two ranks, even with more ranks
        # than batches per shard (8 ranks of a 6-batch dictionary on a node)
        for r, g in enumerate(gathered):
            assert all(tuple(u)[0] == r for u in g)
        units = [tuple(u) for g in gathered for u in g[:6]]
        assert len(set(units)) == len(units)


def test_weak_schedule_covers_each_shard():
    nb = 6
    for world in (1, 2, 8):
        for r in range(world):
            units = weak_units(r, 0, nb, nb)
            assert sorted(b for _, b in units) == list(range(nb)) and {s for s, _ in units} == {r}


def test_contiguous_shards():
    for n in (0, 1, 7, 100, 12345):
        for g in (1, 2, 3, 8):
            parts = [contiguous_shard(n, k, g) for k in range(g)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            for (b0, e0), (b1, e1) in zip(parts, parts[1:]):
                assert e0 == b1
            assert max(e - b for b, e in parts) - min(e - b for b, e in parts) <= 1


def _ok_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dwpa_amd.shard import all_ranks
    q.put((rank, all_ranks(dist, True), all_ranks(dist, rank != 1)))
    dist.destroy_process_group()


def test_all_ranks_verification():
    """bench.py's hits_verified over N ranks: true only if every rank found its own planted PSK."""
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ok_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(a is True and b is False for _, a, b in res)
