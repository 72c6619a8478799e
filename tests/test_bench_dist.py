"""bench.py's multi-rank logic on CPU (gloo, world_size 2): the timed region's max-over-ranks
wall time and the whole-job unit sum, and that ranks draw disjoint shards."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wall = [0.5, 0.75][rank]
    units = [1000.0, 3000.0][rank]
    out = bench.reduce_over_ranks(dist, torch, wall, units, torch.device("cpu"), world)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


def test_reduce_over_ranks_gloo_ws2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert res[r] == (0.75, 4000.0)


def test_reduce_single_rank_passthrough():
    assert bench.reduce_over_ranks(None, torch, 1.5, 42.0, None, 1) == (1.5, 42.0)


def test_shards_are_distinct():
    seeds = {bench.shard_seed(r) for r in range(8)}
    assert len(seeds) == 8
    g = [torch.Generator().manual_seed(bench.shard_seed(r)) for r in range(2)]
    a, b = (torch.rand((1024, 7), generator=x) for x in g)
    assert not torch.equal(a, b)


@pytest.mark.parametrize("n,world", [(1 << 20, 1), (1 << 20, 2), (1 << 20, 8), (1000003, 3), (5, 8)])
def test_strong_slices_partition_the_batch(n, world):
    """--scaling strong: the ranks' contiguous ranges cover the fixed batch exactly once, in order,
    with sizes differing by at most one."""
    parts = [bench.strong_slice(n, r, world) for r in range(world)]
    assert parts[0][0] == 0
    for (lo, m), (lo2, _) in zip(parts, parts[1:]):
        assert lo + m == lo2
    assert sum(m for _, m in parts) == n
    assert max(m for _, m in parts) - min(m for _, m in parts) <= 1


def _strong_worker(rank, world, port, q):
    """the same fixed batch on every rank (same seed), each rank its slice; gathering the slices in
    rank order reproduces the batch"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = torch.rand((1000, 7), generator=torch.Generator().manual_seed(bench.shard_seed(0)))
    lo, m = bench.strong_slice(1000, rank, world)
    mine = full[lo:lo + m].contiguous()
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([m], dtype=torch.int64))
    cap = int(max(sizes))
    pad = torch.zeros((cap, 7))
    pad[:m] = mine
    parts = [torch.zeros((cap, 7)) for _ in range(world)]
    dist.all_gather(parts, pad)
    ok = torch.equal(torch.cat([p[:int(s)] for p, s in zip(parts, sizes)]), full)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, ok))


def test_strong_slices_gloo_ws3():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_strong_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res.values())
