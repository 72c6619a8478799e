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
