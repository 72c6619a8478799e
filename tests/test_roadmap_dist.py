"""PRM vertex stage sharding and its all-gather (vamp_amd/roadmap.py) on CPU with gloo,
world_size 2 and 3.

Each rank produces its shard's valid vertices with the C restatement standing in for the
GPU sampling kernel (test infrastructure only: Halton<8> -> scale -> fkcc on the MBM Fetch
table scene), then runs the product's allgather_vertices.  Every rank must end with exactly the
sequence the reference's build_roadmap loop appends (prm.hh:235-254): valid samples in draw
order -- the single-process oracle run over all draws.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vamp_amd import roadmap


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


N_DRAWS, FIRST = 5000, 999_000  # spans the Halton reset at 1e6


def _shard_rows(lo, n):
    import oracle_py as op
    from conftest import golden
    from test_oracle_fetch import fetch_env
    env = fetch_env(op, golden("fetch_table_pick.npz"))
    q = op.robot_scale("fetch", op.halton(8, np.arange(lo, lo + n))) if n else np.zeros((0, 8), np.float32)
    ok = op.robot_fkcc_threads("fetch", env, q, threads=2) if n else np.zeros(0, bool)
    return q[ok], (np.nonzero(ok)[0] + lo).astype(np.int64)


def _worker(rank, world, port, out_q):
    import sys
    sys.path[:0] = [os.path.join(os.path.dirname(__file__)), os.path.join(os.path.dirname(__file__), "..", "mr-vamp_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, n = roadmap.shard_range(N_DRAWS, rank, world, FIRST)
    rows, draws = _shard_rows(lo, n)
    cnt = len(rows)
    pad = 7  # rows beyond `count` must be ignored
    rows_t = torch.cat([torch.from_numpy(rows), torch.full((pad, 8), 9.0)])
    draws_t = torch.cat([torch.from_numpy(draws), torch.full((pad,), -5, dtype=torch.int64)])
    R, D = roadmap.allgather_vertices(torch, dist, rows_t, draws_t, cnt)
    dist.barrier()
    dist.destroy_process_group()
    out_q.put((rank, R.numpy(), D.numpy()))


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_vertices_gloo(world):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, R, D = q.get(timeout=240)
        res[r] = (R, D)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_r, want_d = _shard_rows(FIRST, N_DRAWS)
    for r in range(world):
        R, D = res[r]
        assert np.array_equal(D, want_d)
        assert np.array_equal(R.view(np.uint32), want_r.view(np.uint32))


def test_shard_range_covers_draws_once():
    for n, w in ((10, 3), (4_000_000, 8), (5, 8), (0, 2)):
        got = []
        for r in range(w):
            lo, c = roadmap.shard_range(n, r, w, 1)
            got.extend(range(lo, lo + c))
        assert got == list(range(1, n + 1))
