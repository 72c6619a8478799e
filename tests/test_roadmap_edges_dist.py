"""The sharded PRM edge stage (vamp_amd/roadmap.py: query_split, allgather_pairs, assemble) on
CPU with gloo, world_size 2 and 3.

Each rank produces the valid (vertex, neighbour) pairs of its query range with the C
restatement standing in for the GPU kNN + validate (test infrastructure only), then runs the
product's exchange and adjacency assembly.  Every rank must end with exactly the graph of the
single-process oracle build_roadmap (prm.hh:255-299): the same per-vertex lists in the same
append order and the same components.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vamp_amd import roadmap

F = np.float32


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem():
    import oracle_py as op
    rng = np.random.default_rng(31)
    env = op.sphere_cage_env()
    q = op.scale(rng.random((2000, 7), dtype=F))
    return op, env, q[op.fkcc_threads(env, q, threads=2)][:300]


def _shard_pairs(op, env, V, qf, qc):
    nbr, dist_, cnt = op.roadmap_knn(V, op.SPACE_MEASURE["panda"], threads=2)
    qi = np.concatenate([np.full(cnt[i], i) for i in range(qf, qf + qc)]).astype(np.int64) if qc else np.zeros(0, np.int64)
    m = np.concatenate([np.arange(cnt[i]) for i in range(qf, qf + qc)]).astype(np.int64) if qc else np.zeros(0, np.int64)
    qj = nbr[qi, m].astype(np.int64)
    ok, _ = op.robot_validate_motions("panda", env, V[qj], V[qi], threads=2) if len(qi) else (np.zeros(0, bool), None)
    return np.stack([qi[ok], qj[ok]], 1) if len(qi) else np.zeros((0, 2), np.int64)


def _worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(__file__)
    sys.path[:0] = [here, os.path.join(here, "..", "mr-vamp_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op, env, V = _problem()
    qf, qc = roadmap.query_split(len(V), rank, world)
    pairs = torch.from_numpy(_shard_pairs(op, env, V, qf, qc))
    allp = roadmap.allgather_pairs(torch, dist, pairs)
    off, adj, comp = roadmap.assemble(len(V), allp.numpy())
    dist.barrier()
    dist.destroy_process_group()
    out_q.put((rank, off, adj, comp))


def test_query_split_covers_and_balances():
    for n, world in ((1000, 8), (7, 3), (0, 2), (100000, 8)):
        parts = [roadmap.query_split(n, r, world) for r in range(world)]
        assert parts[0][0] == 0 and sum(c for _, c in parts) == n
        for (a, c), (b, _) in zip(parts, parts[1:]):
            assert a + c == b
        if n >= 1000:  # sum of prefix lengths per rank within 2 %
            w = [sum(range(a, a + c)) for a, c in parts]
            assert max(w) / min(w) < 1.02


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_edges_gloo(world):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    op, env, V = _problem()
    edges, _ = op.build_roadmap_edges("panda", env, V, threads=4)
    comp = op.components(len(V), edges)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, off, adj, cmp_ in res:
        got = [adj[off[i]:off[i + 1]].tolist() for i in range(len(V))]
        assert got == edges, rank
        assert np.array_equal(cmp_, comp), rank


def test_query_split_python_equals_c_abi():
    """roadmap.query_split (the torch path) and vgpu_query_split (the C collective) draw the same ranges"""
    from vamp_amd import roadmap
    for n in (0, 1, 2, 5, 99, 100000, 2681709, 4_000_000):
        for w in (1, 2, 3, 4, 7, 8):
            for r in range(w):
                assert roadmap.query_split(n, r, w) == roadmap.query_split_c(n, r, w), (n, r, w)
