"""PRM roadmap vertex stage, sharded over the GPUs of one node.

Reference: ``Roadmap::build_roadmap`` (src/impl/vamp/planning/prm.hh:197-299) draws
``rng->next()`` (Halton<dim>), scales it (``Robot::scale_configuration``), checks it with
``Robot::fkcc`` on the configuration broadcast to the rake (prm.hh:246-254) and appends every
valid sample to the roadmap in draw order, after the start and goal vertices (prm.hh:228-233).

Here the draws 1..N are split into contiguous ranges, one per rank (one process per GPU).  Each
rank runs the fused Halton -> scale -> fkcc kernel over its range and compacts its valid rows on
the device (vgpu_sample_fkcc + vgpu_compact).  One exchange step follows: an all-gather of the
per-rank counts, then an all-gather of the count-padded rows and draw indices
(torch.distributed, backend "nccl" = RCCL over xGMI on MI355X).  Concatenated in rank order, the
result is exactly the reference's vertex sequence: valid samples in draw order.

The kernels run on the context's stream; set it to torch's current stream
(``Context.set_stream``) so the collective is ordered after them.  There is no CPU fallback:
without the HIP library the calls raise.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import numpy as np


def shard_range(n_draws: int, rank: int, world: int, first: int = 1) -> Tuple[int, int]:
    """(first draw index, count) of this rank's contiguous slice of draws first..first+n-1."""
    chunk = (n_draws + world - 1) // world
    lo = min(n_draws, rank * chunk)
    hi = min(n_draws, lo + chunk)
    return first + lo, hi - lo


def allgather_vertices(torch, dist, rows, draws, count: int, group=None):
    """Exchange the ranks' compacted vertices.  rows [>= count, dim] float32 and draws
    [>= count] int64 (this rank's first `count` entries valid) -> (all rows, all draws) in rank
    order.  Two collectives: counts, then the rows and draw indices padded to the largest count
    (one all_gather_into_tensor each).  Works on CUDA tensors (RCCL) and CPU tensors (gloo)."""
    world = dist.get_world_size(group)
    dev = rows.device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    cnts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(cnts, cnt, group=group)
    counts = [int(c) for c in cnts.tolist()]
    mx = max(counts) if counts else 0
    dim = rows.shape[1]
    send_r = torch.zeros((mx, dim), dtype=rows.dtype, device=dev)
    send_d = torch.zeros(mx, dtype=torch.int64, device=dev)
    if count:
        send_r[:count] = rows[:count]
        send_d[:count] = draws[:count]
    recv_r = torch.empty((world * mx, dim), dtype=rows.dtype, device=dev)
    recv_d = torch.empty(world * mx, dtype=torch.int64, device=dev)
    if mx:
        dist.all_gather_into_tensor(recv_r, send_r, group=group)
        dist.all_gather_into_tensor(recv_d, send_d, group=group)
    keep = torch.cat([torch.arange(r * mx, r * mx + c, device=dev) for r, c in enumerate(counts)]) \
        if sum(counts) else torch.empty(0, dtype=torch.int64, device=dev)
    return recv_r.index_select(0, keep), recv_d.index_select(0, keep)


def sample_valid_shard(torch, robot, environment, first: int, n: int, ctx, device):
    """This rank's slice: fused Halton<dim> -> scale -> fkcc over draws first..first+n-1, then
    device compaction.  Returns (rows [n, dim] with `count` valid leading rows, draws [n] int64,
    count).  GPU only."""
    dim = robot.dimension()
    q = torch.empty((max(n, 1), dim), dtype=torch.float32, device=device)
    valid = torch.empty(max(n, 1), dtype=torch.uint8, device=device)
    rows = torch.empty_like(q)
    idx = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    count = 0
    if n:
        robot.sample_fkcc_device(first, n, environment, q.data_ptr(), valid.data_ptr(), ctx)
        from . import compact_device
        count = compact_device(q.data_ptr(), valid.data_ptr(), n, dim, rows.data_ptr(), idx.data_ptr(), ctx)
    draws = idx.long() + first
    return rows, draws, count


def roadmap_vertices(robot, environment, n_draws: int, first: int = 1, start=None, goal=None,
                     max_samples: Optional[int] = None, ctx=None, group=None):
    """Vertices of ``build_roadmap`` after ``n_draws`` sampler iterations (prm.hh:235-254):
    [start, goal,] then every valid Halton sample in draw order, truncated at max_samples
    vertices like the reference loop.  Runs sharded when torch.distributed is initialised (one
    rank per GPU), single-GPU otherwise.  Returns (vertices [M, dim], draw_index [M]) as CUDA
    tensors; draw_index is -1 for start/goal."""
    import torch
    import torch.distributed as dist

    from . import context

    ctx = ctx or context()
    device = torch.device("cuda", torch.cuda.current_device())
    ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
    sharded = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if sharded else (0, 1)
    lo, n = shard_range(n_draws, rank, world, first)
    rows, draws, count = sample_valid_shard(torch, robot, environment, lo, n, ctx, device)
    if sharded:
        rows, draws = allgather_vertices(torch, dist, rows, draws, count, group)
    else:
        rows, draws = rows[:count], draws[:count]
    head = []
    if start is not None and goal is not None:
        head = [torch.as_tensor(start, dtype=torch.float32, device=device).reshape(1, -1),
                torch.as_tensor(goal, dtype=torch.float32, device=device).reshape(1, -1)]
    if head:
        rows = torch.cat(head + [rows])
        draws = torch.cat([torch.full((2,), -1, dtype=torch.int64, device=device), draws])
    if max_samples is not None:
        rows, draws = rows[:max_samples], draws[:max_samples]
    return rows, draws


# ---- edge stage (prm.hh:255-299) ----------------------------------------------------------------
def prm_neighbor_params(dim: int, space_measure: float, n: int, gamma_scale: float = 2.0):
    """PRMStarNeighborParams (roadmap.hh:42-77) for roadmap sizes 0 .. n-1: (k[n], r[n])."""
    from . import _lib
    from ._lib import check, load
    k = np.zeros(n, np.uint32)
    r = np.zeros(n, np.float32)
    check(load().vgpu_prm_neighbor_params(dim, float(space_measure), float(gamma_scale), n,
                                          k.ctypes.data_as(_lib.U32P), r.ctypes.data_as(_lib.F32P)))
    return k, r


def cpu_knn(V, queries, space_measure: float, gamma_scale: float = 2.0, kmax=None, threads: int = 0):
    """build_roadmap's causal neighbour queries of the listed vertices on the host CPU (exact k-d tree,
    vgpu_cpu_roadmap_knn): (nbr [m, kmax], dist [m, kmax], cnt [m]) -- the lists vgpu_roadmap_knn gives."""
    from . import _lib
    from ._lib import check, load
    V = np.ascontiguousarray(V, np.float32)
    n, dim = V.shape
    q = np.ascontiguousarray(queries, np.uint32).ravel()
    k, r = prm_neighbor_params(dim, space_measure, n, gamma_scale)
    kmax = int(kmax or max(1, int(k.max()) if n else 1))
    nbr = np.zeros((max(len(q), 1), kmax), np.uint32)
    dist = np.zeros((max(len(q), 1), kmax), np.float32)
    cnt = np.zeros(max(len(q), 1), np.uint32)
    check(load().vgpu_cpu_roadmap_knn(dim, V.ctypes.data_as(_lib.F32P), n, q.ctypes.data_as(_lib.U32P), len(q),
                                      k.ctypes.data_as(_lib.U32P), r.ctypes.data_as(_lib.F32P), kmax,
                                      nbr.ctypes.data_as(_lib.U32P), dist.ctypes.data_as(_lib.F32P),
                                      cnt.ctypes.data_as(_lib.U32P), int(threads)))
    return nbr[:len(q)], dist[:len(q)], cnt[:len(q)]


class Roadmap:
    """Roadmap<dim> (prm.hh:285-299): vertices [n, dim] and, per vertex, the indices of its
    neighbours in the order build_roadmap appended them; plus the connected components."""

    def __init__(self, vertices, offsets, adj, component):
        self.vertices = vertices
        self.offsets = offsets
        self.adj = adj
        self.component = component
        self.nanoseconds = 0  # Roadmap::nanoseconds / iterations (plan.hh:182-188), set by Robot.roadmap
        self.iterations = 0

    # the Python face of the reference's Roadmap (bindings/common.hh:550-574)
    def __len__(self) -> int:
        return len(self.vertices)

    def __getitem__(self, i):
        return self.vertices[i]

    def __iter__(self):
        return iter(self.vertices)

    @property
    def edges(self) -> List[List[int]]:
        o = self.offsets
        return [self.adj[o[i]:o[i + 1]].tolist() for i in range(len(o) - 1)]

    def n_edges(self) -> int:
        return int(self.offsets[-1]) // 2


def build_roadmap_edges(robot, environment, vertices, gamma_scale: float = 2.0, space_measure=None,
                        ctx=None) -> Roadmap:
    """The graph of Roadmap::build_roadmap over a given vertex sequence (start, goal, valid samples
    in draw order): every vertex's PRM* neighbour query and validate_motion of every candidate
    edge on the GPU (vgpu_build_roadmap_host), adjacency in the reference's append order."""
    import ctypes as C

    from . import _lib, context
    from ._lib import check, load
    ctx = ctx or context()
    V = np.ascontiguousarray(vertices, np.float32).reshape(-1, robot.dimension())
    n = V.shape[0]
    sm = robot.space_measure() if space_measure is None else float(space_measure)
    k, _ = prm_neighbor_params(robot.dimension(), sm, n, gamma_scale)
    cap = 2 * int(k.astype(np.int64).sum())
    offsets = np.zeros(n + 1, np.uint64)
    adj = np.zeros(max(cap, 1), np.uint32)
    comp = np.zeros(max(n, 1), np.uint32)
    n_adj = C.c_size_t()
    check(load().vgpu_build_roadmap_host(ctx.h, C.byref(robot.c_robot), environment.handle(ctx),
                                         V.ctypes.data_as(_lib.F32P), n, sm, float(gamma_scale),
                                         offsets.ctypes.data_as(C.POINTER(C.c_size_t)),
                                         adj.ctypes.data_as(_lib.U32P), adj.shape[0], C.byref(n_adj),
                                         comp.ctypes.data_as(_lib.U32P)), ctx.h)
    return Roadmap(V, offsets.astype(np.int64), adj[:n_adj.value], comp[:n])


def build_roadmap(robot, start, goal, environment, max_iterations: int = 100000, max_samples: int = 100000,
                  gamma_scale: float = 2.0, ctx=None, group=None) -> Roadmap:
    """Roadmap::build_roadmap (prm.hh:197-299) with the Halton sampler: vertices = start, goal and
    the valid samples of draws 1..max_iterations, at most max_samples vertices (the sampling
    stage sharded over ranks when torch.distributed is initialised), then the edge stage."""
    rows, _ = roadmap_vertices(robot, environment, max_iterations, 1, start, goal, max_samples, ctx, group)
    return build_roadmap_edges(robot, environment, rows.cpu().numpy(), gamma_scale, None, ctx)


# ---- the edge stage sharded over ranks (every rank holds all vertices after the all-gather) ----
def query_split(n: int, rank: int, world: int) -> Tuple[int, int]:
    """(first, count) of this rank's queries: contiguous ranges with equal sum of prefix lengths
    (query i scans i candidates), boundaries at floor(n * sqrt(r / world) + 0.5) -- the same double
    expression as the C ABI's vgpu_query_split (vgpu_prm_edges_allgather's split)."""
    b = [0] + [min(n, int(math.floor(n * math.sqrt(r / world) + 0.5))) for r in range(1, world)] + [n]
    return b[rank], b[rank + 1] - b[rank]


def edges_shard(torch, robot, environment, V, k, r, kmax: int, q_first: int, q_count: int, ctx):
    """This rank's share of build_roadmap's edge stage on the GPU: neighbour queries of vertices
    q_first .. q_first+q_count-1, then validate_motion(neighbor, vertex) of their candidates.
    V [n, dim], k [n], r [n] are device tensors (all vertices).  Returns the valid (vertex,
    neighbour) pairs in query order, nearest first: int32 tensor [m, 2]."""
    from ._lib import check, load
    dev = V.device
    n, dim = V.shape
    nbr = torch.empty((max(q_count, 1), kmax), dtype=torch.int32, device=dev)
    dist_ = torch.empty((max(q_count, 1), kmax), dtype=torch.float32, device=dev)
    cnt = torch.zeros(max(q_count, 1), dtype=torch.int32, device=dev)
    if q_count == 0:
        return torch.zeros((0, 2), dtype=torch.int32, device=dev)
    check(load().vgpu_roadmap_knn_range(ctx.h, dim, V.data_ptr(), n, q_first, q_count, k.data_ptr(), r.data_ptr(),
                                        kmax, nbr.data_ptr(), dist_.data_ptr(), cnt.data_ptr()), ctx.h)
    cnt = cnt[:q_count]
    off = torch.zeros(q_count + 1, dtype=torch.int32, device=dev)
    off[1:] = torch.cumsum(cnt, 0)
    E = int(off[-1])
    if E == 0:
        return torch.zeros((0, 2), dtype=torch.int32, device=dev)
    starts = torch.empty((E, dim), dtype=torch.float32, device=dev)
    goals = torch.empty_like(starts)
    check(load().vgpu_roadmap_edge_gather(ctx.h, dim, V.data_ptr(), q_first, q_count, nbr.data_ptr(), kmax,
                                          cnt.data_ptr(), off.data_ptr(), starts.data_ptr(), goals.data_ptr()), ctx.h)
    ok = torch.empty(E, dtype=torch.uint8, device=dev)
    robot.validate_device(starts.data_ptr(), goals.data_ptr(), E, environment, ok.data_ptr(), ctx=ctx)
    qi = torch.repeat_interleave(torch.arange(q_first, q_first + q_count, device=dev), cnt.long())
    m = torch.arange(E, device=dev) - off[:-1].long().repeat_interleave(cnt.long())
    qj = nbr[:q_count].long()[qi - q_first, m]
    keep = ok.bool()
    return torch.stack([qi[keep], qj[keep]], 1).to(torch.int32)  # vertex indices < 2^31


def allgather_pairs(torch, dist, pairs, group=None):
    """Concatenate the ranks' valid pairs in rank order (= query order): counts, then count-padded
    pairs, one all_gather_into_tensor each (RCCL on CUDA tensors, gloo on CPU tensors)."""
    world = dist.get_world_size(group)
    dev = pairs.device
    cnt = torch.tensor([pairs.shape[0]], dtype=torch.int64, device=dev)
    cnts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(cnts, cnt, group=group)
    counts = [int(c) for c in cnts.tolist()]
    mx = max(counts)
    send = torch.zeros((mx, 2), dtype=pairs.dtype, device=dev)
    send[:pairs.shape[0]] = pairs
    recv = torch.empty((world * mx, 2), dtype=pairs.dtype, device=dev)
    if mx:
        dist.all_gather_into_tensor(recv, send, group=group)
    return torch.cat([recv[r * mx:r * mx + c] for r, c in enumerate(counts)])


def assemble(n: int, pairs: np.ndarray):
    """Adjacency in build_roadmap's append order from the valid (vertex i, neighbour j) pairs
    listed in query order (i ascending, nearest first): vertex v's list = its own pairs' j, then
    every later i whose pair names v, ascending (prm.hh:270-275).  Host C++ (vgpu_roadmap_assemble).
    Returns (offsets [n+1], adj, component [n] = smallest vertex index of each vertex's
    connected component)."""
    import ctypes as C

    from . import _lib
    from ._lib import check, load
    p = np.asarray(pairs).reshape(-1, 2)
    p = p.view(np.uint32) if p.dtype == np.int32 and p.flags.c_contiguous else np.ascontiguousarray(p, np.uint32)
    offsets = np.zeros(n + 1, np.uint64)
    adj = np.zeros(max(2 * len(p), 1), np.uint32)
    comp = np.zeros(max(n, 1), np.uint32)
    check(load().vgpu_roadmap_assemble(n, p.ctypes.data_as(_lib.U32P), len(p),
                                       offsets.ctypes.data_as(C.POINTER(C.c_size_t)), adj.ctypes.data_as(_lib.U32P),
                                       comp.ctypes.data_as(_lib.U32P)))
    return offsets.astype(np.int64), adj[:2 * len(p)], comp[:n]


def assemble_device(torch, n: int, pairs, ctx):
    """assemble() on the GPU (vgpu_roadmap_assemble_device) from the valid pairs as a device int32 tensor
    [m, 2] (edges_shard / allgather_pairs output): (offsets int64 [n+1], adj int32 [2m], component int32 [n])
    device tensors, equal to the host assembly's."""
    from ._lib import check, load
    dev = pairs.device
    p = pairs.contiguous()
    m = int(p.shape[0])
    offsets = torch.empty(n + 1, dtype=torch.int64, device=dev)
    adj = torch.empty(max(2 * m, 1), dtype=torch.int32, device=dev)
    comp = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    check(load().vgpu_roadmap_assemble_device(ctx.h, n, p.data_ptr() if m else None, m, offsets.data_ptr(),
                                              adj.data_ptr(), comp.data_ptr()), ctx.h)
    return offsets, adj[:2 * m], comp[:n]


def build_roadmap_edges_sharded(torch, dist, robot, environment, V, gamma_scale: float = 2.0, ctx=None,
                                group=None) -> Roadmap:
    """The edge stage with the queries split over the ranks (query_split), each rank validating its
    own candidates on its GPU, then one exchange of the valid pairs; every rank returns the whole
    graph.  V: [n, dim] tensor on this rank's device, identical on all ranks."""
    from . import context
    ctx = ctx or context()
    dev = V.device
    if dev.type == "cuda":  # the kernels run on the context stream: make it torch's
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n, dim = V.shape
    k_np, r_np = prm_neighbor_params(dim, robot.space_measure(), n, gamma_scale)
    kmax = int(max(1, min(int(k_np.max()) if n else 1, n)))
    k = torch.from_numpy(k_np.view(np.int32)).to(dev)
    r = torch.from_numpy(r_np).to(dev)
    sharded = dist is not None and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if sharded else (0, 1)
    qf, qc = query_split(n, rank, world)
    pairs = edges_shard(torch, robot, environment, V, k, r, kmax, qf, qc, ctx)
    if sharded:
        pairs = allgather_pairs(torch, dist, pairs, group)
    offsets, adj, comp = assemble(n, pairs.cpu().numpy())
    return Roadmap(V.cpu().numpy(), offsets, adj, comp)


# ---- the C-level collectives (vgpu_comm_*, include/vamp_gpu.h): RCCL without torch.distributed --------
class Comm:
    """An RCCL communicator owned by the library (vgpu_comm_init; librccl loaded at run time): the
    C-level sharded stages (vgpu_prm_vertices_allgather, vgpu_prm_edges_allgather) run over it.  The
    128-byte id is made on rank 0 and shipped by the caller -- ``from_torch`` ships it over an
    initialised torch.distributed group (any backend), which then carries no data-path traffic."""

    def __init__(self, ctx, rank: int, world: int, uid: Optional[bytes] = None, hub: Optional["Loopback"] = None):
        import ctypes as C

        from ._lib import check, load
        self.ctx, self.rank, self.world = ctx, rank, world
        self.h = C.c_void_p()
        if hub is not None:  # a rank of an in-process loopback hub (vgpu_comm_init_loopback)
            assert hub.world == world
            check(load().vgpu_comm_init_loopback(ctx.h, rank, hub.h, C.byref(self.h)), ctx.h)
            return
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        check(load().vgpu_comm_init(ctx.h, rank, world, buf, C.byref(self.h)), ctx.h)

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C

        from ._lib import check, load
        buf = (C.c_uint8 * 128)()
        check(load().vgpu_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def from_torch(cls, torch, dist, ctx, group=None):
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        uid = cls.unique_id() if rank == 0 else bytes(128)
        if world > 1:
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
                else torch.device("cpu")
            t = torch.tensor(list(uid), dtype=torch.uint8, device=dev)
            dist.broadcast(t, 0, group=group)
            uid = bytes(t.cpu().tolist())
        return cls(ctx, rank, world, uid)

    def last_error(self) -> str:
        from ._lib import load
        m = load().vgpu_comm_last_error(self.h)
        return m.decode() if m else ""

    def check(self, rc: int):
        from ._lib import ERRORS, VgpuError
        if rc != 0:
            raise VgpuError(f"vamp_gpu: {ERRORS.get(rc, rc)}: {self.last_error()} / {self.ctx_error()}", rc)

    def ctx_error(self) -> str:
        from ._lib import load
        m = load().vgpu_last_error(self.ctx.h)
        return m.decode() if m else ""

    def close(self):
        from ._lib import load
        if self.h:
            load().vgpu_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Loopback:
    """An in-process loopback hub (vgpu_loopback_create): ``world`` ranks as threads of this process, each
    with its own context and ``Comm(ctx, rank, world, hub=self)`` -- created from one thread per rank, as creation
    is collective (it ends in a status all-gather, like vgpu_comm_init); the C stages' all-gathers become device
    copies between the ranks' buffers.  Close every Comm on it before closing the hub."""

    def __init__(self, world: int):
        import ctypes as C

        from ._lib import check, load
        self.world = world
        self.h = C.c_void_p()
        check(load().vgpu_loopback_create(world, C.byref(self.h)))

    def close(self):
        from ._lib import check, load
        if self.h:
            check(load().vgpu_loopback_destroy(self.h))
            self.h = None


def query_split_c(n: int, rank: int, world: int) -> Tuple[int, int]:
    """vgpu_query_split (the C edge stage's ranges)."""
    import ctypes as C

    from ._lib import check, load
    f, c = C.c_size_t(), C.c_size_t()
    check(load().vgpu_query_split(n, rank, world, C.byref(f), C.byref(c)))
    return f.value, c.value


class EdgeStageBuffers:
    """Device outputs of vgpu_prm_edges_allgather for n vertices, grown on demand (offsets int64 [n+1],
    adj int32, component int32 [n])."""

    def __init__(self, torch, n: int, dev, adj_cap: int = 0):
        self.torch, self.dev = torch, dev
        self.offsets = torch.empty(n + 1, dtype=torch.int64, device=dev)
        self.comp = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        self.adj = torch.empty(max(adj_cap, 1), dtype=torch.int32, device=dev)


def build_roadmap_edges_comm(torch, robot, environment, V, comm: "Comm", gamma_scale: float = 2.0, ctx=None,
                             bufs: Optional[EdgeStageBuffers] = None):
    """build_roadmap's edge stage through the C ABI's collective (vgpu_prm_edges_allgather): the queries
    split over the communicator's ranks, one exchange of the valid pairs, the roadmap assembled on every
    rank's device.  V: [n, dim] float32 CUDA tensor, identical on all ranks.  Returns (offsets, adj,
    component) device tensors, equal to build_roadmap_edges_sharded's graph."""
    import ctypes as C

    from ._lib import load
    ctx = ctx or comm.ctx
    n, dim = V.shape
    V = V.contiguous()
    if bufs is None:  # adjacency sized by the candidate bound (query i returns at most min(k_i, i))
        k, _ = prm_neighbor_params(dim, robot.space_measure(), n, gamma_scale)
        bound = int(np.minimum(k.astype(np.int64), np.arange(n, dtype=np.int64)).sum())
        bufs = EdgeStageBuffers(torch, n, V.device, 2 * bound)
    n_adj = C.c_size_t()
    lib = load()
    args = lambda: (ctx.h, comm.h, C.byref(robot.c_robot), environment.handle(ctx), V.data_ptr(), n,  # noqa: E731
                    robot.space_measure(), float(gamma_scale), bufs.offsets.data_ptr(), bufs.adj.data_ptr(),
                    bufs.adj.numel(), C.byref(n_adj), bufs.comp.data_ptr())
    rc = lib.vgpu_prm_edges_allgather(*args())
    if rc == -1 and n_adj.value > bufs.adj.numel():  # too small: every rank saw the same size -> grow, retry
        bufs.adj = torch.empty(n_adj.value, dtype=torch.int32, device=V.device)
        rc = lib.vgpu_prm_edges_allgather(*args())
    comm.check(rc)
    return bufs.offsets, bufs.adj[:n_adj.value], bufs.comp[:n]
