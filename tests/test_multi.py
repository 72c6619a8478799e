"""C-level multi-GPU (mr-vamp_amd/csrc/vgpu_multi.cpp).

CPU: vgpu_shard_range splits n units into contiguous, balanced ranges that cover [0, n) in rank order.
GPU (single MI355X): the one-process multi-device entry points run with two contexts on device 0 (two
host threads, two ranges) and equal the single-context results; the RCCL path at world size 1
(vgpu_comm_* + vgpu_prm_vertices_allgather, librccl loaded at run time, no torch.distributed) gives
build_roadmap's vertex sequence exactly as the single-process sampler does."""
import ctypes as C

import numpy as np
import pytest

from test_gpu_parity import gpu_env_from_oracle, random_scene

F = np.float32


def test_shard_range_covers_and_balances():
    from vamp_amd._lib import load
    lib = load()
    for n in (0, 1, 7, 1000, 1 << 20, 4_000_000, (1 << 40) + 3):
        for w in (1, 2, 3, 8, 13):
            prev = 0
            sizes = []
            for r in range(w):
                f, c = C.c_size_t(), C.c_size_t()
                assert lib.vgpu_shard_range(n, r, w, C.byref(f), C.byref(c)) == 0
                assert f.value == prev
                prev += c.value
                sizes.append(c.value)
            assert prev == n and max(sizes) - min(sizes) <= 1
    f, c = C.c_size_t(), C.c_size_t()
    assert lib.vgpu_shard_range(10, 3, 3, C.byref(f), C.byref(c)) != 0
    assert lib.vgpu_shard_range(10, 0, 0, C.byref(f), C.byref(c)) != 0


@pytest.fixture(scope="module")
def multi():
    import vamp_amd
    from vamp_amd._lib import check, load
    assert vamp_amd.context(0) is not None
    lib = load()
    m = C.c_void_p()
    import torch
    # two devices when the box has them (device placement of the per-thread work is then exercised);
    # else two contexts on one device: two host threads, two contiguous ranges
    pair = (0, 1) if torch.cuda.device_count() > 1 else (0, 0)
    devs = (C.c_int * 2)(*pair)
    check(lib.vgpu_multi_create(devs, 2, C.byref(m)))
    yield vamp_amd, lib, m
    lib.vgpu_multi_destroy(m)


def _menv(lib, m, env):
    envs = (C.c_void_p * 2)()
    from vamp_amd._lib import check
    check(lib.vgpu_multi_env_create(m, env.host_handle(), envs))
    return envs


@pytest.mark.gpu
def test_multi_validate_and_sample_equal_single(multi, oracle):
    vamp, lib, m = multi
    from vamp_amd import _lib
    from vamp_amd._lib import check
    rng = np.random.default_rng(51)
    oenv = random_scene(oracle, rng, 4, 3, 2)
    env = gpu_env_from_oracle(vamp, oenv)
    envs = _menv(lib, m, env)
    try:
        robot = vamp.panda_0_0
        s = oracle.scale(rng.random((20001, 7), dtype=F))
        g = (s + (oracle.scale(rng.random((20001, 7), dtype=F)) - s) * F(0.3)).astype(F)
        ok = np.zeros(len(s), np.uint8)
        nb = np.zeros(len(s), np.int32)
        check(lib.vgpu_multi_validate_motions_host(m, C.byref(robot.c_robot), envs, s.ctypes.data_as(_lib.F32P),
                                                   g.ctypes.data_as(_lib.F32P), len(s), ok.ctypes.data_as(_lib.U8P),
                                                   nb.ctypes.data_as(_lib.I32P)))
        ok1, nb1 = robot.validate_batch(s, g, env)
        assert np.array_equal(ok.astype(bool), ok1) and np.array_equal(nb, nb1)
        n_draws = 50001
        rows = np.zeros((n_draws, 8), F)
        draws = np.zeros(n_draws, np.uint64)
        cnt = C.c_size_t()
        check(lib.vgpu_multi_sample_fkcc_host(m, C.byref(vamp.fetch.c_robot), envs, 7, n_draws,
                                              rows.ctypes.data_as(_lib.F32P),
                                              draws.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(cnt)))
        q, v = vamp.fetch.sample_fkcc(7, n_draws, env)
        assert cnt.value == int(v.sum())
        assert np.array_equal(rows[:cnt.value].view(np.uint32), q[v].view(np.uint32))
        assert np.array_equal(draws[:cnt.value], 7 + np.nonzero(v)[0])
    finally:
        for e in envs:
            lib.vgpu_env_destroy(e)


@pytest.mark.gpu
def test_rccl_vertex_allgather_world1(oracle):
    """world size 1 through RCCL: the vertex sequence of the single-process sampler, bit for bit"""
    import torch

    import vamp_amd as vamp
    from vamp_amd import _lib
    from vamp_amd._lib import check, load
    lib = load()
    ctx = vamp.context(0)
    uid = (C.c_uint8 * 128)()
    rc = lib.vgpu_comm_unique_id(uid)
    if rc == -4:
        pytest.skip("librccl.so.1 not loadable on this box")
    check(rc)
    comm = C.c_void_p()
    check(lib.vgpu_comm_init(ctx.h, 0, 1, uid, C.byref(comm)), ctx.h)
    try:
        env = vamp.Environment()
        env.add_sphere(vamp.Sphere([0.5, 0.0, 0.5], 0.3))
        n = 100000
        rows = torch.zeros((n, 7), dtype=torch.float32, device="cuda")
        draws = torch.zeros(n, dtype=torch.int64, device="cuda")
        cnt = C.c_size_t()
        check(lib.vgpu_prm_vertices_allgather(ctx.h, comm, C.byref(vamp.panda_0_0.c_robot), env.handle(ctx), 1, n,
                                              C.c_void_p(rows.data_ptr()), C.c_void_p(draws.data_ptr()), n,
                                              C.byref(cnt)), ctx.h)
        q, v = vamp.panda_0_0.sample_fkcc(1, n, env)
        assert cnt.value == int(v.sum()) > 0
        got = rows[:cnt.value].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), q[v].view(np.uint32))
        assert np.array_equal(draws[:cnt.value].cpu().numpy(), 1 + np.nonzero(v)[0])
    finally:
        lib.vgpu_comm_destroy(comm)


def _comm(vamp, ctx):
    from vamp_amd import roadmap
    try:
        uid = roadmap.Comm.unique_id()
    except Exception as e:  # librccl not loadable: VGPU_ERR_UNSUPPORTED
        pytest.skip(f"RCCL unavailable: {e}")
    return roadmap.Comm(ctx, 0, 1, uid)


@pytest.mark.gpu
def test_rccl_edges_allgather_world1_equals_oracle(oracle):
    """vgpu_prm_edges_allgather at world size 1 (query split, kNN, validate, pair selection, the two
    exchanges, device assembly) == build_roadmap_edges_sharded == the oracle's build_roadmap graph"""
    import torch

    import vamp_amd as vamp
    from vamp_amd import roadmap
    ctx = vamp.context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    comm = _comm(vamp, ctx)
    try:
        rng = np.random.default_rng(24)
        oenv = random_scene(oracle, rng, 4, 4, 2)
        env = gpu_env_from_oracle(vamp, oenv)
        q = oracle.robot_scale("fetch", rng.random((5000, 8), dtype=F))
        V = q[oracle.robot_fkcc_threads("fetch", oenv, q)][:2000]
        Vd = torch.from_numpy(V).cuda()
        off, adj, comp = roadmap.build_roadmap_edges_comm(torch, vamp.fetch, env, Vd, comm)
        off, adj, comp = off.cpu().numpy(), adj.cpu().numpy(), comp.cpu().numpy()
        edges, _ = oracle.build_roadmap_edges("fetch", oenv, V)
        assert [adj[off[i]:off[i + 1]].tolist() for i in range(len(V))] == edges
        assert np.array_equal(comp, oracle.components(len(V), edges))
        rm = roadmap.build_roadmap_edges_sharded(torch, None, vamp.fetch, env, Vd)
        assert np.array_equal(off, rm.offsets) and np.array_equal(adj.view(np.uint32), rm.adj)
        # a second call on the same communicator reuses its buffers and gives the same graph
        off2, adj2, _ = roadmap.build_roadmap_edges_comm(torch, vamp.fetch, env, Vd, comm)
        assert np.array_equal(off2.cpu().numpy(), off) and np.array_equal(adj2.cpu().numpy(), adj)
    finally:
        comm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("site", ["prm_vertices", "prm_edges"])
def test_rccl_failure_is_reported_not_hung(oracle, site, monkeypatch):
    """A rank-local failure (VGPU_FAULT_INJECT forces the allocation-failure path) still enters the count
    exchange and comes back as an error code from every rank -- here world size 1 -- instead of leaving
    peers inside an all-gather; the communicator stays usable for the next call."""
    import ctypes as Cc

    import torch

    import vamp_amd as vamp
    from vamp_amd import roadmap
    from vamp_amd._lib import load
    ctx = vamp.context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    comm = _comm(vamp, ctx)
    lib = load()
    try:
        env = vamp.Environment()
        env.add_sphere(vamp.Sphere([0.5, 0.0, 0.5], 0.3))
        n = 20000
        rows = torch.zeros((n, 7), dtype=torch.float32, device="cuda")
        draws = torch.zeros(n, dtype=torch.int64, device="cuda")
        cnt = Cc.c_size_t()

        def vertices():
            return lib.vgpu_prm_vertices_allgather(ctx.h, comm.h, Cc.byref(vamp.panda_0_0.c_robot), env.handle(ctx), 1,
                                                   n, Cc.c_void_p(rows.data_ptr()), Cc.c_void_p(draws.data_ptr()), n,
                                                   Cc.byref(cnt))

        def edges():
            V = rows[:2000].contiguous()
            bufs = roadmap.EdgeStageBuffers(torch, 2000, V.device, 200000)
            n_adj = Cc.c_size_t()
            return lib.vgpu_prm_edges_allgather(ctx.h, comm.h, Cc.byref(vamp.panda_0_0.c_robot), env.handle(ctx),
                                                V.data_ptr(), 2000, vamp.panda_0_0.space_measure(), 2.0,
                                                bufs.offsets.data_ptr(), bufs.adj.data_ptr(), bufs.adj.numel(),
                                                Cc.byref(n_adj), bufs.comp.data_ptr())

        assert vertices() == 0 and cnt.value > 2000
        call = vertices if site == "prm_vertices" else edges
        monkeypatch.setenv("VGPU_FAULT_INJECT", site)
        assert call() == -3  # VGPU_ERR_OOM, returned (not hung)
        assert "injected" in comm.last_error()
        monkeypatch.setenv("VGPU_FAULT_INJECT", site + "@1")  # another rank's fault: not this one
        assert call() == 0
        monkeypatch.delenv("VGPU_FAULT_INJECT")
        assert call() == 0
        # a capacity too small is reported to every rank alike
        assert lib.vgpu_prm_vertices_allgather(ctx.h, comm.h, Cc.byref(vamp.panda_0_0.c_robot), env.handle(ctx), 1, n,
                                               Cc.c_void_p(rows.data_ptr()), Cc.c_void_p(draws.data_ptr()), 10,
                                               Cc.byref(cnt)) == -1
    finally:
        comm.close()


@pytest.mark.gpu
def test_host_staging_lands_on_the_context_device():
    """vgpu_*_host stage their buffers after selecting the context's device (HIP's current device is per
    thread): with a context on device 1 and the calling thread on device 0, the staging buffer must live
    on device 1.  Needs two GPUs; skipped (and visible as skipped) on a one-GPU box."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU: the cross-device placement case needs device 1")
    import vamp_amd as vamp
    ctx1 = vamp.context(1)
    torch.cuda.set_device(0)
    env = vamp.Environment()
    env.add_sphere(vamp.Sphere([0.5, 0.0, 0.5], 0.2))
    q = np.zeros((64, 7), F)
    got = vamp.panda_0_0.fkcc_batch(q, env, ctx1)
    assert got.shape == (64,)


# ---- world size > 1 on one GPU: the in-process loopback hub (vgpu_comm_init_loopback) -----------------
def _run_ranks(world, fn):
    """fn(rank) on one host thread per rank (ctypes releases the GIL inside the C calls); returns the
    per-rank results, re-raising the first exception"""
    import threading
    out, errs = [None] * world, [None] * world

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errs[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=150)
        assert not t.is_alive(), "a rank did not return (hung exchange)"
    for e in errs:
        if e is not None:
            raise e
    return out


@pytest.fixture
def loopback_ranks(monkeypatch):
    """make(world) -> (contexts, comms): one fresh context per rank on device 0, one loopback hub"""
    import vamp_amd as vamp
    from vamp_amd import roadmap
    monkeypatch.setenv("VGPU_LOOPBACK_TIMEOUT_S", "30")
    made = []

    def make(world):
        ctxs = [vamp.Context(0) for _ in range(world)]
        hub = roadmap.Loopback(world)
        # creation is collective (it ends in a status all-gather): one thread per rank, like vgpu_comm_init
        comms = _run_ranks(world, lambda r: roadmap.Comm(ctxs[r], r, world, hub=hub))
        made.append((ctxs, hub, comms))
        return ctxs, comms

    yield make
    for ctxs, hub, comms in made:
        for c in comms:
            c.close()
        hub.close()


def _vertices_call(lib, vamp, ctx, comm, robot, env, first, n, rows, draws, cap, cnt):
    return lib.vgpu_prm_vertices_allgather(ctx.h if ctx else None, comm.h, C.byref(robot.c_robot),
                                           env.handle(ctx) if ctx else None, first, n,
                                           C.c_void_p(rows.data_ptr()) if rows is not None else None,
                                           C.c_void_p(draws.data_ptr()), cap, C.byref(cnt))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_loopback_vertex_stage_equals_single_process(loopback_ranks, world):
    """vgpu_prm_vertices_allgather at world size 2 / 3 (ranks = threads, each its own context on device 0,
    loopback all-gathers): every rank gets build_roadmap's vertex sequence -- the single-process sampler's
    valid draws in draw order, bit for bit -- including ranks whose share is shorter (n not divisible)."""
    import torch

    import vamp_amd as vamp
    from vamp_amd._lib import load
    lib = load()
    ctxs, comms = loopback_ranks(world)
    env = vamp.Environment()  # a scene the Fetch collides with for some draws only
    env.add_sphere(vamp.Sphere([0.9, 0.3, 0.8], 0.2))
    robot = vamp.fetch
    n, first = 40001, 3
    for c in ctxs:
        env.handle(c)  # realised on every context before the threads start
    q, v = robot.sample_fkcc(first, n, env)
    want_rows, want_draws = q[v], first + np.nonzero(v)[0]
    bufs = [(torch.zeros((n, 8), dtype=torch.float32, device="cuda"), torch.zeros(n, dtype=torch.int64, device="cuda"))
            for _ in range(world)]
    torch.cuda.synchronize()

    def rank(r):
        cnt = C.c_size_t()
        rc = _vertices_call(lib, vamp, ctxs[r], comms[r], robot, env, first, n, bufs[r][0], bufs[r][1], n, cnt)
        return rc, cnt.value

    res = _run_ranks(world, rank)
    torch.cuda.synchronize()
    for r, (rc, cnt) in enumerate(res):
        assert rc == 0, (r, comms[r].last_error())
        assert cnt == len(want_rows) and 0 < cnt < n
        assert np.array_equal(bufs[r][0][:cnt].cpu().numpy().view(np.uint32), want_rows.view(np.uint32))
        assert np.array_equal(bufs[r][1][:cnt].cpu().numpy(), want_draws)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_loopback_edge_stage_equals_oracle(oracle, loopback_ranks, world):
    """vgpu_prm_edges_allgather at world size 2 / 3: each rank's query range (vgpu_query_split), its valid
    pairs all-gathered in rank order, the roadmap assembled on every rank == the single-process C stage ==
    the oracle's build_roadmap graph (adjacency lists in append order, components)."""
    import torch

    import vamp_amd as vamp
    from vamp_amd import roadmap
    ctxs, comms = loopback_ranks(world)
    rng = np.random.default_rng(25)
    oenv = random_scene(oracle, rng, 4, 4, 2)
    env = gpu_env_from_oracle(vamp, oenv)
    for c in ctxs:
        env.handle(c)
    q = oracle.robot_scale("fetch", rng.random((6000, 8), dtype=F))
    V = q[oracle.robot_fkcc_threads("fetch", oenv, q)][:2500]
    Vd = torch.from_numpy(V).cuda()
    torch.cuda.synchronize()
    edges, _ = oracle.build_roadmap_edges("fetch", oenv, V)
    comp_ref = oracle.components(len(V), edges)

    def rank(r):
        off, adj, comp = roadmap.build_roadmap_edges_comm(torch, vamp.fetch, env, Vd, comms[r], ctx=ctxs[r])
        ctxs[r].sync()
        return off.cpu().numpy(), adj.cpu().numpy(), comp.cpu().numpy()

    for off, adj, comp in _run_ranks(world, rank):
        assert [adj[off[i]:off[i + 1]].tolist() for i in range(len(V))] == edges
        assert np.array_equal(comp, comp_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("stage", ["prm_vertices", "prm_edges"])
def test_loopback_rank_failure_reaches_every_rank(loopback_ranks, monkeypatch, world, stage):
    """A failure on rank 1 only -- an argument error (injected, and a real null output / null context), its
    first allocation, or after every allocation -- comes back as the SAME error code from every rank, none
    hangs in an all-gather, and the communicators stay usable for the next call."""
    import torch

    import vamp_amd as vamp
    from vamp_amd import roadmap
    from vamp_amd._lib import load
    lib = load()
    ctxs, comms = loopback_ranks(world)
    env = vamp.Environment()
    env.add_sphere(vamp.Sphere([0.5, 0.0, 0.5], 0.3))
    for c in ctxs:
        env.handle(c)
    robot = vamp.panda_0_0
    n = 20000
    bufs = [(torch.zeros((n, 7), dtype=torch.float32, device="cuda"), torch.zeros(n, dtype=torch.int64, device="cuda"))
            for _ in range(world)]
    V = bufs[0][0][:1500].clone()
    ebufs = [roadmap.EdgeStageBuffers(torch, 1500, V.device, 200000) for _ in range(world)]
    torch.cuda.synchronize()
    null = {"ctx": False, "out": False}

    def call(r):
        bad = r == 1
        ctx = None if (bad and null["ctx"]) else ctxs[r]
        if stage == "prm_vertices":
            cnt = C.c_size_t()
            rows = None if (bad and null["out"]) else bufs[r][0]
            return _vertices_call(lib, vamp, ctx, comms[r], robot, env, 1, n, rows, bufs[r][1], n, cnt)
        n_adj = C.c_size_t()
        b = ebufs[r]
        return lib.vgpu_prm_edges_allgather(ctx.h if ctx else None, comms[r].h, C.byref(robot.c_robot),
                                            env.handle(ctxs[r]), V.data_ptr(), 1500, robot.space_measure(), 2.0,
                                            None if (bad and null["out"]) else b.offsets.data_ptr(),
                                            b.adj.data_ptr(), b.adj.numel(), C.byref(n_adj), b.comp.data_ptr())

    assert _run_ranks(world, call) == [0] * world
    for site, code in ((":args", -1), (":alloc", -3), ("", -3)):
        monkeypatch.setenv("VGPU_FAULT_INJECT", f"{stage}{site}@1")
        got = _run_ranks(world, call)
        assert got == [code] * world, (site, got, [c.last_error() for c in comms])
        assert "injected" in comms[1].last_error()
        assert "rank 1 failed" in comms[0].last_error()
    monkeypatch.delenv("VGPU_FAULT_INJECT")
    for key in ("out", "ctx"):  # real argument errors on rank 1
        null[key] = True
        assert _run_ranks(world, call) == [-1] * world, key
        null[key] = False
    assert _run_ranks(world, call) == [0] * world


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("site", ["comm_init", "comm_init:alloc"])
def test_loopback_comm_init_failure_reaches_every_rank(monkeypatch, world, site):
    """Communicator creation ends in a status all-gather (vgpu_multi.cpp comm_status_exchange): a failure on
    rank 1 only -- after every allocation, or its stream / exchange allocation -- makes EVERY rank's
    vgpu_comm_init_loopback return the same code and hand back no communicator, at once (no rank is left to
    block in its first stage's all-gather; the loopback timeout is set far above the test's limit)."""
    import time

    import vamp_amd as vamp
    from vamp_amd import roadmap
    from vamp_amd._lib import load
    lib = load()
    monkeypatch.setenv("VGPU_LOOPBACK_TIMEOUT_S", "600")
    ctxs = [vamp.Context(0) for _ in range(world)]
    hub = roadmap.Loopback(world)
    code = -2 if site == "comm_init" else -3
    monkeypatch.setenv("VGPU_FAULT_INJECT", f"{site}@1")
    handles = [C.c_void_p() for _ in range(world)]
    t = time.perf_counter()
    got = _run_ranks(world, lambda r: lib.vgpu_comm_init_loopback(ctxs[r].h, r, hub.h, C.byref(handles[r])))
    assert time.perf_counter() - t < 30
    assert got == [code] * world, got
    assert not any(h.value for h in handles)
    monkeypatch.delenv("VGPU_FAULT_INJECT")
    comms = _run_ranks(world, lambda r: roadmap.Comm(ctxs[r], r, world, hub=hub))  # the hub is still usable
    for c in comms:
        c.close()
    hub.close()


@pytest.mark.gpu
def test_loopback_rank_that_never_arrives_fails_the_hub_for_good(monkeypatch):
    """a peer that never enters an exchange makes the waiting ranks fail after
    VGPU_LOOPBACK_TIMEOUT_S, and the hub stays failed -- a late rank cannot pair up with the next call's
    exchange -- so every later stage call on it fails at once instead of mixing data of different calls."""
    import time

    import torch

    import vamp_amd as vamp
    from vamp_amd import roadmap
    from vamp_amd._lib import load
    lib = load()
    monkeypatch.setenv("VGPU_LOOPBACK_TIMEOUT_S", "2")
    world = 2
    ctxs = [vamp.Context(0) for _ in range(world)]
    hub = roadmap.Loopback(world)
    comms = _run_ranks(world, lambda r: roadmap.Comm(ctxs[r], r, world, hub=hub))
    env = vamp.Environment()
    env.add_sphere(vamp.Sphere([0.5, 0.0, 0.5], 0.3))
    for c in ctxs:
        env.handle(c)
    robot = vamp.panda_0_0
    n = 4000
    bufs = [(torch.zeros((n, 7), dtype=torch.float32, device="cuda"), torch.zeros(n, dtype=torch.int64, device="cuda"))
            for _ in range(world)]
    torch.cuda.synchronize()

    def call(r):
        cnt = C.c_size_t()
        return _vertices_call(lib, vamp, ctxs[r], comms[r], robot, env, 1, n, bufs[r][0], bufs[r][1], n, cnt)

    t = time.perf_counter()
    assert call(0) != 0  # rank 1 never arrives: rank 0 times out instead of hanging
    assert time.perf_counter() - t < 20
    t = time.perf_counter()
    assert _run_ranks(world, call) == [-2, -2]
    assert time.perf_counter() - t < 20  # failed hub: no further waiting
    for c in comms:
        c.close()
    hub.close()
