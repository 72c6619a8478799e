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
    devs = (C.c_int * 2)(0, 0)  # two contexts on one device: two host threads, two contiguous ranges
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
