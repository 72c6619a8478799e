"""GPU parity: the HIP path (through the C ABI) against the C restatement and the
reference-DAG fixtures.

On the same host the GPU must equal the oracle BIT FOR BIT (masks, n, FK centres): both
follow the same canonical float32 op sequence and the same host rsqrt table.  Against the
reference-derived fixtures the contract tolerances apply (FK 1e-5, masks margin-filtered,
see tests/test_oracle.py).
"""
import numpy as np
import pytest

from conftest import golden, host_fixture
from test_oracle import EDGE_MIN_COVERAGE, FK_TOL, fixture_check, same_rsqrt_host, stable

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    ctx = vamp_amd.context(0)  # raises if no device / no library: never a silent fallback
    assert ctx is not None
    return vamp_amd


def gpu_env_from_oracle(vamp, oenv):
    """Mirror an oracle Env (already resolved axes/endpoints) into a product Environment."""
    env = vamp.Environment()
    for x, y, z, r, _ in oenv.spheres:
        env.add_sphere(vamp.Sphere([x, y, z], r))
    for row in oenv.cuboids + oenv.zcuboids:
        env.add_cuboid(vamp.Cuboid.from_axes(row[0:3], row[3:6], row[6:9], row[9:12], row[12:15]))
    for row in oenv.capsules + oenv.zcapsules:
        p1 = np.array(row[0:3], F)
        p2 = (p1 + np.array(row[3:6], F)).astype(F)
        env.add_capsule(vamp.Cylinder(p1, p2, row[6]))
    return env


def random_scene(oracle, rng, n_sph=6, n_cub=5, n_cap=4):
    e = oracle.Env()
    for _ in range(n_sph):
        e.add_sphere(rng.uniform([-0.8, -0.8, 0.0], [0.8, 0.8, 1.0]).astype(F), F(rng.uniform(0.05, 0.2)))
    for i in range(n_cub):
        c = rng.uniform([-0.8, -0.8, 0.0], [0.8, 0.8, 1.0]).astype(F)
        h = rng.uniform(0.03, 0.2, 3).astype(F)
        if i % 2 == 0:  # z-aligned (axis_3_z == 1)
            a = rng.uniform(0, 2 * np.pi)
            a1, a2, a3 = [np.cos(a), np.sin(a), 0], [-np.sin(a), np.cos(a), 0], [0, 0, 1]
        else:
            Q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
            a1, a2, a3 = Q[:, 0], Q[:, 1], Q[:, 2]
        e.add_cuboid_axes(c, np.array(a1, F), np.array(a2, F), np.array(a3, F), h)
    for i in range(n_cap):
        p1 = rng.uniform([-0.8, -0.8, 0.0], [0.8, 0.8, 1.0]).astype(F)
        if i % 2 == 0:  # z-aligned capsule
            p2 = (p1 + np.array([0, 0, rng.uniform(0.1, 0.5)], F)).astype(F)
        else:
            p2 = (p1 + rng.uniform(-0.4, 0.4, 3)).astype(F)
        e.add_capsule_endpoints(p1, p2, F(rng.uniform(0.02, 0.1)))
    return e


def test_rsqrt_table_matches_oracle_probe(vamp, oracle):
    lut, kb = vamp.context().rsqrt_table()
    olut, okb = oracle.rsqrt_probe()
    assert kb == okb and np.array_equal(lut, olut)


@pytest.mark.parametrize("tag,base", [("b000", (0, 0, 0)), ("b220", (200, 200, 0)), ("b105", (100, -50, 5))])
def test_sphere_fk(vamp, oracle, tag, base):
    fx = host_fixture("fk_panda.npz", oracle)
    robot = vamp.PandaBase(*base)
    got = robot.sphere_fk_batch(fx["q"])
    ora = oracle.sphere_fk(fx["q"], base)
    assert np.array_equal(got.view(np.uint32), ora.view(np.uint32))  # identical op sequence
    assert np.abs(got - fx[tag]).max() <= FK_TOL
    spheres = robot.fk(fx["q"][0])
    assert len(spheres) == 59 and np.allclose([s.r for s in spheres], fx["radii"])


def test_fkcc_cage(vamp, oracle):
    fx = host_fixture("fkcc_panda_cage.npz", oracle)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    same = same_rsqrt_host(oracle, fx)
    for sfx, base in (("", (0, 0, 0)), ("_b220", (200, 200, 0))):
        q = fx["q" + sfx]
        robot = vamp.PandaBase(*base)
        got = robot.fkcc_batch(q, env)
        assert np.array_equal(got, oracle.fkcc_threads(oenv, q, base)), "GPU != oracle on the same host"
        m = stable(fx["test_margin" + sfx], fx["cull_margin" + sfx], same)
        fixture_check(f"panda fkcc cage{sfx or '_b000'} (GPU)", got, fx["valid" + sfx], m, same)


def test_validate_motions_cage(vamp, oracle):
    fx = host_fixture("edges_panda_cage.npz", oracle)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    robot = vamp.panda_0_0
    ok, n = robot.validate_batch(fx["starts"], fx["goals"], env)
    ook, on = oracle.validate_motions(oenv, fx["starts"], fx["goals"], (0, 0, 0))
    assert np.array_equal(n, on) and np.array_equal(n, fx["n"])
    assert np.array_equal(ok, ook), "GPU != oracle on the same host"
    same = same_rsqrt_host(oracle, fx)
    m = stable(fx["test_margin"], fx["cull_margin"], same)
    fixture_check("panda validate_motion cage edges (GPU)", ok, fx["ok"], m, same, EDGE_MIN_COVERAGE)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mixed_primitives_exact(vamp, oracle, seed):
    """Spheres, capsules, z-capsules, cuboids and z-cuboids: GPU == oracle, configs and edges."""
    rng = np.random.default_rng(seed)
    oenv = random_scene(oracle, rng)
    env = gpu_env_from_oracle(vamp, oenv)
    assert env.counts() == [len(oenv.spheres), len(oenv.capsules), len(oenv.zcapsules), len(oenv.cuboids),
                            len(oenv.zcuboids)]
    q = oracle.scale(rng.random((20000, 7), dtype=F))
    for base in ((0, 0, 0), (200, 200, 0)):
        got = vamp.PandaBase(*base).fkcc_batch(q, env)
        assert np.array_equal(got, oracle.fkcc_threads(oenv, q, base))
    s = oracle.scale(rng.random((3000, 7), dtype=F))
    g = oracle.scale(rng.random((3000, 7), dtype=F))
    g[:1000] = s[:1000] + (g[:1000] - s[:1000]) * F(0.1)
    ok, n = vamp.panda_0_0.validate_batch(s, g, env)
    ook, on = oracle.validate_motions(oenv, s, g, (0, 0, 0))
    assert np.array_equal(n, on) and np.array_equal(ok, ook)


def test_edge_cases(vamp, oracle):
    env = vamp.Environment()  # empty: self-collision only
    oenv = oracle.Env()
    robot = vamp.panda_0_0
    # empty batches
    assert robot.fkcc_batch(np.zeros((0, 7), F), env).shape == (0,)
    ok, n = robot.validate_batch(np.zeros((0, 7), F), np.zeros((0, 7), F), env)
    assert ok.shape == (0,)
    # single configuration API mirrors vamp.panda.validate (bounds check + fkcc)
    q0 = np.zeros(7, F)
    q0[3] = -1.5  # inside joint limits
    assert robot.validate(q0, env) == bool(oracle.fkcc(oenv, q0[None])[0])
    q_out = q0.copy()
    q_out[0] = 3.5  # outside the joint-0 limit -> invalid without any collision check
    assert robot.validate(q_out, env) is False
    # zero-length and very long edges (n large), ragged batch size
    rng = np.random.default_rng(11)
    s = oracle.scale(rng.random((777, 7), dtype=F))
    g = oracle.scale(rng.random((777, 7), dtype=F))
    g[:5] = s[:5]
    g[5:10] = (s[5:10] + F(40.0)).astype(F)  # far outside limits: n ~ 400
    ok, n = robot.validate_batch(s, g, env)
    ook, on = oracle.validate_motions(oenv, s, g, (0, 0, 0))
    assert (n[:5] == 1).all() and (n[5:10] > 300).all()
    assert np.array_equal(n, on) and np.array_equal(ok, ook)


def test_large_batch_properties(vamp, oracle):
    """At bench scale (1M configurations): a random 64k subset equals the oracle exactly and
    adding obstacles never validates a configuration (monotonicity)."""
    rng = np.random.default_rng(5)
    q = oracle.scale(rng.random((1 << 20, 7), dtype=F))
    oenv = oracle.sphere_cage_env()
    cage = gpu_env_from_oracle(vamp, oenv)
    empty = vamp.Environment()
    v_cage = vamp.panda_0_0.fkcc_batch(q, cage)
    v_empty = vamp.panda_0_0.fkcc_batch(q, empty)
    assert (v_cage <= v_empty).all()
    idx = rng.choice(len(q), 65536, replace=False)
    assert np.array_equal(v_cage[idx], oracle.fkcc_threads(oenv, q[idx], (0, 0, 0)))
    assert 0.15 < v_cage.mean() < 0.21


def test_full_mask_mode(vamp, oracle):
    """vgpu_validate_motions_mask (every block evaluated, each block's result kept) == the CPU rake's
    full mask (itself == the oracle per block, tests/test_cpu_rake.py), and its edge results == the
    early-exit validate_motions."""
    import torch
    rng = np.random.default_rng(21)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    s = oracle.scale(rng.random((20000, 7), dtype=F))
    g = oracle.scale(rng.random((20000, 7), dtype=F))
    g[:10000] = s[:10000] + (g[:10000] - s[:10000]) * F(0.2)
    g[:5] = s[:5]
    ok_c, n_c, blk_c, _ = vamp.panda_0_0.cpu_validate_mask(s, g, env)
    dev = torch.device("cuda", 0)
    ds, dg = torch.from_numpy(s).to(dev), torch.from_numpy(g).to(dev)
    ok = torch.empty(len(s), dtype=torch.uint8, device=dev)
    nb = torch.empty(len(s), dtype=torch.int32, device=dev)
    blk = torch.empty(int(n_c.sum()) + 7, dtype=torch.uint8, device=dev)
    ctx = vamp.context(0)
    total = vamp.panda_0_0.validate_mask_device(ds.data_ptr(), dg.data_ptr(), len(s), env, ok.data_ptr(),
                                                nb.data_ptr(), blk.data_ptr(), blk.numel(), ctx)
    ctx.sync()
    assert total == int(n_c.sum())
    assert np.array_equal(nb.cpu().numpy(), n_c)
    assert np.array_equal(ok.cpu().numpy().astype(bool), ok_c)
    assert np.array_equal(blk[:total].cpu().numpy().astype(bool), blk_c)
    ok_e, _ = vamp.panda_0_0.validate_batch(s, g, env)
    assert np.array_equal(ok_e, ok_c)
    with pytest.raises(vamp.VgpuError):  # capacity below the block count
        vamp.panda_0_0.validate_mask_device(ds.data_ptr(), dg.data_ptr(), len(s), env, ok.data_ptr(), 0,
                                            blk.data_ptr(), 10, ctx)


def test_too_many_blocks_rejected(vamp, oracle):
    """The back-step scan and item indices are 32-bit: a batch of edges whose rake blocks exceed 2^32
    (three edges of ~2^31 blocks each) is rejected with VGPU_ERR_INVALID_ARG before any offset is
    used (vgpu_api.cpp item_total), in full-mask and early-exit mode alike."""
    import torch
    env = vamp.Environment()
    s = np.zeros((3, 7), F)
    s[:, 3] = -1.5
    g = s.copy()
    g[:, 0] += F(1e9)  # n = ceil(d / 8 * 32) saturates at 2147483520
    dev = torch.device("cuda", 0)
    ds, dg = torch.from_numpy(s).to(dev), torch.from_numpy(g).to(dev)
    ok = torch.empty(3, dtype=torch.uint8, device=dev)
    nb = torch.empty(3, dtype=torch.int32, device=dev)
    blk = torch.empty(16, dtype=torch.uint8, device=dev)
    ctx = vamp.context(0)
    with pytest.raises(vamp.VgpuError, match="2\\^32"):
        vamp.panda_0_0.validate_mask_device(ds.data_ptr(), dg.data_ptr(), 3, env, ok.data_ptr(), nb.data_ptr(),
                                            blk.data_ptr(), blk.numel(), ctx)
    ctx.sync()
    # the context stays usable
    q = oracle.scale(np.random.default_rng(3).random((256, 7), dtype=F))
    assert np.array_equal(vamp.panda_0_0.fkcc_batch(q, env), oracle.fkcc_threads(oracle.Env(), q))
