"""The CPU rake (host AVX2, mr-vamp_amd/csrc/cpu/) through the C ABI: the reference's single-call
entry points (Robot::fkcc<8>, validate_motion, sphere_fk) and their threaded batches, bit-exact
against the C restatement (oracle/) on the same host and against the reference-DAG fixtures on
the margin-filtered set.  No GPU: these run in the CPU suite."""
import ctypes as C

import numpy as np
import pytest

from conftest import host_fixture
from scenes import R_MAX, R_MIN, R_POINT, cage_points, terrain
from test_gpu_parity import gpu_env_from_oracle, random_scene
from test_oracle import EDGE_MIN_COVERAGE, fixture_check, same_rsqrt_host, stable
from test_oracle_robots import CASES, scene_env

F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    return vamp_amd


def test_cage_fkcc_and_fixture(vamp, oracle):
    fx = host_fixture("fkcc_panda_cage.npz", oracle)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    same = same_rsqrt_host(oracle, fx)
    for sfx, base in (("", (0, 0, 0)), ("_b220", (200, 200, 0))):
        q = fx["q" + sfx]
        got = vamp.PandaBase(*base).cpu_fkcc_batch(q, env)
        assert np.array_equal(got, oracle.fkcc_threads(oenv, q, base)), "CPU rake != oracle"
        m = stable(fx["test_margin" + sfx], fx["cull_margin" + sfx], same)
        fixture_check(f"panda fkcc cage{sfx or '_b000'} (CPU rake)", got, fx["valid" + sfx], m, same)


def test_cage_validate_and_fixture(vamp, oracle):
    fx = host_fixture("edges_panda_cage.npz", oracle)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    ok, n, ev = vamp.panda_0_0.cpu_validate_batch(fx["starts"], fx["goals"], env, threads=4)
    ook, on = oracle.validate_motions(oenv, fx["starts"], fx["goals"], (0, 0, 0))
    assert np.array_equal(n, on) and np.array_equal(ok, ook)
    # early-exit accounting: a valid edge evaluated all its blocks, an invalid one stopped early
    assert (ev[ok] == n[ok]).all() and (ev >= 1).all() and (ev <= n).all()
    m = stable(fx["test_margin"], fx["cull_margin"], same_rsqrt_host(oracle, fx))
    fixture_check("panda validate_motion cage edges (CPU rake)", ok, fx["ok"], m, same_rsqrt_host(oracle, fx),
                  EDGE_MIN_COVERAGE)


def test_evaluated_blocks_are_the_first_failure(vamp, oracle):
    """n_evaluated = index of the first invalid rake block + 1, checked block by block through
    the single-block entry point (Robot::fkcc<8> on the enumerated back-steps)."""
    fx = host_fixture("edges_panda_cage.npz", oracle)
    env = gpu_env_from_oracle(vamp, oracle.sphere_cage_env())
    s, g = fx["starts"][:300], fx["goals"][:300]
    ok, n, ev = vamp.panda_0_0.cpu_validate_batch(s, g, env, threads=1)
    pct = np.arange(1, 9, dtype=F) / F(8)
    for e in np.flatnonzero(~ok)[:40]:
        v = (g[e] - s[e]).astype(F)
        blk = np.empty((7, 8), F)
        for j in range(7):
            blk[j] = np.array([np.float32(np.float64(v[j]) * np.float64(p) + np.float64(s[e][j])) for p in pct], F)
            # fma(v, pct, s): exact product + one rounding == float64 here (24-bit operands)
        back = (v / F(8 * n[e])).astype(F)
        first = None
        for i in range(n[e]):
            if i:
                blk = (blk - back[:, None]).astype(F)
            if not vamp.panda_0_0.cpu_fkcc_block(blk, env):
                first = i
                break
        assert first is not None and ev[e] == first + 1


@pytest.mark.parametrize("seed", [1, 2])
def test_mixed_primitives(vamp, oracle, seed):
    rng = np.random.default_rng(seed)
    oenv = random_scene(oracle, rng)
    env = gpu_env_from_oracle(vamp, oenv)
    q = oracle.scale(rng.random((8000, 7), dtype=F))
    for base in ((0, 0, 0), (200, 200, 0)):
        assert np.array_equal(vamp.PandaBase(*base).cpu_fkcc_batch(q, env), oracle.fkcc_threads(oenv, q, base))
    s = oracle.scale(rng.random((2000, 7), dtype=F))
    g = oracle.scale(rng.random((2000, 7), dtype=F))
    g[:1000] = s[:1000] + (g[:1000] - s[:1000]) * F(0.1)
    g[:4] = s[:4]  # zero-length
    ok, n, _ = vamp.panda_0_0.cpu_validate_batch(s, g, env)
    ook, on = oracle.validate_motions(oenv, s, g, (0, 0, 0))
    assert np.array_equal(n, on) and np.array_equal(ok, ook)


def test_pointcloud_and_heightfield(vamp, oracle):
    rng = np.random.default_rng(61)
    prim = random_scene(oracle, rng, n_sph=2, n_cub=2, n_cap=2)
    hf = terrain(seed=3)
    hf = ((0.2, -0.1, -0.4), hf[1], hf[2], hf[3])
    oenv = oracle.Env()
    for k in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(oenv, k, list(getattr(prim, k)))
    center, scale, dims, data = hf
    oenv.add_heightfield(center, scale, dims[0], dims[1], data)
    oenv.add_pointcloud(cage_points(), R_MIN, R_MAX, R_POINT)
    env = gpu_env_from_oracle(vamp, prim)
    env.add_heightfield(vamp.make_heightfield(*hf))
    env.add_pointcloud(cage_points(), R_MIN, R_MAX, R_POINT)
    q = oracle.scale(rng.random((3000, 7), dtype=F))
    assert np.array_equal(vamp.panda_0_0.cpu_fkcc_batch(q, env), oracle.fkcc(oenv, q, (0, 0, 0), G=1))
    s, g = oracle.scale(rng.random((600, 7), dtype=F)), oracle.scale(rng.random((600, 7), dtype=F))
    g = (s + (g - s) * F(0.15)).astype(F)
    ok, n, _ = vamp.panda_0_0.cpu_validate_batch(s, g, env)
    wok, wn = oracle.validate_motions(oenv, s, g)
    assert np.array_equal(n, wn) and np.array_equal(ok, wok)


@pytest.mark.parametrize("robot", sorted(CASES))
def test_robots_vs_oracle_and_fixture(vamp, oracle, robot):
    fx = host_fixture(CASES[robot], oracle)
    oenv = scene_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    rob = getattr(vamp, robot)
    same = same_rsqrt_host(oracle, fx)
    got = rob.cpu_fkcc_batch(fx["q"], env)
    assert np.array_equal(got, oracle.robot_fkcc_threads(robot, oenv, fx["q"]))
    fixture_check(f"{robot} fkcc (CPU rake)", got, fx["valid"], stable(fx["test_margin"], fx["cull_margin"], same),
                  same)
    ok, n, _ = rob.cpu_validate_batch(fx["starts"], fx["goals"], env)
    rok, rn = oracle.robot_validate_motions(robot, oenv, fx["starts"], fx["goals"])
    assert np.array_equal(n, rn) and np.array_equal(ok, rok)
    fixture_check(f"{robot} validate_motion (CPU rake)", ok, fx["ok"],
                  stable(fx["edge_test_margin"], fx["edge_cull_margin"], same), same, EDGE_MIN_COVERAGE)


@pytest.mark.parametrize("robot", ["panda", "fetch", "ur5", "baxter"])
def test_sphere_fk_block(vamp, oracle, robot):
    rob = vamp.panda_0_0 if robot == "panda" else getattr(vamp, robot)
    dim = rob.dimension()
    rng = np.random.default_rng(7)
    q = rob.scale_configuration(rng.random((8, dim), dtype=F))
    got = rob.cpu_sphere_fk_block(q.T)  # [3][S][8]
    want = oracle.sphere_fk(q, (0, 0, 0)) if robot == "panda" else oracle.robot_sphere_fk(robot, q)
    assert np.array_equal(got.transpose(2, 1, 0), want)


def test_attachment(vamp, oracle):
    fx = host_fixture("attach_panda_cage.npz", oracle)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    tf, rows = fx["att_tf"], fx["att_spheres"]
    a = vamp.Attachment(tf[:3], tf[3:])
    o = oracle.Attachment(tf[:3], tf[3:])
    for r in rows:
        a.add_sphere(vamp.Sphere(r[:3], r[3]))
        o.add_sphere(r[:3], r[3])
    env.attach(a)
    same = same_rsqrt_host(oracle, fx)
    for tag, base in (("b000", (0, 0, 0)), ("b220", (200, 200, 0))):
        q = fx["q_" + tag]
        got = vamp.PandaBase(*base).cpu_fkcc_batch(q, env, attach=True)
        assert np.array_equal(got, oracle.robot_fkcc_attach_threads("panda", oenv, o, q, base))
        m = stable(fx["test_margin_" + tag], fx["cull_margin_" + tag], same)
        fixture_check(f"panda fkcc_attach {tag} (CPU rake)", got, fx["valid_" + tag], m, same)
    ok, n, _ = vamp.panda_0_0.cpu_validate_batch(fx["starts"], fx["goals"], env)
    ook, on = oracle.robot_validate_motions_att("panda", oenv, o, fx["starts"], fx["goals"])
    assert np.array_equal(n, on) and np.array_equal(ok, ook)
    # vamp.<robot>.validate(q, env) = validate_motion(q, q, env): the attachment is checked
    # (validate.hh:43, bindings/common.hh:172-182) -- it disagrees with the plain fkcc where only the
    # held object collides
    q = fx["q_b000"][:400]
    inside = ((vamp.panda_0_0.descale_configuration(q) >= 0) & (vamp.panda_0_0.descale_configuration(q) <= 1)).all(1)
    want = vamp.panda_0_0.cpu_fkcc_batch(q, env, attach=True) & inside
    got = np.array([vamp.panda_0_0.validate(x, env) for x in q])
    assert np.array_equal(got, want)
    assert (got != (vamp.panda_0_0.cpu_fkcc_batch(q, env) & inside)).any()


def test_pair(vamp, oracle):
    rng = np.random.default_rng(9)
    oenv = oracle.pair_scene()
    env = gpu_env_from_oracle(vamp, oenv)
    u = rng.random((3000, 14), dtype=F)
    q = np.concatenate([oracle.scale(u[:, :7]), oracle.scale(u[:, 7:])], 1)
    assert np.array_equal(vamp.panda_pair.cpu_fkcc_batch(q, env), oracle.pair_fkcc_threads(oenv, q))
    s, g = q[:1000], q[1000:2000].copy()
    g = (s + (g - s) * F(0.1)).astype(F)
    ok, n, _ = vamp.panda_pair.cpu_validate_batch(s, g, env)
    rok, rn = oracle.pair_validate_motions(oenv, s, g)
    assert np.array_equal(n, rn) and np.array_equal(ok, rok)


def test_single_calls_and_errors(vamp, oracle):
    from vamp_amd import _lib
    lib = _lib.load()
    env = vamp.Environment()
    q0 = np.zeros(7, F)
    q0[3] = -1.5
    assert vamp.panda_0_0.validate(q0, env) == bool(oracle.fkcc(oracle.Env(), q0[None])[0])
    q_out = q0.copy()
    q_out[0] = 3.5
    assert vamp.panda_0_0.validate(q_out, env) is False
    assert vamp.panda_0_0.validate_motion(q0, q0, env) == vamp.panda_0_0.validate(q0, env)
    assert len(vamp.panda.fk(q0)) == 59
    v = C.c_int()
    blk = np.zeros((7, 8), F)
    bad = _lib.VgpuRobot(99, 0, 0, 0, 0, 0, 0)
    assert lib.vgpu_cpu_fkcc_block(C.byref(bad), env.host_handle(), blk.ctypes.data_as(_lib.F32P), C.byref(v)) == -4
    fetch_off = _lib.VgpuRobot(_lib.VGPU_ROBOT_FETCH, 10, 0, 0, 0, 0, 0)
    assert lib.vgpu_cpu_fkcc_block(C.byref(fetch_off), env.host_handle(), blk.ctypes.data_as(_lib.F32P),
                                   C.byref(v)) == -1
    assert lib.vgpu_cpu_fkcc_attach_block(C.byref(vamp.panda_0_0.c_robot), env.host_handle(),
                                          blk.ctypes.data_as(_lib.F32P), C.byref(v)) == -1  # nothing attached
    assert vamp.panda_0_0.cpu_fkcc_batch(np.zeros((0, 7), F), env).shape == (0,)


def rake_blocks(s, g, n):
    """the rake blocks validate_vector enumerates (validate.hh:31-56): block 0 = fma(v, (l+1)/8, s),
    then n - 1 back-steps of v / (8 n); returns [n][8][dim]"""
    v = (g - s).astype(F)
    pct = np.arange(1, 9, dtype=np.float64) / 8.0
    b = (v.astype(np.float64)[None, :] * pct[:, None] + s.astype(np.float64)[None, :]).astype(F)  # exact fma here
    back = (v / F(8 * n)).astype(F)
    out = [b]
    for _ in range(1, n):
        b = (b - back[None, :]).astype(F)
        out.append(b)
    return np.stack(out)


def test_full_mask_blocks(vamp, oracle):
    """full-mask mode: every block of every edge, each block's result == the oracle's fkcc of that
    8-lane block (group semantics); the edge result == the early-exit validate_motion."""
    fx = host_fixture("edges_panda_cage.npz", oracle)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    s, g = fx["starts"][:600], fx["goals"][:600]
    ok, n, blk, off = vamp.panda_0_0.cpu_validate_mask(s, g, env, threads=4)
    ook, on = oracle.validate_motions(oenv, s, g, (0, 0, 0))
    assert np.array_equal(ok, ook) and np.array_equal(n, on) and off[-1] == blk.size == n.sum()
    for e in range(0, 600, 7):
        want = oracle.fkcc(oenv, rake_blocks(s[e], g[e], int(n[e])).reshape(-1, 7), (0, 0, 0), G=8)
        assert np.array_equal(blk[off[e]:off[e + 1]], want), e
    # a rejected edge may have valid later blocks: the full mask evaluates them anyway
    tails = [blk[off[e] + 1:off[e + 1]] for e in np.flatnonzero(~ok) if n[e] > 1]
    assert any(t.any() for t in tails)
