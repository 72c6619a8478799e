"""Near sets (vgpu_device.hh env_near / env_bits_near): a check's children scan only the obstacle records a sphere
enclosing all of them touches.  Exactness rests on containment (a child hitting a record means the enclosing sphere
hits it too), which holds for distance-valued tests only -- so these cases probe the edges of the argument against
the oracle, configs and motions, at two robot bases:

* environments of 63, 64 and 65 primitive records (the last one past kNearMax: one bit per record no longer fits,
  the scan falls back to every culled record) and 100 records;
* cuboids whose axes are not orthonormal (their test value is no distance: always near) placed where the arm
  moves;
* obstacles crowded around the robot base, where enclosing spheres of the first links reach the origin (their cull
  becomes infinite) and a child centre can sit near 0.
"""
import numpy as np
import pytest

from test_gpu_parity import gpu_env_from_oracle, random_scene

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def check(vamp, oracle, oenv, rng, n_cfg=12000, n_edges=2000):
    env = gpu_env_from_oracle(vamp, oenv)
    q = oracle.scale(rng.random((n_cfg, 7), dtype=F))
    for base in ((0, 0, 0), (2, 2, 0)):
        got = vamp.PandaBase(*base).fkcc_batch(q, env)
        want = oracle.fkcc_threads(oenv, q, base)
        assert np.array_equal(got, want), (base, int((got != want).sum()))
    s = oracle.scale(rng.random((n_edges, 7), dtype=F))
    g = oracle.scale(rng.random((n_edges, 7), dtype=F))
    g[: n_edges // 2] = s[: n_edges // 2] + (g[: n_edges // 2] - s[: n_edges // 2]) * F(0.1)
    ok, n = vamp.panda_0_0.validate_batch(s, g, env)
    ook, on = oracle.validate_motions(oenv, s, g, (0, 0, 0))
    assert np.array_equal(n, on) and np.array_equal(ok, ook)
    return float(np.mean(ook))


@pytest.mark.parametrize("n_sph,n_cub,n_cap", [(23, 20, 20), (24, 20, 20), (25, 20, 20), (40, 30, 30)])
def test_record_counts_around_the_near_limit(vamp, oracle, n_sph, n_cub, n_cap):
    rng = np.random.default_rng(n_sph * 1000 + n_cub)
    oenv = random_scene(oracle, rng, n_sph=n_sph, n_cub=n_cub, n_cap=n_cap)
    frac = check(vamp, oracle, oenv, rng)
    print(f"near limit: {n_sph + n_cub + n_cap} records, edges valid {frac:.3f}", flush=True)


def sheared_scene(oracle, rng, n=12):
    e = oracle.Env()
    for _ in range(n):
        c = rng.uniform([-0.7, -0.7, 0.05], [0.7, 0.7, 1.0]).astype(F)
        A = np.eye(3) + rng.uniform(-0.35, 0.35, (3, 3))  # sheared, unnormalised axes
        h = rng.uniform(0.02, 0.08, 3).astype(F)
        e.add_cuboid_axes(c, A[0].astype(F), A[1].astype(F), A[2].astype(F), h)
    for _ in range(4):
        e.add_sphere(rng.uniform([-0.7, -0.7, 0.0], [0.7, 0.7, 1.0]).astype(F), F(rng.uniform(0.03, 0.08)))
    return e


@pytest.mark.parametrize("seed", [5, 6])
def test_non_orthonormal_cuboids(vamp, oracle, seed):
    rng = np.random.default_rng(seed)
    frac = check(vamp, oracle, sheared_scene(oracle, rng), rng)
    print(f"sheared cuboids: edges valid {frac:.3f}", flush=True)


def test_obstacles_at_the_base(vamp, oracle):
    rng = np.random.default_rng(11)
    e = oracle.Env()
    for _ in range(10):  # small spheres and boxes hugging the base and the first links
        e.add_sphere(rng.uniform([-0.25, -0.25, 0.0], [0.25, 0.25, 0.45]).astype(F), F(rng.uniform(0.005, 0.03)))
    for _ in range(6):
        a = rng.uniform(0, 2 * np.pi)
        e.add_cuboid_axes(rng.uniform([-0.3, -0.3, -0.05], [0.3, 0.3, 0.3]).astype(F),
                          np.array([np.cos(a), np.sin(a), 0], F), np.array([-np.sin(a), np.cos(a), 0], F),
                          np.array([0, 0, 1], F), rng.uniform(0.01, 0.05, 3).astype(F))
    frac = check(vamp, oracle, e, rng)
    print(f"obstacles at the base: edges valid {frac:.3f}", flush=True)
