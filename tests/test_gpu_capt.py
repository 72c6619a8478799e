"""GPU parity for point clouds (CAPT) and heightfields: raw CAPT queries, and fkcc /
validate_motion against environments holding them (validity.hh:133-148), HIP path through the
C ABI vs the C restatement, bit for bit on the same host."""
import numpy as np
import pytest

from scenes import R_MAX, R_MIN, R_POINT, cage_points, raw_queries, terrain
from test_gpu_parity import gpu_env_from_oracle, random_scene

pytestmark = pytest.mark.gpu
F = np.float32
S_M = np.array([5.9342, 3.6652, 5.9342, 3.2289, 5.9342, 3.9095999999999997, 5.9342], F)
S_A = np.array([-2.9671, -1.8326, -2.9671, -3.1416, -2.9671, -0.0873, -2.9671], F)


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def configs(n, seed):
    rng = np.random.default_rng(seed)
    return (S_A + rng.random((n, 7), dtype=F) * S_M).astype(F)


@pytest.mark.parametrize("simd", [False, True])
def test_raw_queries_bit_exact(vamp, oracle, simd):
    pts = cage_points()
    env = vamp.Environment()
    env.add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
    c, r = raw_queries(1 << 18)
    got = env.pointcloud_collides(c, r, simd=simd)
    want = oracle.Capt(pts, R_MIN, R_MAX, R_POINT).collides(c, r, simd=simd)
    assert np.array_equal(got, want)
    assert 0.02 < got.mean() < 0.5


def test_raw_queries_edge_cases(vamp, oracle):
    """one point (nlog2 = 0), two points, queries far outside, on points, zero batch."""
    for n in (1, 2, 3):
        pts = cage_points(n, 20 + n)
        env = vamp.Environment()
        env.add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
        c = np.concatenate([pts, pts + 0.05, np.array([[5, 5, 5], [-5, 0, 0]], F)]).astype(F)
        r = np.full(len(c), 0.03, F)
        for simd in (False, True):
            assert np.array_equal(env.pointcloud_collides(c, r, simd=simd),
                                  oracle.Capt(pts, R_MIN, R_MAX, R_POINT).collides(c, r, simd=simd))
    assert env.pointcloud_collides(np.zeros((0, 3), F), np.zeros(0, F)).shape == (0,)


def _oracle_pc_env(oracle, base_env=None):
    e = base_env or oracle.Env()
    e.add_pointcloud(cage_points(), R_MIN, R_MAX, R_POINT)
    return e


def _gpu_env(vamp, oenv, hf=None, pc=True):
    env = gpu_env_from_oracle(vamp, oenv)
    if hf is not None:
        env.add_heightfield(vamp.make_heightfield(*hf))
    if pc:
        env.add_pointcloud(cage_points(), R_MIN, R_MAX, R_POINT)
    return env


def test_fkcc_pointcloud_env(vamp, oracle):
    """per-configuration fkcc against a CAPT-only environment."""
    q = configs(8192, 31)
    oenv = _oracle_pc_env(oracle)
    want = oracle.fkcc(oenv, q, (0, 0, 0), G=1)
    got = vamp.panda_0_0.fkcc_batch(q, _gpu_env(vamp, oracle.Env()))
    assert np.array_equal(got, want)
    assert 0.1 < got.mean() < 0.95


def test_validate_pointcloud_env(vamp, oracle):
    rng = np.random.default_rng(32)
    s, g = configs(2048, 33), configs(2048, 34)
    g = (s + (g - s) * F(0.2)).astype(F)
    oenv = _oracle_pc_env(oracle)
    want_ok, want_n = oracle.validate_motions(oenv, s, g)
    ok, n = vamp.panda_0_0.validate_batch(s, g, _gpu_env(vamp, oracle.Env()))
    assert np.array_equal(n, want_n) and np.array_equal(ok, want_ok)
    del rng


def _oracle_hf_env(oracle, hf, base_env=None):
    e = base_env or oracle.Env()
    center, scale, dims, data = hf
    e.add_heightfield(center, scale, dims[0], dims[1], data)
    return e


def test_fkcc_heightfield_env(vamp, oracle):
    hf = terrain()
    hf = ((0.0, 0.0, -0.4), hf[1], hf[2], hf[3])  # terrain -0.275 .. -0.025 m: some arms dip in
    q = configs(8192, 41)
    want = oracle.fkcc(_oracle_hf_env(oracle, hf), q, (0, 0, 0), G=1)
    got = vamp.panda_0_0.fkcc_batch(q, _gpu_env(vamp, oracle.Env(), hf=hf, pc=False))
    assert np.array_equal(got, want)
    free = oracle.fkcc(oracle.Env(), q, (0, 0, 0), G=1)
    assert 0.01 < (free & ~got).mean() and got.mean() > 0.5  # the terrain removes some arms


@pytest.mark.parametrize("seed", [51, 52])
def test_all_obstacle_kinds(vamp, oracle, seed):
    """primitives of all five kinds + a heightfield + a point cloud, both G = 1 masks and edges."""
    rng = np.random.default_rng(seed)
    prim = random_scene(oracle, rng, n_sph=3, n_cub=3, n_cap=2)
    hf = terrain(seed=seed)
    hf = ((0.2, -0.1, -0.4), hf[1], hf[2], hf[3])
    oenv = _oracle_pc_env(oracle, _oracle_hf_env(oracle, hf, prim))
    genv = _gpu_env(vamp, prim, hf=hf, pc=True)
    q = configs(4096, seed + 100)
    assert np.array_equal(vamp.panda_0_0.fkcc_batch(q, genv), oracle.fkcc(oenv, q, (0, 0, 0), G=1))
    s, g = configs(1024, seed + 200), configs(1024, seed + 300)
    g = (s + (g - s) * F(0.15)).astype(F)
    ok, n = vamp.panda_0_0.validate_batch(s, g, genv)
    wok, wn = oracle.validate_motions(oenv, s, g)
    assert np.array_equal(n, wn) and np.array_equal(ok, wok)
