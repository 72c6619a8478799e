"""GPU parity for Fetch (robots/fetch.hh): sphere_fk, per-configuration masks, validate_motion
and the fused Halton<8> -> scale -> fkcc PRM sampling stage, through the C ABI, against the C
restatement (bit-exact, same host) and the reference-DAG fixtures of fetch/fk.hh
(tests/golden/fk_fetch.npz, fetch_table_pick.npz; contract tolerances of tests/test_oracle.py).
"""
import numpy as np
import pytest

from conftest import golden, host_fixture
from test_gpu_parity import gpu_env_from_oracle
from test_oracle import EDGE_MIN_COVERAGE, FK_TOL, fixture_check, same_rsqrt_host, stable
from test_oracle_fetch import fetch_env

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None  # raises without a device / library
    return vamp_amd


def test_fetch_sphere_fk(vamp, oracle):
    fx = host_fixture("fk_fetch.npz", oracle)
    got = vamp.fetch.sphere_fk_batch(fx["q"])
    assert np.abs(got - fx["xyz"]).max() <= FK_TOL
    assert np.array_equal(got, oracle.robot_sphere_fk("fetch", fx["q"]))


def test_fetch_fkcc_table_pick(vamp, oracle):
    fx = host_fixture("fetch_table_pick.npz", oracle)
    oenv = fetch_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    got = vamp.fetch.fkcc_batch(fx["q"], env)
    assert np.array_equal(got, oracle.robot_fkcc_threads("fetch", oenv, fx["q"]))
    m = stable(fx["test_margin"], fx["cull_margin"], same_rsqrt_host(oracle, fx))
    fixture_check("fetch fkcc table_pick (GPU)", got, fx["valid"], m, same_rsqrt_host(oracle, fx))
    empty = vamp.Environment()
    got_e = vamp.fetch.fkcc_batch(fx["q_empty"], empty)
    assert np.array_equal(got_e, oracle.robot_fkcc_threads("fetch", oracle.Env(), fx["q_empty"]))


def test_fetch_validate_table_pick(vamp, oracle):
    fx = host_fixture("fetch_table_pick.npz", oracle)
    oenv = fetch_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    ok, n = vamp.fetch.validate_batch(fx["starts"], fx["goals"], env)
    rok, rn = oracle.robot_validate_motions("fetch", oenv, fx["starts"], fx["goals"])
    assert np.array_equal(n, rn) and np.array_equal(n, fx["n"])
    assert np.array_equal(ok, rok)
    m = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same_rsqrt_host(oracle, fx))
    fixture_check("fetch validate_motion table_pick (GPU)", ok, fx["ok"], m, same_rsqrt_host(oracle, fx), EDGE_MIN_COVERAGE)


def test_fetch_validate_long_edges(vamp, oracle):
    """raw full-range edges (n_e up to ~40 blocks) and zero-length edges, empty + table scene"""
    rng = np.random.default_rng(11)
    fx = host_fixture("fetch_table_pick.npz", oracle)
    oenv = fetch_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    s = oracle.robot_scale("fetch", rng.random((3000, 8), dtype=F))
    g = oracle.robot_scale("fetch", rng.random((3000, 8), dtype=F))
    g[:16] = s[:16]
    for e_o, e_g in ((oenv, env), (oracle.Env(), vamp.Environment())):
        ok, n = vamp.fetch.validate_batch(s, g, e_g)
        rok, rn = oracle.robot_validate_motions("fetch", e_o, s, g)
        assert np.array_equal(n, rn)
        assert np.array_equal(ok, rok)


def test_fetch_sample_fkcc(vamp, oracle):
    """PRM vertex stage: Halton<8> draws across the first reset, fused with scale + fkcc"""
    fx = host_fixture("fetch_table_pick.npz", oracle)
    oenv = fetch_env(oracle, fx)
    n, first = 8192, 996_000
    q, ok = vamp.fetch.sample_fkcc(first, n, gpu_env_from_oracle(vamp, oenv))
    qo = oracle.robot_scale("fetch", oracle.halton(8, np.arange(first, first + n)))
    assert np.array_equal(q.view(np.uint32), qo.view(np.uint32))
    assert np.array_equal(ok, oracle.robot_fkcc_threads("fetch", oenv, qo))


def test_roadmap_vertices_single_gpu(vamp, oracle):
    """build_roadmap's vertex sequence (prm.hh:228-254): start, goal, then the valid Halton<8>
    samples in draw order, truncated at max_samples -- through the sharded entry point
    (one rank here; the all-gather itself is covered by tests/test_roadmap_dist.py)."""
    import torch
    from vamp_amd import roadmap
    fx = host_fixture("fetch_table_pick.npz", oracle)
    oenv = fetch_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    n, first = 30000, 990_001
    s, g = fx["starts"][-1], fx["goals"][-1]
    V, D = roadmap.roadmap_vertices(vamp.fetch, env, n, first=first, start=s, goal=g)
    torch.cuda.synchronize()
    qo = oracle.robot_scale("fetch", oracle.halton(8, np.arange(first, first + n)))
    ok = oracle.robot_fkcc_threads("fetch", oenv, qo)
    want = np.concatenate([s[None], g[None], qo[ok]])
    assert np.array_equal(V.cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert np.array_equal(D.cpu().numpy()[2:], np.nonzero(ok)[0] + first)
    V2, _ = roadmap.roadmap_vertices(vamp.fetch, env, n, first=first, start=s, goal=g, max_samples=1000)
    assert V2.shape[0] == 1000 and torch.equal(V2, V[:1000])
