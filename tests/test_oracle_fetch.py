"""The C restatement for Fetch (robots/fetch.hh, 8 dof: prismatic torso + 7 revolute joints
about x/y/z axes) against the reference's generated fetch/fk.hh, interpreted by
tools/fkhh_interp.py (fixtures from tools/make_golden.py --fetch).

Scene: MotionBenchMaker table_pick_fetch scene0001 (resources/fetch/problems.tar.bz2), boxes as
cuboids and cylinders as capsules by resolved rows (tests/oracle_py.py:mbm_env).  Same
tolerances as tests/test_oracle.py: FK within 1e-5 abs, masks bit-exact on the margin-filtered
set, near-boundary flips counted.
"""
import numpy as np

from conftest import golden, host_fixture
from test_oracle import EDGE_MIN_COVERAGE, FK_TOL, fixture_check, same_rsqrt_host, stable


def fetch_env(oracle, fx):
    e = oracle.Env()
    for k in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(e, k, [list(r) for r in fx["env_" + k]])
    return e


def test_fetch_sphere_fk_vs_reference_dag(oracle):
    fx = host_fixture("fk_fetch.npz", oracle)
    got = oracle.robot_sphere_fk("fetch", fx["q"])
    err = np.abs(got - fx["xyz"]).max()
    assert err <= FK_TOL, err


def test_fetch_env_rows_rebuild(oracle):
    """The committed scene rows are what mbm_env builds (sorted by min_distance)."""
    fx = host_fixture("fetch_table_pick.npz", oracle)
    a = fetch_env(oracle, fx).arrays()
    for k in ("cuboids", "capsules"):
        assert np.array_equal(a[k], fx["env_" + k])
    assert len(a["cuboids"]) + len(a["zcuboids"]) >= 5 and len(a["capsules"]) + len(a["zcapsules"]) >= 1


def test_fetch_fkcc_mask_vs_reference_dag(oracle):
    fx = host_fixture("fetch_table_pick.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    env = fetch_env(oracle, fx)
    got = oracle.robot_fkcc_threads("fetch", env, fx["q"])
    m = stable(fx["test_margin"], fx["cull_margin"], same)
    assert m.mean() > 0.9  # 2634 self tests per configuration: more of them near a boundary than Panda
    fixture_check("fetch fkcc table_pick (oracle)", got, fx["valid"], m, same)
    assert int((got != fx["valid"]).sum()) <= max(2, int(2e-4 * len(got)))
    got_e = oracle.robot_fkcc_threads("fetch", oracle.Env(), fx["q_empty"])
    assert np.array_equal(got_e[fx["test_margin_empty"] > 1e-4], fx["valid_empty"][fx["test_margin_empty"] > 1e-4])


def test_fetch_validate_motion_vs_reference_dag(oracle):
    fx = host_fixture("fetch_table_pick.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    env = fetch_env(oracle, fx)
    ok, n = oracle.robot_validate_motions("fetch", env, fx["starts"], fx["goals"])
    assert np.array_equal(n, fx["n"])
    m = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same)
    fixture_check("fetch validate_motion table_pick (oracle)", ok, fx["ok"], m, same, EDGE_MIN_COVERAGE)
    assert int((ok != fx["ok"]).sum()) <= 2


def test_fetch_l2_norm_lane_order(oracle):
    """8-dof distance uses all eight AVX lanes in hsum order (avx.hh:441-452)."""
    import ctypes as C
    rng = np.random.default_rng(3)
    v = rng.normal(size=(256, 8)).astype(np.float32)
    sq = v * v
    want = np.sqrt(((sq[:, 0] + sq[:, 4]) + (sq[:, 2] + sq[:, 6])) + ((sq[:, 1] + sq[:, 5]) + (sq[:, 3] + sq[:, 7])))
    got = np.array([oracle.lib().vo_l2_norm(oracle.fp(np.ascontiguousarray(r)), 8) for r in v], np.float32)
    assert np.array_equal(got, want.astype(np.float32))
