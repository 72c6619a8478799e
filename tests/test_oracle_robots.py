"""The C restatement for the UR5 (robots/ur5.hh, 6 dof) and Baxter (robots/baxter.hh, 14-dof dual
arm, resolution 64) against the reference's generated robots/<robot>/fk.hh, interpreted by
tools/fkhh_interp.py (fixtures: tools/make_golden.py --ur5 / --baxter, on MotionBenchMaker
table_pick_ur5 scene0001 and bookshelf_tall_both_arms_easy_baxter scene0001).  Same contract as
tests/test_oracle.py: FK within 1e-5, masks/edges bit-exact on the margin-filtered set.
"""
import numpy as np
import pytest

from conftest import golden, host_fixture
from test_oracle import FK_TOL, stable, same_rsqrt_host

CASES = {"ur5": "ur5_table_pick.npz", "baxter": "baxter_bookshelf.npz"}


def scene_env(oracle, fx):
    e = oracle.Env()
    for k in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(e, k, [list(r) for r in fx["env_" + k]])
    return e


@pytest.mark.parametrize("robot", sorted(CASES))
def test_sphere_fk_vs_reference_dag(oracle, robot):
    fx = host_fixture(f"fk_{robot}.npz", oracle)
    got = oracle.robot_sphere_fk(robot, fx["q"])
    assert np.abs(got - fx["xyz"]).max() <= FK_TOL


@pytest.mark.parametrize("robot", sorted(CASES))
def test_fkcc_vs_reference_dag(oracle, robot):
    fx = host_fixture(CASES[robot], oracle)
    same = same_rsqrt_host(oracle, fx)
    got = oracle.robot_fkcc_threads(robot, scene_env(oracle, fx), fx["q"])
    m = stable(fx["test_margin"], fx["cull_margin"], same)
    assert m.mean() > 0.9
    assert np.array_equal(got[m], fx["valid"][m])
    assert int((got != fx["valid"]).sum()) <= max(2, int(2e-4 * len(got)))
    got_e = oracle.robot_fkcc_threads(robot, oracle.Env(), fx["q_empty"])
    me = fx["test_margin_empty"] > 1e-4
    assert np.array_equal(got_e[me], fx["valid_empty"][me])


@pytest.mark.parametrize("robot", sorted(CASES))
def test_validate_motion_vs_reference_dag(oracle, robot):
    fx = host_fixture(CASES[robot], oracle)
    same = same_rsqrt_host(oracle, fx)
    ok, n = oracle.robot_validate_motions(robot, scene_env(oracle, fx), fx["starts"], fx["goals"])
    assert np.array_equal(n, fx["n"])
    m = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same)
    assert np.array_equal(ok[m], fx["ok"][m])
    assert int((ok != fx["ok"]).sum()) <= 2
