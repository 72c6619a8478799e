"""Attachments (collision/attachments.hh:14-123): the C restatement's fkcc_attach and the
first-block-only rake branch (planning/validate.hh:43) against the reference's generated
`interleaved_sphere_fk_attachment` (robots/panda/fk.hh:6278-11397), interpreted by
tools/fkhh_interp.py (fixture from tools/make_golden.py --attach).

Object: tests/oracle_py.py:held_object (four spheres of r 3 cm along the hand's z axis, frame
turned 45 degrees).  Scene: the sphere cage.  Same tolerances as tests/test_oracle.py.
"""
import numpy as np
import pytest

from conftest import golden, host_fixture
from test_oracle import stable, same_rsqrt_host


def _att(oracle, fx):
    a = oracle.Attachment(fx["att_tf"][:3], fx["att_tf"][3:])
    for s in fx["att_spheres"]:
        a.add_sphere(s[:3], s[3])
    return a


def test_attachment_fixture_is_the_held_object(oracle):
    fx = host_fixture("attach_panda_cage.npz", oracle)
    ref = oracle.held_object().as_dict()
    assert np.array_equal(fx["att_tf"], ref["tf"]) and np.array_equal(fx["att_spheres"], ref["spheres"])


def test_fkcc_attach_mask_vs_reference_dag(oracle):
    fx = host_fixture("attach_panda_cage.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    env = oracle.sphere_cage_env()
    att = _att(oracle, fx)
    for tag, base in (("b000", (0, 0, 0)), ("b220", (200, 200, 0))):
        got = oracle.robot_fkcc_attach_threads("panda", env, att, fx["q_" + tag], base)
        m = stable(fx["test_margin_" + tag], fx["cull_margin_" + tag], same)
        assert m.mean() > 0.95
        assert np.array_equal(got[m], fx["valid_" + tag][m]), tag
        assert int((got != fx["valid_" + tag]).sum()) <= 2
        # the object matters: some configurations valid without it collide with it
        plain = fx["plain_" + tag]
        assert (plain & ~fx["valid_" + tag]).sum() > 0 and not (~plain & fx["valid_" + tag]).any()


def test_validate_motion_attach_vs_reference_dag(oracle):
    fx = host_fixture("attach_panda_cage.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    env = oracle.sphere_cage_env()
    ok, n = oracle.robot_validate_motions_att("panda", env, _att(oracle, fx), fx["starts"], fx["goals"])
    assert np.array_equal(n, fx["n"])
    m = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same)
    assert np.array_equal(ok[m], fx["ok"][m])
    assert int((ok != fx["ok"]).sum()) <= 2


def test_attach_without_spheres_equals_fkcc(oracle):
    """An attachment with no spheres adds no checks: fkcc_attach == fkcc."""
    rng = np.random.default_rng(5)
    q = oracle.scale(rng.random((2048, 7), dtype=np.float32))
    env = oracle.sphere_cage_env()
    empty = oracle.Attachment((0, 0, 0), (0, 0, 0, 1))
    empty.spheres = []
    a = oracle.robot_fkcc_attach_threads("panda", env, empty, q)
    b = oracle.fkcc_threads(env, q)
    assert np.array_equal(a, b)


def _mbm_env(oracle, fx):
    e = oracle.Env()
    for k in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(e, k, [list(r) for r in fx["env_" + k]])
    return e


@pytest.mark.parametrize("robot", ["ur5", "fetch"])
def test_robot_fkcc_attach_vs_reference_dag(oracle, robot):
    """Fetch (fetch.hh:42) and UR5 (ur5.hh:43) fkcc_attach = their generated
    interleaved_sphere_fk_attachment, on their MBM table_pick scene; edges with the first block
    through it."""
    import os
    from conftest import GOLD
    if not os.path.exists(os.path.join(GOLD, f"attach_{robot}.npz")):
        pytest.skip("fixture not generated")
    fx = host_fixture(f"attach_{robot}.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    env = _mbm_env(oracle, fx)
    att = _att(oracle, fx)
    got = oracle.robot_fkcc_attach_threads(robot, env, att, fx["q"])
    m = stable(fx["test_margin"], fx["cull_margin"], same)
    assert m.mean() > 0.9
    assert np.array_equal(got[m], fx["valid"][m])
    assert int((got != fx["valid"]).sum()) <= max(2, int(2e-4 * len(got)))
    assert (fx["plain"] & ~fx["valid"]).sum() > 0
    ok, n = oracle.robot_validate_motions_att(robot, env, att, fx["starts"], fx["goals"])
    assert np.array_equal(n, fx["n"])
    me = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same)
    assert np.array_equal(ok[me], fx["ok"][me])


def test_baxter_fkcc_attach_is_fkcc(oracle):
    """Baxter's fkcc_attach is its plain interleaved_sphere_fk (baxter.hh:44): the attachment is
    not checked."""
    rng = np.random.default_rng(6)
    q = oracle.robot_scale("baxter", rng.random((1024, 14), dtype=np.float32))
    env = oracle.sphere_cage_env()
    att = oracle.held_object()
    assert np.array_equal(oracle.robot_fkcc_attach_threads("baxter", env, att, q),
                          oracle.robot_fkcc_threads("baxter", env, q))
