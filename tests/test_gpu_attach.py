"""GPU parity of the attachment path: Robot::fkcc_attach
(panda/fk.hh:6278-11397) and validate_motion's first-block branch (planning/validate.hh:43),
through the C ABI, against the C restatement on the same host (bit for bit) and the
reference-DAG fixture tests/golden/attach_panda_cage.npz (margin-filtered)."""
import numpy as np
import pytest

from conftest import golden, host_fixture
from test_gpu_parity import gpu_env_from_oracle, random_scene
from test_oracle import EDGE_MIN_COVERAGE, fixture_check, same_rsqrt_host, stable

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def both(vamp, oracle, fx=None):
    """The held object as a product Attachment and as an oracle Attachment."""
    tf = fx["att_tf"] if fx is not None else oracle.held_object().tf
    rows = fx["att_spheres"] if fx is not None else np.array(oracle.held_object().spheres, F)
    a = vamp.Attachment(tf[:3], tf[3:])
    o = oracle.Attachment(tf[:3], tf[3:])
    for r in rows:
        a.add_sphere(vamp.Sphere(r[:3], r[3]))
        o.add_sphere(r[:3], r[3])
    return a, o


def test_fkcc_attach_cage(vamp, oracle):
    fx = host_fixture("attach_panda_cage.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    a, o = both(vamp, oracle, fx)
    env.attach(a)
    for tag, base in (("b000", (0, 0, 0)), ("b220", (200, 200, 0))):
        q = fx["q_" + tag]
        got = vamp.PandaBase(*base).fkcc_attach_batch(q, env)
        assert np.array_equal(got, oracle.robot_fkcc_attach_threads("panda", oenv, o, q, base)), tag
        m = stable(fx["test_margin_" + tag], fx["cull_margin_" + tag], same)
        fixture_check(f"panda fkcc_attach cage {tag} (GPU)", got, fx["valid_" + tag], m, same)
        # validate(q) ignores attachments (bindings: fkcc, not fkcc_attach)
        assert np.array_equal(vamp.PandaBase(*base).fkcc_batch(q, env), oracle.fkcc_threads(oenv, q, base))


def test_validate_attach_cage(vamp, oracle):
    fx = host_fixture("attach_panda_cage.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    a, o = both(vamp, oracle, fx)
    env.attach(a)
    ok, n = vamp.panda_0_0.validate_batch(fx["starts"], fx["goals"], env)
    ook, on = oracle.robot_validate_motions_att("panda", oenv, o, fx["starts"], fx["goals"])
    assert np.array_equal(n, on) and np.array_equal(n, fx["n"])
    assert np.array_equal(ok, ook), "GPU != oracle on the same host"
    m = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same)
    fixture_check("panda attached validate_motion cage (GPU)", ok, fx["ok"], m, same, EDGE_MIN_COVERAGE)
    assert (~ok).sum() > 0 and ok.sum() > 0
    env.detach()
    ok2, _ = vamp.panda_0_0.validate_batch(fx["starts"], fx["goals"], env)
    ook2, _ = oracle.validate_motions(oenv, fx["starts"], fx["goals"], (0, 0, 0))
    assert np.array_equal(ok2, ook2) and (ok2 & ~ok).sum() > 0


@pytest.mark.parametrize("seed", [4, 5])
def test_attach_mixed_primitives(vamp, oracle, seed):
    """All five primitive types and a larger object (12 spheres)."""
    rng = np.random.default_rng(seed)
    oenv = random_scene(oracle, rng)
    env = gpu_env_from_oracle(vamp, oenv)
    a = vamp.Attachment(rng.uniform(-0.05, 0.05, 3).astype(F), (0.0, 0.0, 0.0, 1.0))
    o = oracle.Attachment(a.tf[:3], a.tf[3:])
    for _ in range(12):
        c, r = rng.uniform(-0.1, 0.1, 3).astype(F), F(rng.uniform(0.01, 0.05))
        a.add_sphere(vamp.Sphere(c, r))
        o.add_sphere(c, r)
    env.attach(a)
    q = oracle.scale(rng.random((16384, 7), dtype=F))
    got = vamp.panda_0_0.fkcc_attach_batch(q, env)
    assert np.array_equal(got, oracle.robot_fkcc_attach_threads("panda", oenv, o, q))
    s = oracle.scale(rng.random((3000, 7), dtype=F))
    g = oracle.scale(rng.random((3000, 7), dtype=F))
    g[:1500] = s[:1500] + (g[:1500] - s[:1500]) * F(0.1)
    ook, on = oracle.robot_validate_motions_att("panda", oenv, o, s, g)
    ok, n = vamp.panda_0_0.validate_batch(s, g, env)
    assert np.array_equal(n, on) and np.array_equal(ok, ook)


def _mbm_env(vamp, oracle, fx):
    o = oracle.Env()
    for k in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(o, k, [list(r) for r in fx["env_" + k]])
    return o, gpu_env_from_oracle(vamp, o)


@pytest.mark.parametrize("robot", ["fetch", "ur5"])
def test_robot_attach(vamp, oracle, robot):
    """Fetch / UR5 fkcc_attach and the attached rake on their MBM scene: GPU == oracle on the
    same host, and == the reference-DAG fixture on the margin-filtered set."""
    fx = host_fixture(f"attach_{robot}.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    oenv, env = _mbm_env(vamp, oracle, fx)
    a, o = both(vamp, oracle, fx)
    env.attach(a)
    r = getattr(vamp, robot)
    got = r.fkcc_attach_batch(fx["q"], env)
    assert np.array_equal(got, oracle.robot_fkcc_attach_threads(robot, oenv, o, fx["q"]))
    m = stable(fx["test_margin"], fx["cull_margin"], same)
    fixture_check(f"{robot} fkcc_attach table_pick (GPU)", got, fx["valid"], m, same)
    ok, n = r.validate_batch(fx["starts"], fx["goals"], env)
    ook, on = oracle.robot_validate_motions_att(robot, oenv, o, fx["starts"], fx["goals"])
    assert np.array_equal(n, on) and np.array_equal(ok, ook)
    me = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same)
    fixture_check(f"{robot} attached validate_motion table_pick (GPU)", ok, fx["ok"], me, same, EDGE_MIN_COVERAGE)


def test_baxter_attach_is_plain(vamp, oracle):
    """Baxter::fkcc_attach = interleaved_sphere_fk (baxter.hh:44): an attachment changes nothing."""
    rng = np.random.default_rng(8)
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    q = oracle.robot_scale("baxter", rng.random((2048, 14), dtype=F))
    s, g = q[:1024], q[1024:]
    plain_ok, plain_n = vamp.baxter.validate_batch(s, g, env)
    a, _ = both(vamp, oracle)
    env.attach(a)
    ok, n = vamp.baxter.validate_batch(s, g, env)
    assert np.array_equal(ok, plain_ok) and np.array_equal(n, plain_n)
    assert np.array_equal(vamp.baxter.fkcc_attach_batch(q, env), oracle.robot_fkcc_threads("baxter", oenv, q))


def test_attach_composite_refused(vamp, oracle):
    env = vamp.Environment()
    a, _ = both(vamp, oracle)
    env.attach(a)
    q = np.zeros((4, 14), F)
    with pytest.raises(vamp.VgpuError):
        vamp.panda_pair.validate_batch(q, q, env)
