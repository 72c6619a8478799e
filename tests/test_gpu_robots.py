"""GPU parity for the UR5 (staged pipeline) and Baxter (monolithic, 388 checks) through the C ABI:
sphere_fk, per-configuration masks, validate_motion (Baxter: resolution 64, two-register
l2_norm) and the fused Halton sampler, bit-exact against the C restatement and, margin-filtered,
against the reference-DAG fixtures (tests/test_oracle_robots.py)."""
import numpy as np
import pytest

from conftest import golden, host_fixture
from test_gpu_parity import gpu_env_from_oracle
from test_oracle import EDGE_MIN_COVERAGE, FK_TOL, fixture_check, same_rsqrt_host, stable
from test_oracle_robots import CASES, scene_env

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


@pytest.mark.parametrize("robot", sorted(CASES))
def test_sphere_fk(vamp, oracle, robot):
    fx = host_fixture(f"fk_{robot}.npz", oracle)
    got = getattr(vamp, robot).sphere_fk_batch(fx["q"])
    assert np.abs(got - fx["xyz"]).max() <= FK_TOL
    assert np.array_equal(got, oracle.robot_sphere_fk(robot, fx["q"]))


@pytest.mark.parametrize("robot", sorted(CASES))
def test_fkcc(vamp, oracle, robot):
    fx = host_fixture(CASES[robot], oracle)
    oenv = scene_env(oracle, fx)
    rob = getattr(vamp, robot)
    got = rob.fkcc_batch(fx["q"], gpu_env_from_oracle(vamp, oenv))
    assert np.array_equal(got, oracle.robot_fkcc_threads(robot, oenv, fx["q"]))
    m = stable(fx["test_margin"], fx["cull_margin"], same_rsqrt_host(oracle, fx))
    fixture_check(f"{robot} fkcc {CASES[robot]} (GPU)", got, fx["valid"], m, same_rsqrt_host(oracle, fx))
    got_e = rob.fkcc_batch(fx["q_empty"], vamp.Environment())
    assert np.array_equal(got_e, oracle.robot_fkcc_threads(robot, oracle.Env(), fx["q_empty"]))


@pytest.mark.parametrize("robot", sorted(CASES))
def test_validate(vamp, oracle, robot):
    fx = host_fixture(CASES[robot], oracle)
    oenv = scene_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    rob = getattr(vamp, robot)
    ok, n = rob.validate_batch(fx["starts"], fx["goals"], env)
    rok, rn = oracle.robot_validate_motions(robot, oenv, fx["starts"], fx["goals"])
    assert np.array_equal(n, rn) and np.array_equal(n, fx["n"])
    assert np.array_equal(ok, rok)
    me = stable(fx["edge_test_margin"], fx["edge_cull_margin"], same_rsqrt_host(oracle, fx))
    fixture_check(f"{robot} validate_motion {CASES[robot]} (GPU)", ok, fx["ok"], me, same_rsqrt_host(oracle, fx), EDGE_MIN_COVERAGE)
    dim = oracle.ROBOTS[robot][1]
    rng = np.random.default_rng(13)
    s = oracle.robot_scale(robot, rng.random((1500, dim), dtype=F))
    g = oracle.robot_scale(robot, rng.random((1500, dim), dtype=F))
    g[:8] = s[:8]
    ok, n = rob.validate_batch(s, g, env)
    rok, rn = oracle.robot_validate_motions(robot, oenv, s, g)
    assert np.array_equal(n, rn) and np.array_equal(ok, rok)


@pytest.mark.parametrize("robot", sorted(CASES))
def test_sample_fkcc(vamp, oracle, robot):
    fx = host_fixture(CASES[robot], oracle)
    oenv = scene_env(oracle, fx)
    dim = oracle.ROBOTS[robot][1]
    n, first = 4096, 998_000
    q, ok = getattr(vamp, robot).sample_fkcc(first, n, gpu_env_from_oracle(vamp, oenv))
    qo = oracle.robot_scale(robot, oracle.halton(dim, np.arange(first, first + n)))
    assert np.array_equal(q.view(np.uint32), qo.view(np.uint32))
    assert np.array_equal(ok, oracle.robot_fkcc_threads(robot, oenv, qo))
