"""GPU parity for the two-Panda composite (BASELINE configs[4]) through the C ABI
(VGPU_ROBOT_PANDA_PAIR): per-configuration masks and 14-dof validate_motion, bit-exact against
the C restatement (vo_pair_*) and, margin-filtered, against the DAG composition fixture."""
import numpy as np
import pytest

from conftest import golden, host_fixture
from test_gpu_parity import gpu_env_from_oracle
from test_oracle import MARGIN_CULL, fixture_check, same_rsqrt_host
from test_oracle_pair import INTER_MARGIN, pair_env

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def test_pair_fkcc(vamp, oracle):
    fx = host_fixture("pair_scene.npz", oracle)
    oenv = pair_env(oracle, fx)
    got = vamp.panda_pair.fkcc_batch(fx["q"], gpu_env_from_oracle(vamp, oenv))
    assert np.array_equal(got, oracle.pair_fkcc_threads(oenv, fx["q"]))
    m = (fx["test_margin"] > 1e-4) & (fx["inter_margin"] > INTER_MARGIN)
    if not same_rsqrt_host(oracle, fx):
        m &= fx["cull_margin"] > MARGIN_CULL
    fixture_check("panda_pair fkcc (GPU)", got, fx["valid"], m, same_rsqrt_host(oracle, fx))


def test_pair_validate(vamp, oracle):
    fx = host_fixture("pair_scene.npz", oracle)
    oenv = pair_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    ok, n = vamp.panda_pair.validate_batch(fx["starts"], fx["goals"], env)
    rok, rn = oracle.pair_validate_motions(oenv, fx["starts"], fx["goals"])
    assert np.array_equal(n, rn) and np.array_equal(ok, rok)
    # raw long edges across the whole range (many back-steps) and zero-length edges
    rng = np.random.default_rng(5)
    u = rng.random((4000, 14), dtype=F)
    v = rng.random((4000, 14), dtype=F)
    s = np.concatenate([oracle.scale(u[:, :7]), oracle.scale(u[:, 7:])], 1)
    g = np.concatenate([oracle.scale(v[:, :7]), oracle.scale(v[:, 7:])], 1)
    g[:8] = s[:8]
    ok, n = vamp.panda_pair.validate_batch(s, g, env)
    rok, rn = oracle.pair_validate_motions(oenv, s, g)
    assert np.array_equal(n, rn) and np.array_equal(ok, rok)


def test_pair_other_bases(vamp, oracle):
    """arms facing each other at 0.8 m (more inter-arm contact), A lifted 5 cm"""
    rng = np.random.default_rng(9)
    u = rng.random((8192, 14), dtype=F)
    q = np.concatenate([oracle.scale(u[:, :7]), oracle.scale(u[:, 7:])], 1)
    robot = vamp.PandaPair((0, 0, 5), (80, 10, 0))
    oenv = oracle.pair_scene()
    got = robot.fkcc_batch(q, gpu_env_from_oracle(vamp, oenv))
    want = oracle.pair_fkcc_threads(oenv, q, (0, 0, 5), (80, 10, 0))
    assert np.array_equal(got, want)
    va = oracle.fkcc_threads(oenv, q[:, :7], (0, 0, 5)) & oracle.fkcc_threads(oenv, q[:, 7:], (80, 10, 0))
    assert (va & ~want).mean() > 0.01  # inter-arm collisions present
