"""Chained staged passes (vgpu_api.cpp chain_pass): the two-Panda composite (arm A, arm B and two chunks
of inter-arm checks, vgpu_pair_staged.hip) and the Baxter (388 checks in 7 chunks, vgpu_baxter_staged.hip)
run as several staged passes ANDed into one flag.  Their results equal the monolithic kernels' (a second
context created with VAMP_AMD_STAGED=0) and the oracle's, for per-configuration masks and validate_motion,
including the gated wrist checks of the Panda arms (model/panda_pair_gate.json)."""
import os

import numpy as np
import pytest

from test_gpu_parity import gpu_env_from_oracle, random_scene

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def ctxs():
    import vamp_amd
    staged = vamp_amd.context(0)
    os.environ["VAMP_AMD_STAGED"] = "0"
    try:
        mono = vamp_amd.Context(0)  # reads VAMP_AMD_STAGED at creation
    finally:
        del os.environ["VAMP_AMD_STAGED"]
    return vamp_amd, staged, mono


def test_pair_staged_equals_monolithic_and_oracle(ctxs, oracle):
    vamp, staged, mono = ctxs
    oenv = oracle.pair_scene()
    rng = np.random.default_rng(41)
    u = rng.random((30000, 14), dtype=F)
    q = np.concatenate([oracle.scale(u[:, :7]), oracle.scale(u[:, 7:])], 1)
    for robot, ba, bb in ((vamp.panda_pair, (0, 0, 0), (100, 0, 0)), (vamp.PandaPair((0, 0, 5), (80, 10, 0)),
                                                                       (0, 0, 5), (80, 10, 0))):
        env = gpu_env_from_oracle(vamp, oenv)
        a = robot.fkcc_batch(q, env, staged)
        b = robot.fkcc_batch(q, env, mono)
        assert np.array_equal(a, b)
        assert np.array_equal(a[:8192], oracle.pair_fkcc_threads(oenv, q[:8192], ba, bb))
        s, g = q[:5000], q[5000:10000].copy()
        g[:2500] = s[:2500] + (g[:2500] - s[:2500]) * F(0.15)
        oka, na = robot.validate_batch(s, g, env, staged)
        okb, nb = robot.validate_batch(s, g, env, mono)
        assert np.array_equal(na, nb) and np.array_equal(oka, okb)
        ro, rn = oracle.pair_validate_motions(oenv, s, g, ba, bb)
        assert np.array_equal(oka, ro) and np.array_equal(na, rn)
        assert 0.02 < oka.mean() < 0.98


def test_baxter_staged_equals_monolithic_and_oracle(ctxs, oracle):
    vamp, staged, mono = ctxs
    rng = np.random.default_rng(42)
    oenv = random_scene(oracle, rng, 4, 4, 3)
    env = gpu_env_from_oracle(vamp, oenv)
    q = oracle.robot_scale("baxter", rng.random((20000, 14), dtype=F))
    a = vamp.baxter.fkcc_batch(q, env, staged)
    assert np.array_equal(a, vamp.baxter.fkcc_batch(q, env, mono))
    assert np.array_equal(a[:4096], oracle.robot_fkcc_threads("baxter", oenv, q[:4096]))
    s, g = q[:3000], q[3000:6000].copy()
    g[:1500] = s[:1500] + (g[:1500] - s[:1500]) * F(0.1)
    oka, na = vamp.baxter.validate_batch(s, g, env, staged)
    okb, nb = vamp.baxter.validate_batch(s, g, env, mono)
    assert np.array_equal(na, nb) and np.array_equal(oka, okb)
    ro, rn = oracle.robot_validate_motions("baxter", oenv, s, g)
    assert np.array_equal(oka, ro) and np.array_equal(na, rn)
    # the PRM sampling stage of the Baxter (chained samples source)
    qs, vs = vamp.baxter.sample_fkcc(1, 20000, env, staged)
    qm, vm = vamp.baxter.sample_fkcc(1, 20000, env, mono)
    assert np.array_equal(qs.view(np.uint32), qm.view(np.uint32)) and np.array_equal(vs, vm)


def test_panda_gate_exact_on_wrist_contacts(ctxs, oracle):
    """Configurations sampled where the wrist checks (15, 21, 26, 30) fire or graze: the gated bound stage
    keeps every one of them (staged == monolithic == oracle)."""
    vamp, staged, mono = ctxs
    rng = np.random.default_rng(43)
    q = oracle.scale(rng.random((400000, 7), dtype=F))
    empty = oracle.Env()
    v = oracle.fkcc_threads(empty, q)  # self-collision only
    q = np.concatenate([q[~v][:20000], q[v][:20000]])
    env = vamp.Environment()
    for robot, base in ((vamp.panda_0_0, (0, 0, 0)), (vamp.panda, (200, 200, 0))):
        a = robot.fkcc_batch(q, env, staged)
        assert np.array_equal(a, robot.fkcc_batch(q, env, mono))
        assert np.array_equal(a, oracle.fkcc_threads(empty, q, base))
