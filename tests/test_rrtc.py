"""BASELINE configs[0]: Panda RRT-Connect on MotionBenchMaker table_pick problems on the CPU rake
(mr-vamp_amd/csrc/cpu/vcpu_rrtc.cpp, planning/rrtc.hh:33-248), RRTCSettings with range 1.0 and 1e6
iterations/samples (src/vamp/constants.py:1,49-55; src/vamp/__init__.py:80-102), Halton<7> reset per
problem (scripts/evaluate_mbm.py:95-96).

Checks: the straight start -> goal validate_motion of each problem equals the reference-DAG fixture;
the product planner equals an independent Python restatement (tests/rrtc_py.py, oracle
validate_vector) path for path, bit for bit, with the same iterations, tree sizes and cost; every
solved path starts at the start, ends at the goal (to the last increment), and each of its segments passes validate_motion
(oracle) or is one of the planner's own validate_vector-checked extensions."""
import numpy as np
import pytest

import rrtc_py
from conftest import host_fixture
from test_gpu_parity import gpu_env_from_oracle
from test_oracle import EDGE_MIN_COVERAGE, MARGIN_TEST, fixture_check, same_rsqrt_host, stable

F = np.float32
SETTINGS = dict(range=1.0, max_iterations=1000000, max_samples=1000000)


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    return vamp_amd


def problem(oracle, fx, k):
    o = oracle.Env()
    for key in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(o, key, [list(r) for r in fx[f"p{k}_env_{key}"]])
    return o, fx[f"p{k}_start"], fx[f"p{k}_goal"]


def test_straight_line_vs_reference_dag(vamp, oracle):
    fx = host_fixture("panda_table_pick_problems.npz", oracle)
    same = same_rsqrt_host(oracle, fx)
    got, ref, keep = [], [], []
    for k in range(1, int(fx["n_problems"]) + 1):
        o, s, g = problem(oracle, fx, k)
        ok, n, _ = vamp.panda_0_0.cpu_validate_batch(s[None], g[None], gpu_env_from_oracle(vamp, o))
        ook, on = oracle.validate_motions(o, s[None], g[None], (0, 0, 0))
        assert ok[0] == ook[0] and n[0] == on[0] == fx[f"p{k}_n"][0]
        got.append(ok[0])
        ref.append(fx[f"p{k}_ok"][0])
        keep.append(stable(fx[f"p{k}_test_margin"], fx[f"p{k}_cull_margin"], same)[0])
    fixture_check("panda table_pick start->goal (CPU rake)", np.array(got), np.array(ref), np.array(keep), same, 0.5)


def test_table_pick_scene_fixture(vamp, oracle):
    """configs[1]'s MBM run: per-configuration masks and edges on
    table_pick scene0001 vs the reference DAG."""
    from test_oracle_robots import scene_env
    fx = host_fixture("panda_table_pick.npz", oracle)
    oenv = scene_env(oracle, fx)
    env = gpu_env_from_oracle(vamp, oenv)
    same = same_rsqrt_host(oracle, fx)
    got = vamp.panda_0_0.cpu_fkcc_batch(fx["q"], env)
    assert np.array_equal(got, oracle.fkcc_threads(oenv, fx["q"], (0, 0, 0)))
    fixture_check("panda fkcc table_pick (CPU rake)", got, fx["valid"], stable(fx["test_margin"], fx["cull_margin"],
                                                                                  same), same)
    ok, n, _ = vamp.panda_0_0.cpu_validate_batch(fx["starts"], fx["goals"], env)
    rok, rn = oracle.validate_motions(oenv, fx["starts"], fx["goals"], (0, 0, 0))
    assert np.array_equal(ok, rok) and np.array_equal(n, rn) and np.array_equal(n, fx["n"])
    fixture_check("panda validate_motion table_pick (CPU rake)", ok, fx["ok"],
                  stable(fx["edge_test_margin"], fx["edge_cull_margin"], same), same, EDGE_MIN_COVERAGE)


@pytest.mark.parametrize("k,base", [(1, (0, 0, 0)), (1, (200, 200, 0)), (2, (0, 0, 0)), (3, (0, 0, 0)),
                                    (4, (0, 0, 0)), (5, (0, 0, 0)), (6, (0, 0, 0))])
def test_rrtc_matches_restatement(vamp, oracle, k, base):
    fx = host_fixture("panda_table_pick_problems.npz", oracle)
    o, s, g = problem(oracle, fx, k)
    env = gpu_env_from_oracle(vamp, o)
    robot = vamp.PandaBase(*base)
    rng = robot.halton()
    res = robot.rrtc(s, g, env, vamp.RRTCSettings(**SETTINGS), rng)
    p, cost, it, sizes, idx = rrtc_py.rrtc("panda", o, s, g, SETTINGS, 1, base)
    assert res.solved and len(p)
    assert res.iterations == it and res.size == sizes and rng.index == idx
    assert np.array_equal(res.path.view(np.uint32), p.view(np.uint32))
    assert np.float32(res.cost).view(np.uint32) == np.float32(cost).view(np.uint32)
    # the ends are the start and goal, or the connect step's last increment onto them (rrtc.hh:213-221
    # walks the other tree from the nearest node's parent)
    assert np.abs(res.path[0] - s).max() <= 1e-5 and np.abs(res.path[-1] - g).max() <= 1e-5
    # segments: collision-free under the planner's own checks (validate_vector with the planner's
    # vector and distance); validate_motion recomputes both from the endpoints, which rakes slightly
    # different interpolants -- so a disagreement is only admissible on a segment that grazes an
    # obstacle.  Counted exactly: every failing segment must have an interpolant within the fixture
    # margin band (MARGIN_TEST) of a contact; on the host the fixtures were made on: exactly 0.
    ok, n = oracle.validate_motions(o, res.path[:-1], res.path[1:], base)
    bad = np.nonzero(~ok.astype(bool))[0]
    for i in bad:
        a, b = res.path[i].astype(np.float64), res.path[i + 1].astype(np.float64)
        t = np.arange(1, 8 * int(n[i]) + 1) / (8.0 * int(n[i]))
        q = (a[None] + (b - a)[None] * t[:, None]).astype(F)
        _, tm, _, _ = oracle.fkcc(o, q, base, stats=True)
        assert np.abs(tm).min() <= MARGIN_TEST, f"segment {i} invalid far from any contact: {np.abs(tm).min()}"
    if same_rsqrt_host(oracle, fx):
        assert len(bad) == 0, f"{len(bad)} near-boundary segment disagreements: {bad}"


def test_rrtc_rng_and_settings(vamp, oracle):
    """a second solve continues the sampler (evaluate_mbm runs trials without reset); max_iterations
    bounds the search; an unsolvable problem reports solved = False."""
    fx = host_fixture("panda_table_pick_problems.npz", oracle)
    o, s, g = problem(oracle, fx, 2)
    env = gpu_env_from_oracle(vamp, o)
    robot = vamp.panda_0_0
    rng = robot.halton()
    r1 = robot.rrtc(s, g, env, vamp.RRTCSettings(**SETTINGS), rng)
    i1 = rng.index
    r2 = robot.rrtc(s, g, env, vamp.RRTCSettings(**SETTINGS), rng)
    p, _, it, _, idx = rrtc_py.rrtc("panda", o, s, g, SETTINGS, i1)
    assert r2.iterations == it and rng.index == idx and np.array_equal(r2.path, p)
    assert r1.solved and r2.solved
    capped = robot.rrtc(s, g, env, vamp.RRTCSettings(range=1.0, max_iterations=3, max_samples=1000), robot.halton())
    assert capped.iterations <= 4
    # the goal inside an obstacle: no path within the iteration budget
    blocked = vamp.Environment()
    blocked.add_sphere(vamp.Sphere([0.0, 0.0, 0.4], 0.6))
    r = robot.rrtc(s, g, blocked, vamp.RRTCSettings(range=1.0, max_iterations=200, max_samples=1000), robot.halton())
    assert not r.solved and r.path.shape == (0, 7) and r.iterations == 201


# ---- BASELINE configs[4]'s planner half: RRT-Connect on the two-Panda composite -------------------------------
PAIR_BASES = ((0, 0, 0), (100, 0, 0))  # vamp_amd.panda_pair: arm A at the origin, arm B 1 m along x


def pair_problems(oracle, n, seed=41):
    """configs[4]'s scene (oracle_py.pair_scene: a table under both arms, three spheres between them) and n
    start/goal composite configurations, collision-free, whose straight validate_motion FAILS (so the planner
    has to search), from seeded uniform draws -- no reference counterpart (SURVEY §0 finding 10): the anchor is
    rrtc.hh:33-248 over the composed validity"""
    o = oracle.pair_scene()
    rng = np.random.default_rng(seed)
    q = oracle.pair_scale(rng.random((40 * n, 14), dtype=F))
    q = q[oracle.pair_fkcc_threads(o, q, *PAIR_BASES)]
    s, g = q[0::2][:8 * n], q[1::2][:8 * n]
    m = min(len(s), len(g))
    ok, _ = oracle.pair_validate_motions(o, s[:m], g[:m], *PAIR_BASES)
    hard = np.nonzero(~ok.astype(bool))[0][:n]
    assert len(hard) == n
    return o, s[hard], g[hard]


@pytest.mark.parametrize("k", range(6))
def test_pair_rrtc_matches_restatement(vamp, oracle, k):
    """vamp_amd.panda_pair.rrtc == the Python restatement over the oracle's composite validate_vector
    (oracle vo_pair_validate_vector), Halton<14> and the two-register l2_norm: path bit for bit, cost,
    iterations, tree sizes, sampler index; every segment of the path passes the oracle's validate_motion."""
    o, S, G = pair_problems(oracle, 6)
    env = gpu_env_from_oracle(vamp, o)
    robot = vamp.panda_pair
    rng = robot.halton()
    res = robot.rrtc(S[k], G[k], env, vamp.RRTCSettings(**SETTINGS), rng)
    p, cost, it, sizes, idx = rrtc_py.rrtc("pair", o, S[k], G[k], SETTINGS, 1, PAIR_BASES)
    assert res.solved and len(p) > 2
    assert res.iterations == it and res.size == sizes and rng.index == idx
    assert np.array_equal(res.path.view(np.uint32), p.view(np.uint32))
    assert np.float32(res.cost).view(np.uint32) == np.float32(cost).view(np.uint32)
    ok, _ = oracle.pair_validate_motions(o, res.path[:-1], res.path[1:], *PAIR_BASES)
    assert ok.all(), np.nonzero(~ok.astype(bool))[0]
