"""The two-Panda composite (BASELINE configs[4]) and the multi-register
l2_norm it needs.

There is no composite robot in the reference (SURVEY §0 finding 10).  The C restatement
(vo_pair_*) composes reference primitives: fkcc of each arm at its base and a bounding-first
inter-arm sphere test.  It is checked here against an independent composition built from the
reference DAG (tools/make_golden.py --pair: interleaved_sphere_fk of each arm + the flat 59 x 59
sphere_sphere test on the DAG's sphere_fk centres).  The two agree except where the hierarchy
matters: a child pair may overlap while its link-bounding pair does not (the generated bounding
spheres under-cover their links by up to 0.6 mm), so the margin filter here is 1e-3 m^2.
"""
import numpy as np

from conftest import golden, host_fixture
from test_oracle import same_rsqrt_host

INTER_MARGIN = 1e-3


def test_l2_norm_pins(oracle):
    """FloatVector<7|8|14>::l2_norm bit-exact against the compiled reference vector layer."""
    p = golden("ref_pins_l2.npz")
    for dim in (7, 8, 14):
        v = p[f"v{dim}"]
        got = np.array([oracle.lib().vo_l2_norm(oracle.fp(np.ascontiguousarray(r)), dim) for r in v], np.float32)
        assert np.array_equal(got.view(np.uint32), p[f"d{dim}"].view(np.uint32)), dim


def pair_env(oracle, fx):
    e = oracle.Env()
    for k in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(e, k, [list(r) for r in fx["env_" + k]])
    return e


def test_pair_scene_rows(oracle):
    fx = host_fixture("pair_scene.npz", oracle)
    a = oracle.pair_scene().arrays()
    for k in ("spheres", "zcuboids"):
        assert np.array_equal(a[k], fx["env_" + k])


def test_pair_fkcc_vs_dag_composition(oracle):
    fx = host_fixture("pair_scene.npz", oracle)
    env = pair_env(oracle, fx)
    got = oracle.pair_fkcc_threads(env, fx["q"])
    m = (fx["test_margin"] > 1e-4) & (fx["inter_margin"] > INTER_MARGIN)
    if not same_rsqrt_host(oracle, fx):
        m &= fx["cull_margin"] > 2e-3
    assert m.mean() > 0.8
    assert np.array_equal(got[m], fx["valid"][m])
    assert int((got != fx["valid"]).sum()) <= max(2, int(1e-3 * len(got)))
    # the composition's parts: each arm alone equals the single-arm oracle
    va = oracle.fkcc_threads(env, fx["q"][:, :7], (0, 0, 0))
    vb = oracle.fkcc_threads(env, fx["q"][:, 7:], (100, 0, 0))
    assert (got <= (va & vb)).all()
    assert np.array_equal(va[m], fx["valid_a"][m]) and np.array_equal(vb[m], fx["valid_b"][m])
    assert fx["inter_hit"].mean() > 0.005  # the scene exercises the inter-arm test


def test_pair_validate_vs_dag_composition(oracle):
    fx = host_fixture("pair_scene.npz", oracle)
    env = pair_env(oracle, fx)
    ok, n = oracle.pair_validate_motions(env, fx["starts"], fx["goals"])
    assert np.array_equal(n, fx["n"])
    m = (fx["edge_test_margin"] > 1e-4) & (fx["edge_inter_margin"] > INTER_MARGIN)
    assert np.array_equal(ok[m], fx["ok"][m])
    assert int((ok != fx["ok"]).sum()) <= 2
