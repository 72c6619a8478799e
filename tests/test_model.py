"""The kernel model (model/panda.json): the unreachable self-collision pairs that the generated
kernels skip inside the analysed joint range (tools/prune_pairs.py) must never come close on the
oracle's FK -- a dense random check complementing the analysis's grid + Lipschitz bound."""
import json
import os

import numpy as np

from conftest import ROOT

F = np.float32


def test_unreachable_pairs_never_fire(oracle):
    m = json.load(open(os.path.join(ROOT, "model", "panda.json")))
    lo, hi = np.array(m["reach_lo"], F), np.array(m["reach_hi"], F)
    rng = np.random.default_rng(11)
    n = 40000
    q = (lo + rng.random((n, 7), dtype=F) * (hi - lo)).astype(F)
    q[:64] = np.where(rng.random((64, 7)) < 0.5, lo, hi)  # corners of the range
    xyz = oracle.sphere_fk(q)  # [n, 59, 3]
    r = np.array([s["radius"] for s in m["spheres"]])
    checked = 0
    for ck in m["self_checks"]:
        for i in ck.get("unreachable", []):
            a, b = ck["children"][i]
            d = np.linalg.norm(xyz[:, a].astype(np.float64) - xyz[:, b], axis=1) - (r[a] + r[b])
            assert d.min() > 0.005, (ck["links"], a, b, d.min())
            checked += 1
    assert checked >= 200


def test_reach_range_covers_joint_limits():
    m = json.load(open(os.path.join(ROOT, "model", "panda.json")))
    lo = np.array(m["s_a"])
    hi = lo + np.array(m["s_m"])
    assert (np.array(m["reach_lo"]) < lo).all() and (np.array(m["reach_hi"]) > hi).all()
