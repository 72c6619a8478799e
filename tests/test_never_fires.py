"""Self checks proven silent inside the joint limits (tools/prove_self_checks.py; CPU tests).

The Fetch's self checks 7, 9, 10, 11 and 12 (torso / shoulder links against the upper-arm links) have child
sphere pairs that cannot touch anywhere inside the joint limits widened by a margin: the branch-and-bound
proof of tools/prove_self_checks.py bounds every pair's gap from below over boxes of the joints between the
two links.  The generated staged bound stage (tools/gen_kernels.py) then leaves those checks' bits clear
for groups whose lanes all lie in the proven box (the reference's check reports nothing there), and
evaluates them as before for any other group.  Here: the proof is re-run for the quick checks, the recorded
checks never fire on an independent random sample (the oracle's float32 FK), and the generated code guards
exactly the recorded checks."""
import json
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

F = np.float32


def model():
    return json.load(open(os.path.join(ROOT, "model", "fetch.json")))


def never(m):
    return [(c, m["self_checks"][o["index"]]) for c, o in enumerate(m["check_order"])
            if o["kind"] == "self" and m["self_checks"][o["index"]].get("never_fires")]


def test_recorded_checks():
    m = model()
    assert [c for c, _ in never(m)] == [7, 9, 10, 11, 12]
    for c, ck in never(m):
        d = ck["never_dofs"]
        assert len(d) == len(ck["never_lo"]) == len(ck["never_hi"]) > 0
        for k, lo, hi in zip(d, ck["never_lo"], ck["never_hi"]):  # the box contains the joint limits
            assert lo < m["s_a"][k] and hi > m["s_a"][k] + m["s_m"][k]


@pytest.mark.parametrize("check", [7, 9])
def test_proof_reproduces(check):
    import prove_self_checks as P
    m = model()
    ck = m["self_checks"][m["check_order"][check]["index"]]
    mq = ck["never_lo"][0] - m["s_a"][ck["never_dofs"][0]]
    ok, dofs, _ = P.prove(m, ck, -mq)
    assert ok and dofs == ck["never_dofs"]


def test_proof_rejects_a_check_that_fires():
    """check 8 (head pan vs upper-arm roll) fires for ~2 % of random configurations: not provable"""
    import prove_self_checks as P
    m = model()
    ok, _, _ = P.prove(m, m["self_checks"][m["check_order"][8]["index"]], max_iter=30)
    assert not ok


def test_recorded_checks_never_fire_on_a_sample(oracle):
    """uniform configurations inside the proven boxes (the other joints anywhere in their limits), including
    the boxes' faces: no child pair of a recorded check overlaps (float32 FK of the oracle)"""
    m = model()
    rng = np.random.default_rng(11)
    n = 60000
    rad = np.array([s["radius"] for s in m["spheres"]], F)
    for c, ck in never(m):
        q = oracle.robot_scale("fetch", rng.random((n, 8), dtype=F))
        for k, lo, hi in zip(ck["never_dofs"], ck["never_lo"], ck["never_hi"]):
            u = rng.random(n)
            u[: n // 10] = rng.integers(0, 2, n // 10)  # a tenth on the box faces
            q[:, k] = (lo + u * (hi - lo)).astype(F)
        C = oracle.robot_sphere_fk("fetch", q)
        p = np.array(ck["children"])
        d = C[:, p[:, 0]] - C[:, p[:, 1]]
        v = (d * d).sum(2) - (rad[p[:, 0]] + rad[p[:, 1]]) ** 2
        assert (v > 0).all(), (c, float(v.min()))


def test_generated_guards_match_the_model():
    m = model()
    inc = open(os.path.join(ROOT, "mr-vamp_amd", "csrc", "gen", "fetch_fk.inc")).read()
    # one guarded line per check (the 8-lane groups' per-lane form: tools/gen_kernels.py LANE_BITS)
    guarded = sorted(int(x) for x in re.findall(r"<< (\d+);(?: \})?  // proven silent inside", inc))
    assert guarded == [c for c, _ in never(m)]


def test_lever_counts_later_prismatic_travel():
    """a revolute joint's lever includes the travel of every prismatic joint after it in the chain (a
    point pushed out along a slide moves farther per radian); a prismatic joint itself moves the point 1:1"""
    import prove_self_checks as P
    frames = [{"dof": 0, "jtype": "revolute", "t": [0.0, 0.0, 0.0], "axis": [0, 0, 1]},
              {"dof": 1, "jtype": "prismatic", "t": [0.5, 0.0, 0.0], "axis": [1, 0, 0]},
              {"dof": -1, "t": [0.0, 0.2, 0.0]}]
    reach = np.array([3.0, 0.4])
    lev = P.levers(frames, [0, 1, 2], [0.0, 0.0, 0.1], reach)
    assert lev[1] == 1.0
    assert abs(lev[0] - (0.5 + 0.2 + 0.1 + 0.4)) < 1e-12
