"""Conservative (q5, q6) gate table for the Panda's wrist self checks (model/panda_pair_gate.json).

Checks 15 (link5 x link7), 21 (link5 x hand), 26 and 30 (link5 x fingers) of panda/fk.hh depend on joints 6
and 7 only (q5, q6: reach_dofs [5, 6] in model/panda.json): link5's spheres are fixed in link5's frame and
the other link's spheres move with the two wrist joints.  Their bounding spheres overlap for ~every
configuration, so the staged pipeline queued them for ~every group although a child pair fires only in a
small part of the (q5, q6) square.

Over the reach range (joint limits +- 0.02, the range tools/prune_pairs.py analysed) the square is split into
N5 x N6 cells; a cell's bit k is CLEAR only when no child pair of check k can fire anywhere in the cell:
every pair's centre distance, sampled on an S x S sub-grid of the cell (float32 FK of the oracle, other
joints 0 -- the pair distance does not depend on them), stays above r_i + r_j + slack + MARGIN, where
slack = L5 * h5 / 2 + L6 * h6 / 2 bounds the distance change between a point of the cell and its nearest
sample (L = the moving sphere's largest distance from the joint-6 / joint-7 origin, an upper bound of its
lever arm) and MARGIN = 1 mm covers float32 FK rounding (~1e-6 m) and the approximate sin/cos (~2e-5 rad).
The bound stage then sets check k's bit only when the bounding test fires AND some lane's cell allows it
(lanes outside the table: always allowed) -- a check that cannot fire is never queued, results unchanged.

    python tools/make_pair_gate.py        (needs oracle/_build/libvamp_oracle.so)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as op  # noqa: E402

N5, N6, S = 128, 128, 4
MARGIN = 1e-3
CHECKS = [15, 21, 26, 30]


def main():
    op.build()
    m = json.load(open(os.path.join(ROOT, "model", "panda.json")))
    lo, hi = m["reach_lo"], m["reach_hi"]
    order = m["check_order"]
    pairs = {}
    for c in CHECKS:
        o = order[c]
        assert o["kind"] == "self"
        ck = m["self_checks"][o["index"]]
        assert ck.get("reach_dofs") == [5, 6], (c, ck.get("reach_dofs"))
        pairs[c] = np.array(ck["children"], np.int64)
    radii = np.array([s["radius"] for s in m["spheres"]], np.float64)
    h5 = (hi[5] - lo[5]) / N5
    h6 = (hi[6] - lo[6]) / N6
    q5s = lo[5] + (np.arange(N5 * S) + 0.5) * (h5 / S)
    q6s = lo[6] + (np.arange(N6 * S) + 0.5) * (h6 / S)
    Q = np.zeros((len(q5s) * len(q6s), 7), np.float32)
    Q[:, 5] = np.repeat(q5s, len(q6s))
    Q[:, 6] = np.tile(q6s, len(q5s))
    C = op.sphere_fk(Q, (0, 0, 0)).astype(np.float64)  # [n][59][3]
    # joint origins: joint 6 at link6's origin (= link5's), joint 7 at link7's (model frames 6, 7)
    o6 = frame_origin(m, Q, 6)
    o7 = frame_origin(m, Q, 7)
    gate = np.zeros((N5, N6), np.uint8)
    stats = {}
    for bit, c in enumerate(CHECKS):
        p = pairs[c]
        d = np.linalg.norm(C[:, p[:, 0]] - C[:, p[:, 1]], axis=2)  # [n][pairs]
        # lever arms of the moving spheres (the second of each pair: link7/hand/finger)
        mv = np.unique(p[:, 1])
        L5 = np.linalg.norm(C[:, mv] - o6[:, None], axis=2).max(0)
        L6 = np.linalg.norm(C[:, mv] - o7[:, None], axis=2).max(0)
        Lmap = dict(zip(mv.tolist(), zip(L5.tolist(), L6.tolist())))
        slack = np.array([Lmap[j][0] * h5 / (2 * S) + Lmap[j][1] * h6 / (2 * S) for j in p[:, 1]]) * 1.25
        free = d - (radii[p[:, 0]] + radii[p[:, 1]]) - slack - MARGIN  # > 0: provably no contact
        free = free.reshape(N5, S, N6, S, -1).min(axis=(1, 3, 4))     # over the cell's samples and pairs
        allowed = free <= 0.0
        gate |= (allowed.astype(np.uint8) << bit)
        stats[c] = float(allowed.mean())
    out = {"checks": CHECKS, "dofs": [5, 6], "lo": [lo[5], lo[6]], "h": [h5, h6], "n": [N5, N6], "sub": S,
           "margin": MARGIN, "allowed_fraction": stats,
           "gate": gate.ravel().tolist()}
    verify(m, pairs, radii, gate, lo, h5, h6)
    path = os.path.join(ROOT, "model", "panda_pair_gate.json")
    json.dump(out, open(path, "w"))
    print("wrote", path, "allowed fraction per check:", stats)


def verify(m, pairs, radii, gate, lo, h5, h6, n=200000):
    """Independent check: random configurations (all joints uniform in the limits), the oracle's float32
    FK, every child pair's exact test value; a pair that fires must lie in a cell whose bit is set."""
    rng = np.random.default_rng(1)
    q = op.scale(rng.random((n, 7), dtype=np.float32))
    C = op.sphere_fk(q, (0, 0, 0)).astype(np.float32)
    i5 = np.floor((q[:, 5].astype(np.float64) - lo[5]) / h5).astype(np.int64)
    i6 = np.floor((q[:, 6].astype(np.float64) - lo[6]) / h6).astype(np.int64)
    assert (i5 >= 0).all() and (i5 < N5).all() and (i6 >= 0).all() and (i6 < N6).all()
    fired_total = 0
    for bit, c in enumerate(CHECKS):
        p = pairs[c]
        d = C[:, p[:, 0]] - C[:, p[:, 1]]
        v = (d * d).sum(2) - (radii[p[:, 0]] + radii[p[:, 1]]).astype(np.float32) ** 2
        fired = (v < 1e-4).any(1)  # fires, or within the fixtures' near-boundary band
        fired_total += int(fired.sum())
        ok = ((gate[i5, i6] >> bit) & 1).astype(bool)
        bad = int((fired & ~ok).sum())
        assert bad == 0, (c, bad)
    print(f"verify: {n} random configurations, {fired_total} near/firing check instances, all inside allowed cells")


def frame_origin(m, Q, f):
    """world origin of model frame f at each configuration (float64 FK restated from the model;
    only used for lever-arm bounds, which take a 25 % safety factor)."""
    frames = m["frames"]
    n = Q.shape[0]
    R = np.tile(np.eye(3), (n, 1, 1))
    P = np.zeros((n, 3))
    chain = []
    k = f
    while k >= 0:
        chain.append(k)
        k = frames[k]["parent"]
    for k in reversed(chain):
        fr = frames[k]
        if fr["parent"] < 0:
            P = np.tile(np.array(fr["t"], np.float64), (n, 1))
            R = np.tile(quat_mat(fr["qf"]), (n, 1, 1))
            continue
        P = P + np.einsum("nij,j->ni", R, np.array(fr["t"], np.float64))
        R = R @ quat_mat(fr["qf"])
        if fr["dof"] >= 0:
            a = Q[:, fr["dof"]].astype(np.float64)
            c, s = np.cos(a), np.sin(a)
            Rz = np.zeros((n, 3, 3))
            Rz[:, 0, 0], Rz[:, 0, 1], Rz[:, 1, 0], Rz[:, 1, 1], Rz[:, 2, 2] = c, -s, s, c, 1
            R = R @ Rz
    return P


def quat_mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


if __name__ == "__main__":
    main()
