"""Find self-collision child pairs that cannot fire inside the joint limits.

    python tools/prune_pairs.py model/panda.json          (rewrites the file in place)

For every self check whose two links are separated by at most two revolute joints, the relative
pose of the links depends on those joints only.  Each child pair's centre distance is sampled on
a grid over the joint ranges widened by MARGIN_Q on both sides; a pair is marked unreachable
when the sampled minimum of (distance - r_a - r_b) exceeds

    gap_min = (grid half-step) x (lever arm bound) x (joints) + SAFETY

(between grid points a centre moves less than half-step x its distance to each joint axis;
the bound on that distance is computed per check, ~0.3-0.55 m, so gap_min ~ 0.015-0.021 m).  The FK is evaluated with the
reference's own sin/cos approximations (vector/interface.hh:438-469), in float64; the float32
rounding of the kernels adds ~1e-6 m.
Such a pair's test value sql2 - (ra + rb)^2 is positive for every configuration whose joints lie
within the widened range, so dropping it leaves the check's result unchanged there.  The
generated kernels drop these pairs only for groups whose joints are all inside the range
(`reach_lo`, `reach_hi` below) and evaluate the full list otherwise -- results stay identical
to the reference's for every input.
"""
from __future__ import annotations

import json
import sys

import numpy as np

STEP = 0.02
MARGIN_Q = 0.02
SAFETY = 0.01  # m, beyond the grid-interpolation bound


def vsin(x):
    """FloatVector::sin() (vector/interface.hh:438-456), the approximation the FK actually uses"""
    c1, c2, c3, c4, c5 = -0.478637850138, 1.503684069359, 0.011596870476, 0.140024078368, 0.665200679751
    p = x * (c2 + c1 * np.abs(x))
    ap = np.abs(p)
    return p * (c5 + ap * (c4 + ap * c3))


def vcos(x):
    v = x + np.pi / 2
    return vsin(v - np.where(v >= np.pi, 2 * np.pi, 0.0))


def qmul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.stack([aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx, aw * bz + ax * by - ay * bx + az * bw])


def qmat(q):
    w, x, y, z = q
    return np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)]),
                     np.stack([2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)]),
                     np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)])])


def path(frames, fa, fb):
    out, f = [], fb
    while f != fa:
        if f < 0:
            return None
        out.append(f)
        f = frames[f]["parent"]
    return out[::-1]


def relative_pose(frames, chain, qs, n):
    Q = np.tile(np.array([1.0, 0, 0, 0])[:, None], (1, n))
    P = np.zeros((3, n))
    for f in chain:
        P = P + np.einsum("ijn,j->in", qmat(Q), np.array(frames[f]["t"]))
        A = qmul(Q, np.array(frames[f]["qf"])[:, None] * np.ones((1, n)))
        d = frames[f]["dof"]
        if d >= 0:
            h = qs[d] * 0.5
            A = qmul(A, np.stack([vcos(h), 0 * h, 0 * h, vsin(h)]))
        Q = A
    return qmat(Q), P


def main():
    path_json = sys.argv[1]
    m = json.load(open(path_json))
    frames, spheres = m["frames"], m["spheres"]
    lo = np.array(m["s_a"])
    hi = lo + np.array(m["s_m"])
    m["reach_lo"] = [float(v) for v in lo - MARGIN_Q]
    m["reach_hi"] = [float(v) for v in hi + MARGIN_Q]
    for ck in m["self_checks"]:
        ck.pop("unreachable", None)
        ck.pop("reach_dofs", None)
        pairs = ck["children"]
        fa, fb = spheres[pairs[0][0]]["frame"], spheres[pairs[0][1]]["frame"]
        if any(spheres[a]["frame"] != fa or spheres[b]["frame"] != fb for a, b in pairs):
            continue
        chain = path(frames, fa, fb)
        if chain is None:
            continue
        dofs = [frames[f]["dof"] for f in chain if frames[f]["dof"] >= 0]
        if not 0 < len(dofs) <= 2:
            continue
        grids = [np.arange(lo[d] - MARGIN_Q, hi[d] + MARGIN_Q + STEP, STEP) for d in dofs]
        mesh = np.meshgrid(*grids, indexing="ij")
        qs = {d: g.ravel() for d, g in zip(dofs, mesh)}
        n = mesh[0].size
        R, P = relative_pose(frames, chain, qs, n)
        tsum = sum(np.linalg.norm(frames[f]["t"]) for f in chain)
        cbs = [P + np.einsum("ijn,j->in", R, np.array(spheres[b]["offset"])) for _, b in pairs]
        # every joint axis of the chain passes within sum |t| of frame fa's origin, so a centre is
        # at most |cb| + sum |t| from any of them: between grid points it moves < half-step x that
        lever = max(np.linalg.norm(cb, axis=0).max() for cb in cbs) + tsum
        gap_min = 0.5 * STEP * lever * len(dofs) + SAFETY
        drop = []
        for i, ((a, b), cb) in enumerate(zip(pairs, cbs)):
            ca = np.array(spheres[a]["offset"])[:, None]
            gap = np.linalg.norm(cb - ca, axis=0).min() - (spheres[a]["radius"] + spheres[b]["radius"])
            if gap > gap_min:
                drop.append(i)
        if drop:
            ck["unreachable"] = drop
            ck["reach_dofs"] = dofs
        print(f"{ck['links'][0]} x {ck['links'][1]}: joints {dofs}, {len(drop)} of {len(pairs)} pairs unreachable"
              f" (lever arm <= {lever:.3f} m, required gap {gap_min:.4f} m)")
    json.dump(m, open(path_json, "w"), indent=1)


if __name__ == "__main__":
    main()
