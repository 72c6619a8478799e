"""Prove self checks that cannot fire anywhere inside the joint limits (branch and bound).

    python tools/prove_self_checks.py model/fetch.json [--checks 7,9,10,11,12] [--write]

A self check of the staged pipeline (vgpu_staged.hh) is a link-bounding test plus child sphere pairs; the
reference reports a collision only when a child pair overlaps.  For a check whose two links are joined
through joints J (the joints between their common ancestor frame and each link), every child pair's centre
distance depends on q_J only.  Over the box of q_J (joint limits widened by MARGIN_Q), this tool splits the
box until, in every sub-box B, the pair gaps at B's centre exceed the most they can shrink inside B:

    gap_ij(centre) - 1.05 * sum_j lever_ij,j * halfwidth_j  >  MARGIN          for every child pair ij,

lever_ij,j bounding how far a child sphere centre moves per unit of joint j (revolute: its distance from
joint j's origin, bounded by the link offsets down the chain plus the sphere's offset -- a point at
distance L from the axis moves at most L * |dq|; prismatic: 1 per metre), summed over the two spheres'
joints.  The FK is the reference's (quaternion chain with FloatVector::sin/cos, vector/interface.hh:438-469)
in float64; the 1.05 factor covers the approximate sin/cos's derivative and non-unit quaternions (both
< 1e-3 relative), MARGIN = 1 mm the float32 rounding of the kernels (~1e-6 m).  A proven check's test value
sql2 - (ra + rb)^2 is positive for every child pair and every configuration in the widened box, so the
reference's check reports nothing there: the generated staged bound stage (tools/gen_kernels.py) leaves
the check's bit clear for groups whose lanes all lie inside the box, and evaluates it as before
otherwise -- results identical to the reference's for every input.

--write records the proven checks in the model: self_checks[k]["never_fires"] = True with "never_dofs" = J
and the proven box "never_lo" / "never_hi" (the joint limits -+ MARGIN_Q, or -+ MARGIN_Q_TIGHT for a check
whose children come within ~1 mm of contact just outside the limits).  A random
sample of configurations is checked independently afterwards (no proven check may fire).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

MARGIN_Q = 0.02
MARGIN_Q_TIGHT = 0.002  # rad / m: still far above the rounding of in-limit samples and rake interpolants
MARGIN = 1e-3
LIP = 1.05
MIN_HALF = 1e-5  # a box this small that is still undecided: the check may fire (not proven)


def vsin(x):
    """FloatVector::sin() (vector/interface.hh:438-456) -- vgpu_device.hh vamp_sin, in float64"""
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


def ancestors(frames, f):
    out = []
    while f >= 0:
        out.append(f)
        f = frames[f]["parent"]
    return out


def paths(frames, fa, fb):
    """(common ancestor, frames strictly below it down to fa, likewise to fb), root-first"""
    aa, ab = ancestors(frames, fa), ancestors(frames, fb)
    anc = next(f for f in aa if f in ab)
    return anc, aa[:aa.index(anc)][::-1], ab[:ab.index(anc)][::-1]


def chain_fk(frames, chain, q):
    """poses (R [3,3,n], P [3,n]) of each frame of `chain` relative to the chain's parent, for q [n, dim]"""
    n = q.shape[0]
    Q = np.tile(np.array([1.0, 0, 0, 0])[:, None], (1, n))
    P = np.zeros((3, n))
    out = {}
    for f in chain:
        fr = frames[f]
        P = P + np.einsum("ijn,j->in", qmat(Q), np.array(fr["t"], np.float64))
        A = qmul(Q, np.array(fr["qf"], np.float64)[:, None] * np.ones((1, n)))
        d = fr["dof"]
        ax = np.array(fr.get("axis") or [0.0, 0.0, 1.0], np.float64)
        if d >= 0 and fr.get("jtype") == "prismatic":
            P = P + np.einsum("ijn,j->in", qmat(A), ax) * q[:, d][None, :]
            Q = A
        elif d >= 0:
            h = q[:, d] * 0.5
            s = vsin(h)
            Q = qmul(A, np.stack([vcos(h), s * ax[0], s * ax[1], s * ax[2]]))
        else:
            Q = A
        out[f] = (qmat(Q), P.copy())
    return out


def levers(frames, chain, offset, reach):
    """{dof: movement bound per unit of that joint} for a point at `offset` in the last frame of chain.  A revolute
    joint's lever is the point's largest distance from its axis: the fixed translations of the later frames, the
    offset, and the travel of every LATER prismatic joint (reach[dof] = max |q| over the widened limits) -- without
    that travel the bound is unsound for a chain with a prismatic joint after a revolute one"""
    lev = {}
    for i, f in enumerate(chain):
        fr = frames[f]
        if fr["dof"] < 0:
            continue
        if fr.get("jtype") == "prismatic":
            lev[fr["dof"]] = 1.0
        else:
            travel = sum(reach[frames[g]["dof"]] for g in chain[i + 1:]
                         if frames[g]["dof"] >= 0 and frames[g].get("jtype") == "prismatic")
            lev[fr["dof"]] = sum(np.linalg.norm(frames[g]["t"]) for g in chain[i + 1:]) + np.linalg.norm(offset) + \
                travel
    return lev


def prove(m, ck, margin_q=MARGIN_Q, max_iter=60, verbose=False):
    """(proven, dofs, boxes evaluated) for one self check over the joint limits widened by margin_q"""
    frames, spheres = m["frames"], m["spheres"]
    pairs = ck["children"]
    fa = {spheres[a]["frame"] for a, _ in pairs}
    fb = {spheres[b]["frame"] for _, b in pairs}
    if len(fa) != 1 or len(fb) != 1:
        return False, [], 0
    fa, fb = fa.pop(), fb.pop()
    anc, pa, pb = paths(frames, fa, fb)
    dofs = sorted({frames[f]["dof"] for f in pa + pb if frames[f]["dof"] >= 0})
    if not dofs:
        return False, [], 0
    lo0 = np.array(m["s_a"], np.float64) - margin_q
    hi0 = lo0 + np.array(m["s_m"], np.float64) + 2 * margin_q
    dim = m["dimension"]
    ia = np.array([a for a, _ in pairs])
    ib = np.array([b for _, b in pairs])
    rr = np.array([spheres[a]["radius"] + spheres[b]["radius"] for a, b in pairs])
    # per pair and dof: the joint's movement bound for the two spheres
    L = np.zeros((len(pairs), len(dofs)))
    for k, (a, b) in enumerate(pairs):
        reach = np.maximum(np.abs(lo0), np.abs(hi0))
        la = levers(frames, pa, spheres[a]["offset"], reach)
        lb = levers(frames, pb, spheres[b]["offset"], reach)
        for di, d in enumerate(dofs):
            L[k, di] = la.get(d, 0.0) + lb.get(d, 0.0)
    lo = lo0[dofs][None, :].copy()
    hi = hi0[dofs][None, :].copy()
    evaluated = 0
    for it in range(max_iter):
        if len(lo) == 0:
            return True, dofs, evaluated
        c = (lo + hi) / 2
        hw = (hi - lo) / 2
        q = np.zeros((len(c), dim))
        q[:, dofs] = c
        ra, rb = chain_fk(frames, pa, q), chain_fk(frames, pb, q)
        Ra, Pa = ra[fa] if pa else (np.tile(np.eye(3)[:, :, None], (1, 1, len(c))), np.zeros((3, len(c))))
        Rb, Pb = rb[fb] if pb else (np.tile(np.eye(3)[:, :, None], (1, 1, len(c))), np.zeros((3, len(c))))
        oa = np.array([spheres[a]["offset"] for a in ia], np.float64)  # [pairs, 3]
        ob = np.array([spheres[b]["offset"] for b in ib], np.float64)
        ca = Pa[None] + np.einsum("ijn,pj->pin", Ra, oa)  # [pairs, 3, n]
        cb = Pb[None] + np.einsum("ijn,pj->pin", Rb, ob)
        gap = np.linalg.norm(ca - cb, axis=1) - rr[:, None]  # [pairs, n]
        slack = LIP * (L @ hw.T)  # [pairs, n]
        evaluated += len(c)
        if (gap < -1e-9).any():
            return False, dofs, evaluated  # a child pair overlaps at a box centre: the check can fire
        free = ((gap - slack) > MARGIN).all(0)
        keep = ~free
        lo, hi, hw = lo[keep], hi[keep], hw[keep]
        if verbose:
            print(f"  iter {it}: {len(c)} boxes, {int(free.sum())} proven, {int(keep.sum())} split")
        if len(lo) == 0:
            return True, dofs, evaluated
        if (hw.max(1) < MIN_HALF).any():
            return False, dofs, evaluated
        if len(lo) > 4_000_000:
            return False, dofs, evaluated
        # split each box in two along the dof that dominates its slack
        contrib = L.max(0)[None, :] * hw
        ax = contrib.argmax(1)
        mid = (lo[np.arange(len(lo)), ax] + hi[np.arange(len(lo)), ax]) / 2
        lo2, hi2 = lo.copy(), hi.copy()
        hi[np.arange(len(lo)), ax] = mid
        lo2[np.arange(len(lo)), ax] = mid
        lo, hi = np.concatenate([lo, lo2]), np.concatenate([hi, hi2])
    return False, dofs, evaluated


def verify(m, checks, n=400000, seed=3):
    """independent sample: uniform configurations inside the joint limits, the float32 oracle's sphere FK;
    no child pair of a proven check may overlap"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tests"))
    import oracle_py as op
    op.build()
    robot = m["robot"]
    rng = np.random.default_rng(seed)
    q = op.robot_scale(robot, rng.random((n, m["dimension"]), dtype=np.float32))
    C = op.robot_sphere_fk(robot, q).astype(np.float32)
    rad = np.array([s["radius"] for s in m["spheres"]], np.float32)
    worst = {}
    for c in checks:
        ck = m["self_checks"][m["check_order"][c]["index"]]
        p = np.array(ck["children"])
        d = C[:, p[:, 0]] - C[:, p[:, 1]]
        v = (d * d).sum(2) - (rad[p[:, 0]] + rad[p[:, 1]]) ** 2
        assert not (v < 0).any(), f"check {c} fires on a sampled configuration"
        worst[c] = float(np.sqrt((d * d).sum(2)).min() if len(p) else 0)
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("--checks", default=None, help="comma-separated check indices (default: every self check)")
    ap.add_argument("--write", action="store_true")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    m = json.load(open(a.model))
    order = m["check_order"]
    cand = [int(x) for x in a.checks.split(",")] if a.checks else [c for c, o in enumerate(order) if o["kind"] == "self"]
    proven = []
    for c in cand:
        o = order[c]
        if o["kind"] != "self":
            continue
        ck = m["self_checks"][o["index"]]
        for mq in (MARGIN_Q, MARGIN_Q_TIGHT):  # the tighter widening for checks near contact at the limits
            ok, dofs, ev = prove(m, ck, mq, verbose=a.v)
            print(f"check {c} {ck['links']}: joints {dofs}, limits -+ {mq}: "
                  f"{'PROVEN never fires' if ok else 'not proven'} ({ev} boxes)")
            if ok:
                proven.append((c, dofs, mq))
                break
    if proven:
        worst = verify(m, [c for c, _, _ in proven])
        print("independent sample: no proven check fires;", {c: round(v, 4) for c, v in worst.items()})
    if a.write:
        for ck in m["self_checks"]:
            for k in ("never_fires", "never_dofs", "never_lo", "never_hi"):
                ck.pop(k, None)
        for c, dofs, mq in proven:
            ck = m["self_checks"][order[c]["index"]]
            ck["never_fires"] = True
            ck["never_dofs"] = [int(d) for d in dofs]
            ck["never_lo"] = [float(m["s_a"][d] - mq) for d in dofs]
            ck["never_hi"] = [float(m["s_a"][d] + m["s_m"][d] + mq) for d in dofs]
        json.dump(m, open(a.model, "w"), indent=1)
        print("wrote", a.model)


if __name__ == "__main__":
    main()
