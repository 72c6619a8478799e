"""An independent Python restatement of RRT-Connect (planning/rrtc.hh:33-248) -- test
infrastructure, the checker of the product's C++ planner (mr-vamp_amd/csrc/cpu/vcpu_rrtc.cpp).

Its edge checks are the oracle's validate_vector (oracle/vamp_oracle.c), its samples the oracle's
Halton closed form + scale_configuration, its nearest neighbours a numpy scan in float32 with
FloatVector::l2_norm's lane order (nn.hh:53-57).  Both restate the same source independently, so
equal paths, costs, iterations and tree sizes pin the product's planner logic (the reference
itself cannot be compiled here: nigh is absent)."""
import numpy as np

import oracle_py as op

F = np.float32
FMAX = np.finfo(np.float32).max


def fma_sq(a, c):
    """float32 fma(a, a, c), correctly rounded (one rounding of a*a + c), vectorised: a*a is exact in float64,
    TwoSum gives the float64 sum's error, and a sum that sits exactly on a float32 rounding midpoint is nudged
    toward the error's sign so the float32 conversion rounds the exact value"""
    a64 = np.asarray(a, np.float64)
    c64 = np.asarray(c, np.float64)
    p = a64 * a64
    s = p + c64
    bv = s - p
    e = (p - (s - bv)) + (c64 - bv)
    r = s.astype(F)
    other = np.nextafter(r, np.where(s > r, np.inf, -np.inf).astype(F)).astype(F)
    mid = (r.astype(np.float64) + other.astype(np.float64)) / 2
    tie = (s == mid) & (e != 0)
    if tie.any():
        s = np.where(tie, np.nextafter(s, s + e), s)
        r = s.astype(F)
    return r


def l2_rows(d):
    """FloatVector<dim>::l2_norm of each row (hsum order of avx.hh:441-452; dim <= 8: one register; dim 9-16:
    two, combined lane-wise as fma(lo, lo, hi * hi) by the release build -- ref_probe l2norm)"""
    d = np.asarray(d, F)
    s = np.zeros((d.shape[0], 8), F)
    if d.shape[1] <= 8:
        s[:, :d.shape[1]] = d * d
    else:
        hi = np.zeros((d.shape[0], 8), F)
        hi[:, :d.shape[1] - 8] = d[:, 8:]
        s[:] = fma_sq(d[:, :8], (hi * hi).astype(F))
    a = (s[:, 0] + s[:, 4]) + (s[:, 2] + s[:, 6])
    b = (s[:, 1] + s[:, 5]) + (s[:, 3] + s[:, 7])
    return np.sqrt(a + b).astype(F)


def rrtc(robot, oenv, start, goals, settings, rng_index, base100=(0, 0, 0)):
    S = dict(range=2.0, dynamic_domain=True, radius=4.0, alpha=0.0001, min_radius=1.0, balance=True,
             tree_ratio=1.0, max_iterations=100000, max_samples=100000, start_tree_first=True)
    S.update(settings)
    rng_f = F(S["range"])
    ec = oenv.c()
    dim = len(start)
    start = np.asarray(start, F)
    goals = np.asarray(goals, F).reshape(-1, dim)

    def vv(s, v, d):
        if robot == "pair":  # the configs[4] composite: base100 = (arm A's base, arm B's base)
            return op.pair_validate_vector(ec, s, v, d, *base100)
        return op.robot_validate_vector(robot, ec, s, v, d, base100)

    def scale(u):
        return op.pair_scale(u) if robot == "pair" else op.robot_scale(robot, u)

    for g in goals:  # rrtc.hh:61-73
        if vv(start, (g - start).astype(F), l2_rows((g - start)[None])[0]):
            return np.stack([start, g]), F(0), 0, (1, 1), rng_index

    buf, parents, radii = [], [], []

    def push(q, parent=None):
        buf.append(np.asarray(q, F).copy())
        parents.append(len(buf) - 1 if parent is None else parent)
        radii.append(FMAX)
        return len(buf) - 1

    start_tree, goal_tree = [push(start)], []
    for g in goals:
        goal_tree.append(push(g))
    tree_a_is_start = not S["start_tree_first"]
    ta, tb = (goal_tree, start_tree) if S["start_tree_first"] else (start_tree, goal_tree)

    def nearest(tree, q):
        C = np.stack([buf[i] for i in tree])
        d = l2_rows((q[None, :] - C).astype(F))
        k = int(np.argmin(d))
        return tree[k], d[k]

    it = 0
    path = []
    cost = F(0)
    while True:
        it += 1
        if not (it - 1 < S["max_iterations"] and len(buf) < S["max_samples"]):
            break
        asize, bsize = F(len(ta)), F(len(tb))
        ratio = F(abs(asize - bsize)) / asize
        if (not S["balance"]) or ratio < F(S["tree_ratio"]):
            ta, tb = tb, ta
            tree_a_is_start = not tree_a_is_start
        temp = scale(op.halton(dim, [rng_index]))[0]
        rng_index += 1
        nn, nd = nearest(ta, temp)
        nr = radii[nn]
        if S["dynamic_domain"] and nr < nd:
            continue
        nc = buf[nn]
        v = (temp - nc).astype(F)
        reach = nd < rng_f
        ext = v if reach else (v * (rng_f / nd)).astype(F)
        if vv(nc, ext, nd if reach else rng_f):
            newc = (nc + ext).astype(F)
            ta.append(push(newc, nn))
            if S["dynamic_domain"] and nr != FMAX:
                radii[nn] = F(radii[nn] * (F(1) + F(S["alpha"])))
            on, od = nearest(tb, newc)
            onv = (buf[on] - newc).astype(F)
            n_ext = int(np.ceil(od / rng_f))
            inc_len = F(od / F(n_ext)) if n_ext else F(np.nan)
            inc = (onv * (F(1) / F(n_ext))).astype(F) if n_ext else onv
            prior = newc
            i = 0
            while i < n_ext and vv(prior, inc, inc_len) and len(buf) < S["max_samples"]:
                nxt = (prior + inc).astype(F)
                ta.append(push(nxt, len(buf) - 1))
                prior = nxt
                i += 1
            if i == n_ext:
                cur = len(buf) - 1
                path = [buf[cur]]
                while parents[cur] != cur:
                    cur = parents[cur]
                    path.append(buf[cur])
                    cost = F(cost + l2_rows((path[-1] - path[-2])[None])[0])
                path.reverse()
                cur = on
                while parents[cur] != cur:
                    cur = parents[cur]
                    path.append(buf[cur])
                    cost = F(cost + l2_rows((path[-1] - path[-2])[None])[0])
                if not tree_a_is_start:
                    path.reverse()
                break
        elif S["dynamic_domain"]:
            radii[nn] = F(S["radius"]) if nr == FMAX else max(F(radii[nn] * (F(1) - F(S["alpha"]))),
                                                              F(S["min_radius"]))
    sizes = (len(start_tree), len(goal_tree))
    return (np.stack(path) if path else np.zeros((0, dim), F)), cost, it, sizes, rng_index
