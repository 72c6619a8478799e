"""Robot kinematic model: URDF tree -> frames/spheres, and extraction of the reference's
collision hierarchy as data.

MODEL EXTRACTION ONLY (build container).  The output, ``model/<robot>.json``, is plain data
(joint offsets, sphere offsets/radii, link-bounding spheres, self-collision pairs); the
product's kernels and the oracle are generated from / driven by that data, not from any
reference source text.

Sources of the data:
* kinematic tree, joint origins and collision spheres: the reference's spherized URDF
  (``resources/panda/panda_spherized.urdf``) -- the same file its FK generator consumed;
* the sphere ordering (0..58), the 11 link-bounding spheres, which children each
  bounding check covers, the 21 self-collision link pairs, and the base-offset quirks:
  recovered numerically from ``robots/panda/fk.hh`` by evaluating its expression DAG with
  ``tools/fkhh_interp.py`` (exact64 mode) at random configurations and solving for the
  frame-local offsets.  Every extracted number is checked to be configuration-independent.
"""
from __future__ import annotations

import json
import math
import xml.etree.ElementTree as ET
from typing import Dict, List, Tuple

import numpy as np


def rpy_to_quat(r, p, y):
    """URDF fixed-axis rpy -> quaternion (w, x, y, z) = qz(y) * qy(p) * qx(r)."""
    cr, sr = math.cos(r / 2), math.sin(r / 2)
    cp, sp = math.cos(p / 2), math.sin(p / 2)
    cy, sy = math.cos(y / 2), math.sin(y / 2)
    return (
        cy * cp * cr + sy * sp * sr,
        cy * cp * sr - sy * sp * cr,
        sy * cp * sr + cy * sp * cr,
        sy * cp * cr - cy * sp * sr,
    )


def qmul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return (
        aw * bw - ax * bx - ay * by - az * bz,
        aw * bx + ax * bw + ay * bz - az * by,
        aw * by - ax * bz + ay * bw + az * bx,
        aw * bz + ax * by - ay * bx + az * bw,
    )


def qmat(q):
    w, x, y, z = q
    return np.array(
        [
            [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
            [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
            [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
        ]
    )


def parse_urdf(path):
    root = ET.parse(path).getroot()
    links = {}
    for ln in root.findall("link"):
        spheres = []
        for col in ln.findall("collision"):
            g = col.find("geometry")
            s = g.find("sphere") if g is not None else None
            if s is None:
                continue
            o = col.find("origin")
            xyz = [float(v) for v in o.get("xyz", "0 0 0").split()] if o is not None else [0, 0, 0]
            spheres.append((xyz, float(s.get("radius"))))
        links[ln.get("name")] = spheres
    joints = []
    for j in root.findall("joint"):
        o = j.find("origin")
        xyz = [float(v) for v in o.get("xyz", "0 0 0").split()] if o is not None else [0.0, 0.0, 0.0]
        rpy = [float(v) for v in o.get("rpy", "0 0 0").split()] if o is not None else [0.0, 0.0, 0.0]
        ax = j.find("axis")
        axis = [float(v) for v in ax.get("xyz").split()] if ax is not None else [0.0, 0.0, 0.0]
        lim = j.find("limit")
        joints.append(
            dict(
                name=j.get("name"),
                type=j.get("type"),
                parent=j.find("parent").get("link"),
                child=j.find("child").get("link"),
                xyz=xyz,
                rpy=rpy,
                axis=axis,
                lower=float(lim.get("lower")) if lim is not None and lim.get("lower") else None,
                upper=float(lim.get("upper")) if lim is not None and lim.get("upper") else None,
            )
        )
    return links, joints


def round_const(v):
    """The reference generator prints irrational constants with 7 significant digits
    (e.g. 0.7071068, 0.9238795); exact decimals stay exact."""
    if abs(v) < 1e-12:
        return 0.0
    r = float(f"{v:.7g}")
    return r


def build_frames(links, joints, root_link):
    """Frames in topological order: [{name, parent, t(xyz), qf(wxyz), joint (dof idx or -1)}]."""
    children: Dict[str, List[dict]] = {}
    for j in joints:
        children.setdefault(j["parent"], []).append(j)
    movable = [j["name"] for j in joints if j["type"] in ("revolute", "continuous", "prismatic")
               and (links.get(j["child"]) or children.get(j["child"]))]
    frames = [dict(name=root_link, parent=-1, t=[0.0, 0.0, 0.0], qf=[1.0, 0.0, 0.0, 0.0], dof=-1, jtype="root")]
    dof = 0
    order = [root_link]
    idx = {root_link: 0}
    stack = [root_link]
    while stack:
        ln = stack.pop(0)
        for j in children.get(ln, []):
            c = j["child"]
            if not links.get(c) and not children.get(c):
                # frames with neither spheres nor descendants (grasptarget) are irrelevant
                continue
            qf = [round_const(v) for v in rpy_to_quat(*j["rpy"])]
            d = -1
            axis = [0.0, 0.0, 0.0]
            if j["type"] in ("revolute", "continuous", "prismatic"):
                # unit coordinate axes (+-x, +-y, +-z): the joint quaternion / displacement keeps
                # the other two components structurally zero
                assert sorted(abs(v) for v in j["axis"]) == [0.0, 0.0, 1.0], f"axis {j['axis']} ({j['name']})"
                axis = [float(v) for v in j["axis"]]
                # configuration index = the joint's position among the URDF's movable joints in
                # document order (the reference generator's q order; BFS order differs for
                # branching robots such as Baxter's two arms)
                d = movable.index(j["name"])
                dof += 1
            frames.append(
                dict(name=c, parent=idx[ln], t=[float(v) for v in j["xyz"]], qf=qf, dof=d,
                     jtype=j["type"] if d >= 0 else "fixed", axis=axis, lower=j["lower"], upper=j["upper"])
            )
            idx[c] = len(frames) - 1
            order.append(c)
            stack.append(c)
    return frames


def fk_exact(frames, q):
    """Exact (float64, exact trig) frame poses for one configuration."""
    Q = []
    P = []
    for f in frames:
        if f["parent"] < 0:
            Q.append((1.0, 0.0, 0.0, 0.0))
            P.append(np.zeros(3))
            continue
        qp, pp = Q[f["parent"]], P[f["parent"]]
        qc = qmul(qp, tuple(f["qf"]))
        pc = pp + qmat(qp) @ np.array(f["t"])
        if f["dof"] >= 0 and f.get("jtype") == "prismatic":
            pc = pc + qmat(qc) @ (q[f["dof"]] * np.array(f["axis"]))
        elif f["dof"] >= 0:
            th = q[f["dof"]]
            ax = f.get("axis", [0.0, 0.0, 1.0])
            s = math.sin(th / 2)
            qc = qmul(qc, (math.cos(th / 2), s * ax[0], s * ax[1], s * ax[2]))
        Q.append(qc)
        P.append(pc)
    return Q, P


def locate(points_by_q, poses_by_q, frames, tol=1e-7):
    """For a point evaluated at several configurations, find the frame in which its local
    coordinates are constant.  points_by_q: (K, 3); poses_by_q: list over K of (Q, P).
    Returns (frame_index, local_offset)."""
    best = None
    for fi_ in range(len(frames)):
        locs = []
        for k in range(points_by_q.shape[0]):
            Q, P = poses_by_q[k]
            R = qmat(Q[fi_])
            locs.append(R.T @ (points_by_q[k] - P[fi_]))
        locs = np.array(locs)
        spread = np.abs(locs - locs[0]).max()
        if spread < tol:
            # prefer the deepest (last) frame with a constant offset whose offset is "nice"
            cand = (fi_, locs.mean(0))
            if best is None or frames[fi_]["dof"] >= 0 or np.abs(cand[1]).sum() < np.abs(best[1]).sum() - 1e-9:
                best = cand
    return best
