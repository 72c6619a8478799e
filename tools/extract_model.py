"""Extract ``model/panda.json`` (kinematic tree + collision hierarchy, as data).

    python tools/extract_model.py [--ref /root/reference] [--out model/panda.json]

Build-container tool; see tools/robot_model.py for what is extracted and from where.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import fkhh_interp as fi  # noqa: E402
import robot_model as rm  # noqa: E402


def collect_calls(ast, Q, base100):
    ev = fi.Evaluator(Q, base100, "exact64")
    ev.bind_base()
    calls = []

    def walk(stmts, depth, parent):
        for st in stmts:
            if st[0] in ("decl", "fdecl"):
                ev.env[st[1]] = ev.ev(st[2])
            elif st[0] == "if":
                args = [ev.arg(a) for a in st[1][1]]
                calls.append(dict(depth=depth, kind=st[1][0], args=args, parent=parent))
                walk(st[2], depth + 1, len(calls) - 1)

    walk(ast, 0, -1)
    return calls


# Per-robot sources: spherized URDF (the file the reference's FK generator consumed), generated
# fk.hh, root link, and the robot struct's resolution (robots/panda_base.hh:21, robots/fetch.hh:13).
ROBOTS = {
    "panda": dict(urdf="resources/panda/panda_spherized.urdf", fk="src/impl/vamp/robots/panda/fk.hh",
                  root="panda_link0", resolution=32, has_base=True),
    "fetch": dict(urdf="resources/fetch/fetch_spherized.urdf", fk="src/impl/vamp/robots/fetch/fk.hh",
                  root="base_link", resolution=32, has_base=False),
    "ur5": dict(urdf="resources/ur5/ur5_spherized.urdf", fk="src/impl/vamp/robots/ur5/fk.hh",
                root="offset_link", resolution=32, has_base=False),         # robots/ur5.hh:11-12
    "baxter": dict(urdf="resources/baxter/baxter_spherized.urdf", fk="src/impl/vamp/robots/baxter/fk.hh",
                   root="base", resolution=64, has_base=False),             # robots/baxter.hh:11-12
}


def parse_const_array(src, name):
    m = re.search(name + r"\{([^}]*)\}", src)
    return [float(v.strip().rstrip("f")) for v in m.group(1).split(",")]


def extract_robot(ref, robot, variant=""):
    """variant "" = interleaved_sphere_fk (Robot::fkcc); "attach" = interleaved_sphere_fk_attachment
    (Robot::fkcc_attach, planning/validate.hh:43): its own bounding spheres, plus checks of the
    attached spheres against links ("att") and against the environment ("attenv"), posed at the
    end-effector frame recorded as ee_frame."""
    cfg = ROBOTS[robot]
    fn = "interleaved_sphere_fk_attachment" if variant == "attach" else "interleaved_sphere_fk"
    urdf = f"{ref}/{cfg['urdf']}"
    fkhh = f"{ref}/{cfg['fk']}"
    src = open(fkhh).read()
    links, joints = rm.parse_urdf(urdf)
    frames = rm.build_frames(links, joints, cfg["root"])
    fname = [f["name"] for f in frames]
    fk = fi.parse_function(src, r"inline void sphere_fk\(")
    cc = fi.parse_function(src, rf"inline bool {fn}\(")
    cc_text = fi.function_body(src, rf"inline bool {fn}\(")
    # top-level checks in text order: the generator's link label, or None for an unlabeled
    # single-sphere link tested directly (a leaf: its hit is a collision, no children)
    labels = [m.group(2) for m in re.finditer(r"^        if \((/\*(.*?)\*/)?", cc_text, re.M)]

    rng = np.random.default_rng(12345)
    K = 8
    lo = np.array([f["lower"] for f in frames if f["dof"] >= 0])
    hi = np.array([f["upper"] for f in frames if f["dof"] >= 0])
    Q = lo + rng.random((K, len(lo))) * (hi - lo)
    xyz, rad = fi.run_sphere_fk(fk, Q, (0, 0, 0), mode="exact64")
    poses = [rm.fk_exact(frames, Q[k]) for k in range(K)]

    def local_in(fidx, pts):
        loc = np.array([rm.qmat(poses[k][0][fidx]).T @ (pts[k] - poses[k][1][fidx]) for k in range(K)])
        return loc, np.abs(loc - loc[0]).max()

    # ---- spheres: reference index -> (frame, URDF offset, radius)
    spheres = []
    for s in range(xyz.shape[1]):
        pts = xyz[:, s, :].T
        found = None
        for fidx, f in enumerate(frames):
            loc, spread = local_in(fidx, pts)
            if spread > 2e-6:
                continue
            for j, (o, r) in enumerate(links[f["name"]]):
                if np.abs(np.array(o) - loc[0]).max() < 2e-6 and abs(r - rad[s]) < 1e-9:
                    found = dict(frame=fidx, offset=[float(v) for v in o], radius=float(r), link=f["name"], urdf_index=j)
        if found is None:
            raise RuntimeError(f"sphere {s} not matched")
        spheres.append(found)

    def sphere_at(pts, r):
        d = np.abs(xyz - pts.T[:, None, :]).max(axis=(0, 2))
        hits = [s for s in range(len(spheres)) if d[s] < 2e-6 and abs(rad[s] - r) < 1e-9]
        return hits[0] if len(hits) == 1 else None

    calls0 = collect_calls(cc, Q, (0, 0, 0))
    calls1 = collect_calls(cc, Q, (200, 200, 0))
    top = [i for i, c in enumerate(calls0) if c["depth"] == 0]
    assert len(top) == len(labels), (len(top), len(labels))

    bounding = {}  # link -> dict
    env_checks = []
    self_checks = []

    def has_base(i, argslice):
        a = np.stack([calls0[i]["args"][k] for k in argslice])
        b = np.stack([calls1[i]["args"][k] for k in argslice])
        d = b - a
        if np.abs(d).max() < 1e-9:
            return False
        assert np.allclose(d[0], 2.0) and np.allclose(d[1], 2.0) and np.allclose(d[2], 0.0), d
        return True

    # pass 1: env bounding spheres (link named in the generator's comment)
    for t, lab in zip(top, labels):
        c = calls0[t]
        if c["kind"] != "env":
            continue
        pts = np.stack(c["args"][:3]).T
        if lab is None:  # leaf: one sphere, `return false` on a hit (fetch/fk.hh torso_lift_link_collision_2)
            s = sphere_at(pts, float(c["args"][3][0]))
            assert s is not None and not any(cc_["parent"] == t for cc_ in calls0)
            link = spheres[s]["link"]
            b = dict(link=link, frame=spheres[s]["frame"], offset=spheres[s]["offset"], radius=spheres[s]["radius"],
                     base=has_base(t, range(3)), leaf_sphere=s)
            bounding[link] = b
            env_checks.append(dict(link=link, bounding_base=b["base"], children=[], leaf=True))
            continue
        link = lab.strip()
        fidx = fname.index(link)
        loc, spread = local_in(fidx, pts)
        assert spread < 2e-6, (link, spread)
        r = float(c["args"][3][0])
        kids = [i for i, cc_ in enumerate(calls0) if cc_["parent"] == t]
        children = []
        for i in kids:
            kp = np.stack(calls0[i]["args"][:3]).T
            s = sphere_at(kp, float(calls0[i]["args"][3][0]))
            assert s is not None, (link, i)
            children.append(dict(sphere=s, base=has_base(i, range(3))))
        b = dict(link=link, frame=fidx, offset=[float(round(v, 6)) for v in loc[0]], radius=r, base=has_base(t, range(3)))
        bounding[link] = b
        ck = dict(link=link, bounding_base=b["base"], children=children)
        if not kids:  # a labeled single-sphere link tested directly (ur5/fk.hh fts_robotside): leaf
            ck["leaf"] = True
        env_checks.append(ck)

    def entity(pts, r):
        s = sphere_at(pts, r)
        if s is not None:
            return dict(sphere=s)
        for link, b in bounding.items():
            fidx = b["frame"]
            loc, spread = local_in(fidx, pts)
            if spread < 2e-6 and np.abs(loc[0] - np.array(b["offset"])).max() < 2e-6 and abs(r - b["radius"]) < 1e-9:
                return dict(bound=link)
        raise RuntimeError("unmatched self-collision entity")

    def entity_or_new(pts, r, link):
        try:
            return entity(pts, r)
        except RuntimeError:  # a link-bounding sphere that no environment check uses
            fidx = fname.index(link)
            loc, spread = local_in(fidx, pts)
            assert spread < 2e-6, (link, spread)
            key = f"{link}#att"
            bounding[key] = dict(link=key, frame=fidx, offset=[float(round(v, 6)) for v in loc[0]], radius=r,
                                 base=False)
            return dict(bound=key)

    att_checks = []
    order = []
    for t, lab in zip(top, labels):
        c = calls0[t]
        if c["kind"] == "attenv":  # attached spheres vs the environment (validity.hh:251-266)
            order.append(dict(kind="attenv", index=0))
            continue
        if c["kind"] == "att":  # "attachment vs. <link>" (validity.hh:269-293)
            link = lab.split("vs.")[1].strip()
            e = entity_or_new(np.stack(c["args"][:3]).T, float(c["args"][3][0]), link)
            kids = [i for i, cc_ in enumerate(calls0) if cc_["parent"] == t]
            ch = [sphere_at(np.stack(calls0[i]["args"][:3]).T, float(calls0[i]["args"][3][0])) for i in kids]
            assert all(x is not None for x in ch)
            ck = dict(link=link, ent=e, children=ch)
            if not kids:
                ck["leaf"] = True
            att_checks.append(ck)
            order.append(dict(kind="att", index=len(att_checks) - 1))
            continue
        if c["kind"] == "env":
            lk = lab.strip() if lab is not None else spheres[sphere_at(np.stack(c["args"][:3]).T, float(c["args"][3][0]))]["link"]
            order.append(dict(kind="env", index=[e["link"] for e in env_checks].index(lk)))
            continue
        a_link, b_link = [s.strip() for s in lab.split("vs.")]
        pa, pb = np.stack(c["args"][:3]).T, np.stack(c["args"][4:7]).T
        ea = entity_or_new(pa, float(c["args"][3][0]), a_link)
        eb = entity_or_new(pb, float(c["args"][7][0]), b_link)
        kids = [i for i, cc_ in enumerate(calls0) if cc_["parent"] == t]
        pairs = []
        for i in kids:
            ka = sphere_at(np.stack(calls0[i]["args"][:3]).T, float(calls0[i]["args"][3][0]))
            kb = sphere_at(np.stack(calls0[i]["args"][4:7]).T, float(calls0[i]["args"][7][0]))
            assert ka is not None and kb is not None
            pairs.append([ka, kb])
        self_checks.append(dict(links=[a_link, b_link], a=ea, b=eb, children=pairs))
        order.append(dict(kind="self", index=len(self_checks) - 1))

    dof_frames = [f for f in frames if f["dof"] >= 0]
    s_m = parse_const_array(src, "s_m_a")
    s_a = parse_const_array(src, "s_a_a")
    d_m = parse_const_array(src, "d_m_a")
    space = float(re.search(r"space_measure\(\) noexcept -> float\s*\{\s*return ([0-9.e+-]+);", src).group(1))
    assert len(s_m) == len(dof_frames)
    model = dict(
        robot=robot,
        source=dict(urdf=cfg["urdf"], fk=cfg["fk"]),
        dimension=len(dof_frames),
        resolution=cfg["resolution"],
        # scale_configuration: q * s_m + s_a; descale (q - s_a) * d_m (fk.hh s_m_a/s_a_a/d_m_a arrays)
        s_m=s_m,
        s_a=s_a,
        d_m=d_m,
        space_measure=space,
        frames=[dict(name=f["name"], parent=f["parent"], t=f["t"], qf=f["qf"], dof=f["dof"],
                     **({} if f["jtype"] in ("fixed", "root") or (f["jtype"] != "prismatic" and f["axis"] == [0.0, 0.0, 1.0])
                        else dict(jtype=f["jtype"], axis=f["axis"])))
                for f in frames],
        spheres=spheres,
        bounding=list(bounding.values()),
        env_checks=env_checks,
        self_checks=self_checks,
        check_order=order,
    )
    if variant == "attach":
        model["robot"] = f"{robot}_attach"
        model["att_checks"] = att_checks
        model["ee_frame"] = ee_frame_of(cc, frames, Q, poses, fi)
    return model


def ee_frame_of(cc, frames, Q, poses, fi):
    """The frame whose pose set_attachment_pose receives: position = its origin, orientation =
    its quaternion (x, y, z, w), checked over the sample configurations."""
    ev = fi.Evaluator(Q, (0, 0, 0), "exact64")
    ev.bind_base()
    vals = None
    for st in cc:
        if st[0] in ("decl", "fdecl"):
            ev.env[st[1]] = ev.ev(st[2])
        elif st[0] == "setpose":
            vals = np.array([ev.arg(a) for a in st[1]])
            break
    for fidx in range(len(frames)):
        ok = True
        for k in range(Q.shape[0]):
            qf, pf = poses[k][0][fidx], poses[k][1][fidx]
            w, x, y, z = qf
            if np.abs(vals[:3, k] - pf).max() > 2e-6 or np.abs(vals[3:, k] - np.array([x, y, z, w])).max() > 2e-6:
                ok = False
                break
        if ok:
            return fidx
    raise RuntimeError("end-effector frame not found")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--robot", default="panda", choices=sorted(ROBOTS))
    ap.add_argument("--variant", default="", choices=["", "attach"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.out is None:
        suffix = "_attach" if a.variant else ""
        a.out = os.path.join(os.path.dirname(__file__), "..", "model", f"{a.robot}{suffix}.json")
    m = extract_robot(a.ref, a.robot, a.variant)
    with open(a.out, "w") as f:
        json.dump(m, f, indent=1)
    print(f"wrote {a.out}: {len(m['spheres'])} spheres, {len(m['env_checks'])} env checks "
          f"({sum(len(c['children']) for c in m['env_checks'])} children), {len(m['self_checks'])} self pairs "
          f"({sum(len(c['children']) for c in m['self_checks'])} children)")


if __name__ == "__main__":
    main()
