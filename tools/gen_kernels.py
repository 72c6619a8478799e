"""Generate the robot-specific HIP device code from model/<robot>.json.

    python tools/gen_kernels.py model/panda.json mr-vamp_amd/csrc/gen/panda_fk.inc

Emits two straight-line device functions for a robot:

* ``<robot>_sphere_fk_store``  -- all collision-sphere centres of one configuration,
  streamed to SoA outputs (the HBM-bound FK kernel);
* ``<robot>_fkcc<Grp>``       -- FK interleaved with the hierarchical environment and
  self-collision checks (the VALU-bound mask kernel), early-exiting per rake group.

The FK arithmetic follows the canonical order documented in oracle/vamp_oracle.c (half
angle -> Horner sin/cos -> Hamilton products -> R(Q) -> P + R o), with structurally-zero
terms dropped and constant subexpressions folded in IEEE float32 (numpy), so every
emitted operation is one float32 op identical to the oracle's.  The generator is this
project's own; it consumes only the data in model/<robot>.json.
"""
from __future__ import annotations

import json
import sys
from typing import Dict, List, Optional, Tuple

import numpy as np

F = np.float32
REMAT = False  # rebuild rotation matrices per check (A/B on MI355X: 5.80 -> 6.81 ms, off)
HOLD = True    # GPU self-pair children: hold the smaller side's centres, stream the other (--no-hold: chunks)
GATE = True    # GPU staged bound stage: the wrist checks' (q5, q6) gate table when the model has one (--no-gate)
# GPU staged bound stage (--mids): mid-level spheres between a link-bounding sphere and its children.  A check
# whose bounding test fires gets its bit only if one of a few spheres, each enclosing a cluster of the
# check's children with a 0.1 mm margin, passes a CONSERVATIVE test (environment: a cull extent that bounds
# the reference's approximate one from above; self: a plain overlap).  A child the reference reports hit
# lies inside some mid sphere, so that sphere's test fires: results are unchanged, and bounding hits that no
# child confirms (most of a validate tail's) queue no children.  {link: clusters} / {(link_a, link_b): ...}
# The mid tests sit behind the bound function's MID template flag: the staged kernels turn it on per source
# kind (R::kMidKinds, vgpu_staged.hh MidBound), since they pay only where bounding hits rarely confirm.
MIDS = None
# GPU staged lead pass: {robot: link} -- that link's environment check, bounding test and children in one
# monolithic pass before the bound stage (vgpu_staged.hh lead_kernel), so that the groups it invalidates
# skip the bound stage.  The Panda's link 5: it fires for ~every group of an invalid-heavy batch and
# its children confirm 97 % of them there (tools/hitstats.py).
LEAD = {"panda": "panda_link5"}
# GPU staged children: robots whose environment children leave at the group's first hit (primitive
# environments).  Off: for the Panda it changed nothing measurable (set B 2.33-2.36 vs 2.33-2.34 ms, pair
# 10.49 vs 10.43-10.50; profiles/r04q_early_ab.log) -- unlike the lead pass, where it took set A 1.06 -> 0.81
EARLY_CHILDREN = set()
# GPU staged bound stage: each check's test bit accumulated per LANE (lm |= bit << c), one OR over the
# group at the end -- instead of a group reduction (3 DPP ops) and a divergent branch per check (--no-lane-bits).
# Checks whose branch saves work keep it: mid-sphere tests, the never-fires guard, the gate.  8-lane groups
# only (validate heads and tails): A/B on MI355X (profiles/r05j_ab.log) Fetch edge-stage validation 371 -> 298 ms
# at 2.68M vertices (its 8-lane bound kernels 92 -> 62 VGPRs), Panda set B 2.22-2.24 -> 2.17-2.19 ms, composite
# 8.67 -> 8.50 ms; single-lane groups keep the branch (the CAPT bound kernel went 77 -> 81 VGPRs, 0.52 -> 0.54 ms)
LANE_BITS = True
MID_ENV = {"panda_link5": 4, "panda_hand": 4, "panda_link7": 3}
MID_SELF_LINKS = {"panda_link1": 2, "panda_link2": 2, "panda_link5": 4,
                  # Fetch (--mids on fetch.json): the self checks whose tails queue the most children items and
                  # whose children almost never confirm (tools/hitstats.py --fetch, profiles/r04n_hitstats_fetch.json)
                  "head_pan_link": 4, "upperarm_roll_link": 2, "elbow_flex_link": 2, "forearm_roll_link": 2,
                  "base_link": 3, "torso_lift_link": 2, "torso_fixed_link": 2}
# (finer Fetch clusters -- head 8, upper arm 4, elbow 3, forearm 3, base 6 -- measured slower on MI355X: edge-stage
# validation 297 -> 346 ms at 2.68M vertices, profiles/r05p_ab.log; the extra mid tests cost more than they filter)
MID_SELF_CHECKS = [("panda_link1", "panda_link5"), ("panda_link2", "panda_link5"),
                   ("head_pan_link", "upperarm_roll_link"), ("head_pan_link", "elbow_flex_link"),
                   ("head_pan_link", "forearm_roll_link"), ("base_link", "elbow_flex_link"),
                   ("base_link", "forearm_roll_link"), ("torso_lift_link", "forearm_roll_link"),
                   ("forearm_roll_link", "torso_fixed_link"), ("elbow_flex_link", "torso_fixed_link"),
                   ("torso_lift_link", "elbow_flex_link")]
MID_MARGIN = 1e-4
# GPU lead pass (--no-near: off): the lead check's children after one sphere S enclosing every child with MID_MARGIN
# is scanned against the environment (vgpu_device.hh env_near: per lane, the records S touches); each child then walks
# only its lane's records (env_bits_near) -- a child can only hit a record its enclosing sphere touches, so the
# results are the reference's.  Lead only: in the staged children kernels the near-set code pushed the class-0
# kernel past its 64-VGPR budget (spills) and made them slower (A/B on MI355X).  Children spread
# over several frames or base flags keep the full scans.
NEAR = True
# GPU staged children with near sets too: {robot: least number of children} -- the checks with that many children
# (the Panda's link 5: 12, hand: 18), which the robot's kernels run in a children class of their own (vgpu_staged.hip
# PandaR::kClassOf): in the shared class-0 kernel the near code of every check spilled (see NEAR)
NEAR_CHILDREN = {"panda": 8}
# GPU staged bound stage (--cluster): the bounding tests of these links share one near set -- a sphere E enclosing
# their bounding spheres, built per configuration from the centres the tests use (so it encloses them whatever the
# base-offset quirks), scanned once (env_near), then each member's test walks only its lane's records E touches
# (env_bits_e: env_bits_near, or env_bits without near sets / with point clouds).
CLUSTER = {}
CLUSTER_LINKS = {"panda": ["panda_link6", "panda_link7", "panda_hand", "panda_leftfinger", "panda_rightfinger"]}

# Emitted types.  The HIP kernels compute one configuration per lane in `float` with the
# per-lane check bits in `uint32_t`; the CPU restatement (--cpu, mr-vamp_amd/csrc/cpu/) emits
# the SAME expression text over 8-lane AVX2 vectors: `V` (one rake block, __m256) and `VB`
# (sign-bit lane masks), so both are the same op sequence (vcpu_simd.hh supplies the operators).
TY = {"f": "float", "b": "uint32_t", "b0": "0u", "qual": "__device__ __forceinline__", "cpu": False}
TY_CPU = {"f": "V", "b": "VB", "b0": "VB()", "qual": "VCPU_INLINE", "cpu": True}


def bdecl(name, comment=""):
    """declaration of a zeroed check-bit accumulator"""
    return f"{TY['b']} {name} = {TY['b0']};" + (f"  // {comment}" if comment else "")


def xyzr_decl():
    return "V X, Y, Z; float R;" if TY["cpu"] else "float X, Y, Z, R;"


def flit(v) -> str:
    v = float(F(v))
    if v == 0.0:
        return "0.0f"
    return f"{v.hex()}f"


class SV:
    """A structural value: zero, a float32 constant, or a named runtime float."""

    __slots__ = ("kind", "val", "name")

    def __init__(self, kind, val=None, name=None):
        self.kind, self.val, self.name = kind, val, name

    @staticmethod
    def zero():
        return SV("zero")

    @staticmethod
    def const(v):
        v = F(v)
        return SV("zero") if v == 0 else SV("const", v)

    def expr(self):
        if self.kind == "zero":
            return "0.0f"
        if self.kind == "const":
            return flit(self.val)
        return self.name


class Emitter:
    def __init__(self):
        self.lines: List[str] = []
        self.n = 0
        self.indent = 1
        self.flops = 0

    def tmp(self, expr) -> SV:
        name = f"t{self.n}"
        self.n += 1
        self.lines.append("    " * self.indent + f"const {TY['f']} {name} = {expr};")
        self.flops += 1
        return SV("var", name=name)

    def raw(self, line):
        self.lines.append("    " * self.indent + line)

    def opaque(self, a: SV) -> SV:
        """A copy of a runtime value the compiler cannot see through (empty asm with a "+v"
        constraint), so values recomputed from it are not merged back with earlier ones by
        CSE/GVN -- rematerialisation instead of a long live range."""
        if a.kind != "var":
            return a
        name = f"t{self.n}"
        self.n += 1
        self.lines.append("    " * self.indent + f"float {name} = {a.name}; __asm__ volatile(\"\" : \"+v\"({name}));")
        return SV("var", name=name)

    # --- sv arithmetic mirroring oracle/vamp_oracle.c sv_* ---
    def mul(self, a: SV, b: SV) -> SV:
        if a.kind == "zero" or b.kind == "zero":
            return SV.zero()
        if a.kind == "const" and b.kind == "const":
            return SV.const(F(a.val) * F(b.val))
        # x * 1 and x * -1 are exact: no op needed, same bits
        for x, y in ((a, b), (b, a)):
            if y.kind == "const" and y.val == F(1):
                return x
        return self.tmp(f"{a.expr()} * {b.expr()}")

    def neg(self, a: SV) -> SV:
        if a.kind == "zero":
            return a
        if a.kind == "const":
            return SV.const(-a.val)
        return self.tmp(f"-{a.expr()}")

    def add(self, a: SV, b: SV) -> SV:
        if a.kind == "zero":
            return b
        if b.kind == "zero":
            return a
        if a.kind == "const" and b.kind == "const":
            return SV.const(F(a.val) + F(b.val))
        return self.tmp(f"{a.expr()} + {b.expr()}")

    def sub(self, a: SV, b: SV) -> SV:
        if b.kind == "zero":
            return a
        if a.kind == "zero":
            return self.neg(b)
        if a.kind == "const" and b.kind == "const":
            return SV.const(F(a.val) - F(b.val))
        return self.tmp(f"{a.expr()} - {b.expr()}")


def qmul(E: Emitter, a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    m = E.mul
    w = E.sub(E.sub(E.sub(m(aw, bw), m(ax, bx)), m(ay, by)), m(az, bz))
    x = E.sub(E.add(E.add(m(aw, bx), m(ax, bw)), m(ay, bz)), m(az, by))
    y = E.add(E.add(E.sub(m(aw, by), m(ax, bz)), m(ay, bw)), m(az, bx))
    z = E.add(E.sub(E.add(m(aw, bz), m(ax, by)), m(ay, bx)), m(az, bw))
    return (w, x, y, z)


def qmat(E: Emitter, q):
    w, x, y, z = q
    one, two = SV.const(1.0), SV.const(2.0)
    m = E.mul
    xx, yy, zz = m(x, x), m(y, y), m(z, z)
    xy, xz, yz = m(x, y), m(x, z), m(y, z)
    wx, wy, wz = m(w, x), m(w, y), m(w, z)
    R = [[None] * 3 for _ in range(3)]
    R[0][0] = E.sub(one, m(E.add(yy, zz), two))
    R[0][1] = m(E.sub(xy, wz), two)
    R[0][2] = m(E.add(xz, wy), two)
    R[1][0] = m(E.add(xy, wz), two)
    R[1][1] = E.sub(one, m(E.add(xx, zz), two))
    R[1][2] = m(E.sub(yz, wx), two)
    R[2][0] = m(E.sub(xz, wy), two)
    R[2][1] = m(E.add(yz, wx), two)
    R[2][2] = E.sub(one, m(E.add(xx, yy), two))
    return R


def xform(E: Emitter, R, P, o):
    out = []
    for i in range(3):
        acc = SV.zero()
        for k in range(3):
            acc = E.add(acc, E.mul(R[i][k], SV.const(o[k])))
        out.append(E.add(P[i], acc))
    return out


def joint(E: Emitter, fr: dict, A, R_A, P, qoff: int = 0, qname: str = "q"):
    """Apply frame fr's joint after its fixed rotation: returns (Q, P).  Revolute about the unit
    axis a: Q = A (x) (c, s*a) (other components structurally zero; a negative axis negates s).
    Prismatic along a: Q = A, P += R(A) (a*q) (oracle/vamp_oracle.c robot_fk_frames)."""
    d = fr["dof"]
    if d < 0:
        return A, P
    d += qoff  # joint variable q<d>: a composite's second arm reads q7..q13
    ax = fr.get("axis", [0.0, 0.0, 1.0])
    if fr.get("jtype") == "prismatic":
        qv = SV("var", name=f"{qname}{d}")
        dq = [SV.zero() if a == 0 else (qv if a > 0 else E.neg(qv)) for a in ax]
        RA = R_A()
        out = []
        for i in range(3):
            acc = SV.zero()
            for k in range(3):
                acc = E.add(acc, E.mul(RA[i][k], dq[k]))
            out.append(E.add(P[i], acc))
        return A, out
    h = E.tmp(f"{qname}{d} * 0.5f")
    c = E.tmp(f"vamp_cos({h.name})")
    sn = E.tmp(f"vamp_sin({h.name})")
    E.flops += 2 * 16
    comp = [SV.zero() if a == 0 else (sn if a > 0 else E.neg(sn)) for a in ax]
    return qmul(E, A, (c, comp[0], comp[1], comp[2])), P


def mid_spheres(offsets, radii, k):
    """k spheres enclosing the given child spheres (offsets in one frame): children sorted along the
    principal axis of their offsets and cut into k runs of near-equal size; each run's sphere is centred on
    its box and reaches every member's far side plus MID_MARGIN (radius rounded up to float)."""
    P = np.asarray(offsets, np.float64)
    r = np.asarray(radii, np.float64)
    k = max(1, min(k, len(P)))
    if len(P) > 1:
        _, _, vt = np.linalg.svd(P - P.mean(0))
        order = np.argsort(P @ vt[0], kind="stable")
    else:
        order = np.arange(len(P))
    out = []
    for run in np.array_split(order, k):
        lo = (P[run] - r[run, None]).min(0)
        hi = (P[run] + r[run, None]).max(0)
        c = (lo + hi) / 2
        R = max(np.linalg.norm(P[i] - c) + r[i] for i in run) + MID_MARGIN
        Rf = np.float32(R)
        if float(Rf) < R:
            Rf = np.nextafter(Rf, np.float32(np.inf))
        out.append(([float(np.float32(v)) for v in c], float(Rf)))
    return out


class RobotGen:
    def __init__(self, model):
        self.m = model
        self.name = model["robot"]

    def frames_fk(self, E: Emitter, needed_frames=None):
        """Emit frame poses in topological order (all frames; cheap relative to checks)."""
        frames = self.m["frames"]
        Q, P, R = {}, {}, {}
        for f, fr in enumerate(frames):
            qf = tuple(SV.const(v) for v in fr["qf"])
            if fr["parent"] < 0:
                Q[f] = qf
                P[f] = [SV.const(v) for v in fr["t"]]
            else:
                p = fr["parent"]
                ident = list(fr["qf"]) == [1.0, 0.0, 0.0, 0.0]
                A = Q[p] if ident else qmul(E, Q[p], qf)
                if fr.get("jtype") == "prismatic":
                    if p not in R:
                        R[p] = qmat(E, Q[p])
                    Pt = xform(E, R[p], P[p], fr["t"])
                    Q[f], P[f] = joint(E, fr, A, lambda: R[p] if ident else qmat(E, A), Pt)
                else:  # emission order as before the prismatic support (same generated Panda code)
                    Q[f], _ = joint(E, fr, A, None, None)
                    if p not in R:
                        R[p] = qmat(E, Q[p])
                    P[f] = xform(E, R[p], P[p], fr["t"])
            R[f] = qmat(E, Q[f])
        return Q, P, R

    def center(self, E, R, P, frame, off):
        return xform(E, R[frame], P[frame], off)

    # ---------------------------------------------------------------------------------
    def gen_sphere_fk(self) -> str:
        E = Emitter()
        m = self.m
        dim = m["dimension"]
        Q, P, R = self.frames_fk(E)
        for s, sp in enumerate(m["spheres"]):
            c = self.center(E, R, P, sp["frame"], sp["offset"])
            for i, comp in enumerate("xyz"):
                b = ("bx", "by", "bz")[i]
                # world = base + C  (fk.hh: out.x[i] = base_x + EXPR)
                E.raw(f"out[({i} * {len(m['spheres'])} + {s}) * ld] = {b} + {c[i].expr()};")
        hdr = [
            f"// GENERATED by tools/gen_kernels.py from model/{self.name}.json -- do not edit.",
            f"// {E.flops} float ops (Horner sin/cos counted as 16 each).",
            f"{TY['qual']} void {self.name}_sphere_fk_store(",
            "    " + ", ".join(f"{TY['f']} q{i}" for i in range(dim)) + ",",
            f"    float bx, float by, float bz, {TY['f']}* __restrict__ out, size_t ld)",
            "{",
        ]
        return "\n".join(hdr + E.lines + ["}", ""])

    # ---------------------------------------------------------------------------------
    class Frames:
        """Lazily emitted frame poses (Q, P, R) and bounding centres over one Emitter."""

        def __init__(self, gen, E, qoff=0, qname="q"):
            self.g, self.E, self.qoff, self.qname = gen, E, qoff, qname
            self.Q, self.P, self.R, self.bc = {}, {}, {}, {}
            self.built = set()

        def frame(self, f):
            Q, P, E = self.Q, self.P, self.E
            if f in Q:
                return
            fr = self.g.m["frames"][f]
            qf = tuple(SV.const(v) for v in fr["qf"])
            if fr["parent"] < 0:
                Q[f] = qf
                P[f] = [SV.const(v) for v in fr["t"]]
                return
            p = fr["parent"]
            self.rot(p)
            ident = list(fr["qf"]) == [1.0, 0.0, 0.0, 0.0]
            A = Q[p] if ident else qmul(E, Q[p], qf)
            if fr.get("jtype") == "prismatic":
                Pt = xform(E, self.R[p], P[p], fr["t"])
                Q[f], P[f] = joint(E, fr, A, lambda: self.R[p] if ident else qmat(E, A), Pt, self.qoff, self.qname)
            else:
                Q[f], _ = joint(E, fr, A, None, None, self.qoff, self.qname)
                P[f] = xform(E, self.R[p], P[p], fr["t"])

        def rot(self, f):
            # REMAT: rotation matrices live only within one check (A/B: slower, kept off)
            self.frame(f)
            if f not in self.R:
                if f in self.built and REMAT:
                    self.R[f] = qmat(self.E, tuple(self.E.opaque(v) for v in self.Q[f]))
                else:
                    self.R[f] = qmat(self.E, self.Q[f])
                    self.built.add(f)

        def center(self, frame, off):
            self.rot(frame)
            return xform(self.E, self.R[frame], self.P[frame], off)

        def bound_center(self, b):
            if b not in self.bc:
                bd = self.g.m["bounding"][b]
                self.bc[b] = self.center(bd["frame"], bd["offset"])
            return self.bc[b]

    @staticmethod
    def world(c, base):
        if not base:
            return [x.expr() for x in c]
        return [f"({c[i].expr()} + {('bx', 'by', 'bz')[i]})" if c[i].kind != "zero" else ("bx", "by", "bz")[i]
                for i in range(3)]

    def bound_test(self, fr, o):
        """(kind, C expression) of the bounding test of check `o`: env -> bit pattern whose sign
        is this lane's hit; self -> bool of this lane."""
        m = self.m
        links = [b["link"] for b in m["bounding"]]
        if o["kind"] == "env":
            ck = m["env_checks"][o["index"]]
            b = links.index(ck["link"])
            bd = m["bounding"][b]
            w = self.world(fr.bound_center(b), bd["base"])
            if ck["link"] in getattr(self, "cluster_on", ()):
                return "env", f"env_bits_e<Grp, EXT>(env, nsE, {w[0]}, {w[1]}, {w[2]}, {flit(bd['radius'])})", ck
            return "env", f"env_bits<Grp, EXT>(env, {w[0]}, {w[1]}, {w[2]}, {flit(bd['radius'])})", ck
        ck = m["self_checks"][o["index"]]
        (ca, ra), (cb, rb) = self.self_ent(fr, ck["a"]), self.self_ent(fr, ck["b"])
        return "self", (f"self_lane({ca[0].expr()}, {ca[1].expr()}, {ca[2].expr()}, {flit(ra)}, "
                        f"{cb[0].expr()}, {cb[1].expr()}, {cb[2].expr()}, {flit(rb)})"), ck

    def self_ent(self, fr, e):
        m = self.m
        if "sphere" in e:
            sp = m["spheres"][e["sphere"]]
            return fr.center(sp["frame"], sp["offset"]), sp["radius"]
        links = [b["link"] for b in m["bounding"]]
        bi = links.index(e["bound"])
        return fr.bound_center(bi), m["bounding"][bi]["radius"]

    def emit_children(self, E, fr, kind, ck, on_hit, early=False, near_ok=False, near_gate="true"):
        """Children of a fired check; `on_hit` is the statement run when any lane's child fires.
        early: environment children leave as soon as one fires for the group (a group whose
        answer is known stops; the wave stops when all its groups have); "primitive": only in
        instantiations without point clouds (EXT false)."""
        spheres = self.m["spheres"]
        if kind == "env":
            E.raw(bdecl("h", "sign bit: this lane hit (a hit lane keeps no obstacle loop alive)"))
            kids = ck["children"]
            frames = {spheres[k["sphere"]]["frame"] for k in kids}
            bases = {k["base"] for k in kids}
            near = near_ok and NEAR and not TY["cpu"] and len(frames) == 1 and len(bases) == 1 and len(kids) > 1

            def kid_scans(use_near):
                for i, kid in enumerate(kids):
                    sp = spheres[kid["sphere"]]
                    cw = self.world(fr.center(sp["frame"], sp["offset"]), kid["base"])
                    if use_near:
                        E.raw(f"h = env_bits_near<Grp>(env, ns, {cw[0]}, {cw[1]}, {cw[2]}, {flit(sp['radius'])}, h);")
                    else:
                        E.raw(f"h = env_bits<Grp, EXT>(env, {cw[0]}, {cw[1]}, {cw[2]}, {flit(sp['radius'])}, h);")
                    if early == "primitive" and i + 1 < len(kids):  # staged: point-cloud queries may be deferred
                        E.raw(f"if constexpr (!EXT) {{ if (Grp::any_bits(h)) {on_hit} }}")
                    elif early and i + 1 < len(kids):
                        E.raw(f"if (Grp::any_bits(h)) {on_hit}")

            if near:  # S: one sphere enclosing every child (env_near / env_bits_near); centres per branch
                (off, R), = mid_spheres([spheres[k["sphere"]]["offset"] for k in kids],
                                        [spheres[k["sphere"]]["radius"] for k in kids], 1)
                E.raw(f"if (!EXT && {near_gate} && env.near_ok) {{  // primitive records only, at most kNearMax")
                E.indent += 1
                w = self.world(fr.center(next(iter(frames)), off), next(iter(bases)))
                E.raw(f"const NearSet ns = env_near<Grp>(env, {w[0]}, {w[1]}, {w[2]}, {flit(R)});  "
                      f"// the records the {len(kids)} children can touch")
                kid_scans(True)
                E.indent -= 1
                E.raw("} else {")
                E.indent += 1
                kid_scans(False)
                E.indent -= 1
                E.raw("}")
            else:
                kid_scans(False)
            E.raw(f"if (Grp::any_bits(h)) {on_hit}")
            return
        pairs = ck["children"]
        drop = set(ck.get("unreachable", []))
        if not drop:
            self.emit_self_pairs(E, fr, pairs, on_hit)
            return
        # pairs that cannot fire while the joints between the two links stay inside the analysed
        # range (tools/prune_pairs.py) are skipped for groups entirely inside it
        lo, hi = self.m["reach_lo"], self.m["reach_hi"]
        inside = " && ".join(f"q{d} >= {flit(lo[d])} && q{d} <= {flit(hi[d])}" for d in ck["reach_dofs"])
        E.raw(f"if (Grp::any(!({inside}))) {{  // some lane outside the analysed joint range: all pairs")
        E.indent += 1
        self.emit_self_pairs(E, fr, pairs, on_hit)
        E.indent -= 1
        E.raw(f"}} else {{  // {len(pairs) - len(drop)} of {len(pairs)} pairs can fire")
        E.indent += 1
        self.emit_self_pairs(E, fr, [p for i, p in enumerate(pairs) if i not in drop], on_hit)
        E.indent -= 1
        E.raw("}")

    def emit_self_pairs(self, E, fr, pairs, on_hit):
        if not TY["cpu"] and HOLD:
            return self.emit_self_pairs_held(E, fr, pairs, on_hit)
        spheres = self.m["spheres"]
        E.raw("{")
        E.indent += 1
        E.raw(bdecl("h", "OR of the children's test-value bits: sign bit = any child fired"))
        # Child pairs in chunks of CH distinct b-spheres: the chunk's b centres stay in
        # registers while each a-sphere centre is recomputed per chunk (bounded live set;
        # the OR is order-independent).
        CH = 6
        bs = sorted(set(p[1] for p in pairs))
        nchunks = (len(bs) + CH - 1) // CH
        for ci in range(nchunks):
            chunk = bs[ci * CH:(ci + 1) * CH]
            E.raw("{")
            E.indent += 1
            bcen = {sb: fr.center(spheres[sb]["frame"], spheres[sb]["offset"]) for sb in chunk}
            for sa in sorted(set(p[0] for p in pairs if p[1] in bcen)):
                a_ = fr.center(spheres[sa]["frame"], spheres[sa]["offset"])
                for sb in chunk:
                    if [sa, sb] not in pairs:
                        continue
                    b_ = bcen[sb]
                    E.raw(f"h |= self_bits({a_[0].expr()}, {a_[1].expr()}, {a_[2].expr()}, "
                          f"{flit(spheres[sa]['radius'])}, {b_[0].expr()}, {b_[1].expr()}, {b_[2].expr()}, "
                          f"{flit(spheres[sb]['radius'])});")
            E.indent -= 1
            E.raw("}")
            if ci + 1 < nchunks:
                E.raw(f"if (Grp::any_bits(h)) {on_hit}  // early exit (work only)")
        E.raw(f"if (Grp::any_bits(h)) {on_hit}")
        E.indent -= 1
        E.raw("}")

    def emit_self_pairs_held(self, E, fr, pairs, on_hit):
        """GPU form: the centres of the side with fewer distinct spheres are computed once and held;
        the other side's spheres are streamed one at a time (each centre lives only for its own tests),
        so the live set is |held| x 3 + one frame + a centre -- not both sides.  Same expressions,
        same bits; the OR is order-independent.  Early exit every CH streamed spheres."""
        spheres = self.m["spheres"]
        CH = 6
        sa = sorted(set(p[0] for p in pairs))
        sb = sorted(set(p[1] for p in pairs))
        hold_a = len(sa) <= len(sb)
        held, stream = (sa, sb) if hold_a else (sb, sa)
        pset = set((p[0], p[1]) for p in pairs)
        E.raw("{")
        E.indent += 1
        E.raw(bdecl("h", "OR of the children's test-value bits: sign bit = any child fired"))
        hc = {x: fr.center(spheres[x]["frame"], spheres[x]["offset"]) for x in held}
        for ci in range(0, len(stream), CH):
            E.raw("{")
            E.indent += 1
            for y in stream[ci:ci + CH]:
                c = fr.center(spheres[y]["frame"], spheres[y]["offset"])
                for x in held:
                    a, b = (x, y) if hold_a else (y, x)
                    if (a, b) not in pset:
                        continue
                    ca, cb = (hc[x], c) if hold_a else (c, hc[x])
                    E.raw(f"h |= self_bits({ca[0].expr()}, {ca[1].expr()}, {ca[2].expr()}, "
                          f"{flit(spheres[a]['radius'])}, {cb[0].expr()}, {cb[1].expr()}, {cb[2].expr()}, "
                          f"{flit(spheres[b]['radius'])});")
            E.indent -= 1
            E.raw("}")
            if ci + CH < len(stream):
                E.raw(f"if (Grp::any_bits(h)) {on_hit}  // early exit (work only)")
        E.raw(f"if (Grp::any_bits(h)) {on_hit}")
        E.indent -= 1
        E.raw("}")

    def gen_pair_inter(self) -> str:
        """Inter-robot check of a two-arm composite of this robot (BASELINE configs[4]; the C
        restatement is oracle/vamp_oracle.c pair_inter_collide): arm A = q0..q(d-1) at base
        (ax, ay, az), arm B = q(d)..q(2d-1) at base (bx, by, bz).  Every link-bounding pair in
        link order (world frame: both bases applied to every sphere); when a pair overlaps for
        any lane of the group, the two links' sphere pairs (frames recomputed inside the block,
        so only the 2 x 33 bounding centres stay live across the 121 tests).  Returns true on
        a collision."""
        m = self.m
        dim = m["dimension"]
        E = Emitter()
        fa, fb = self.Frames(self, E, 0), self.Frames(self, E, dim)
        nb = len(m["bounding"])

        def wc(c, pre):
            return [E.add(c[i], SV("var", name=f"{pre}{'xyz'[i]}")) for i in range(3)]

        bca = [wc(fa.bound_center(b), "a") for b in range(nb)]
        bcb = [wc(fb.bound_center(b), "b") for b in range(nb)]
        spheres = m["spheres"]
        links = [b["link"] for b in m["bounding"]]
        if TY["cpu"]:
            # CPU: every sphere centre of both arms once, up front (the same op sequence per centre
            # as the per-block recomputation below, so the same bits), then the tests -- one
            # straight-line function a host compiler handles (the GPU form recomputes frames per
            # fired pair to keep its register live set small)
            cas = {i: wc(fa.center(sp["frame"], sp["offset"]), "a") for i, sp in enumerate(spheres)}
            cbs = {j: wc(fb.center(sp["frame"], sp["offset"]), "b") for j, sp in enumerate(spheres)}
        for la in range(nb):
            for lb in range(nb):
                if not TY["cpu"]:
                    break
                ra, rb = m["bounding"][la]["radius"], m["bounding"][lb]["radius"]
                A_, B_ = bca[la], bcb[lb]
                E.raw(f"// {links[la]} (A) vs {links[lb]} (B)")
                E.raw(f"if (Grp::any(self_lane({A_[0].expr()}, {A_[1].expr()}, {A_[2].expr()}, {flit(ra)}, "
                      f"{B_[0].expr()}, {B_[1].expr()}, {B_[2].expr()}, {flit(rb)}))) {{")
                E.indent += 1
                E.raw(bdecl("h"))
                for i in [i for i, sp in enumerate(spheres) if sp["link"] == links[la]]:
                    for j in [j for j, sp in enumerate(spheres) if sp["link"] == links[lb]]:
                        ca, cb = cas[i], cbs[j]
                        E.raw(f"h |= self_bits({ca[0].expr()}, {ca[1].expr()}, {ca[2].expr()}, "
                              f"{flit(spheres[i]['radius'])}, {cb[0].expr()}, {cb[1].expr()}, "
                              f"{cb[2].expr()}, {flit(spheres[j]['radius'])});")
                E.raw("if (Grp::any_bits(h)) return true;")
                E.indent -= 1
                E.raw("}")
            if TY["cpu"]:
                continue
        for la in range(nb):
            for lb in range(nb):
                if TY["cpu"]:
                    break
                ra, rb = m["bounding"][la]["radius"], m["bounding"][lb]["radius"]
                A_, B_ = bca[la], bcb[lb]
                E.raw(f"// {links[la]} (A) vs {links[lb]} (B)")
                E.raw(f"if (Grp::any(self_lane({A_[0].expr()}, {A_[1].expr()}, {A_[2].expr()}, {flit(ra)}, "
                      f"{B_[0].expr()}, {B_[1].expr()}, {B_[2].expr()}, {flit(rb)}))) {{")
                E.indent += 1
                ga, gb = self.Frames(self, E, 0), self.Frames(self, E, dim)
                sa_ = [i for i, sp in enumerate(spheres) if sp["link"] == links[la]]
                sb_ = [i for i, sp in enumerate(spheres) if sp["link"] == links[lb]]
                E.raw(bdecl("h"))
                cb = {j: wc(gb.center(spheres[j]["frame"], spheres[j]["offset"]), "b") for j in sb_}
                for i in sa_:
                    ca = wc(ga.center(spheres[i]["frame"], spheres[i]["offset"]), "a")
                    for j in sb_:
                        E.raw(f"h |= self_bits({ca[0].expr()}, {ca[1].expr()}, {ca[2].expr()}, "
                              f"{flit(spheres[i]['radius'])}, {cb[j][0].expr()}, {cb[j][1].expr()}, "
                              f"{cb[j][2].expr()}, {flit(spheres[j]['radius'])});")
                E.raw("if (Grp::any_bits(h)) return true;")
                E.indent -= 1
                E.raw("}")
        E.raw("return false;")
        args = ", ".join(f"{TY['f']} q{i}" for i in range(2 * dim))
        hdr = [f"// GENERATED by tools/gen_kernels.py from model/{self.name}.json -- do not edit.",
               "// Two-arm composite: inter-robot sphere check, bounding-first.",
               "template <class Grp>",
               f"{TY['qual']} bool {self.name}_pair_inter(",
               f"    {args},",
               "    float ax, float ay, float az, float bx, float by, float bz)",
               "{"]
        return "\n".join(hdr + E.lines + ["}", ""])

    def load_gate(self):
        """model/<robot>_pair_gate.json (tools/make_pair_gate.py), used by the GPU staged bound stage;
        None without one (or for the CPU restatement, which evaluates every check)."""
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "model", f"{self.name}_pair_gate.json")
        if TY["cpu"] or not GATE or not os.path.exists(path):
            return None
        return json.load(open(path))

    def gate_function(self, gate):
        n0, n1 = gate["n"]
        lo0, lo1 = gate["lo"]
        h0, h1 = gate["h"]
        allmask = (1 << len(gate["checks"])) - 1
        vals = ", ".join(str(v) for v in gate["gate"])
        return [f"// (q_{gate['dofs'][0]}, q_{gate['dofs'][1]}) gate of checks {gate['checks']}: bit k set when check",
                f"// checks[k] can fire somewhere in the cell (tools/make_pair_gate.py, margin {gate['margin']} m);",
                "// outside the table (or NaN) every check is allowed",
                f"static __device__ const uint8_t {self.name}_gate_table[{n0 * n1}] = {{{vals}}};",
                f"__device__ __forceinline__ uint32_t {self.name}_gate(float a, float b)",
                "{",
                f"    const float fa = (a - {flit(lo0)}) * {flit(1.0 / h0)};",
                f"    const float fb = (b - {flit(lo1)}) * {flit(1.0 / h1)};",
                f"    if (!(fa >= 0.0f && fa < {flit(n0)} && fb >= 0.0f && fb < {flit(n1)})) return {allmask}u;",
                f"    return {self.name}_gate_table[(int)fa * {n1} + (int)fb];",
                "}", ""]

    def gen_pair_staged(self, chunk=64) -> str:
        """Staged form of the composite's inter-arm check (vgpu_staged.hh; BASELINE configs[4]): check
        c = link-bounding pair (la, lb) in the same link-major order as gen_pair_inter, split into
        chunks of <= 64 checks, one bound function per chunk (u64 mask of the chunk's bounding tests
        that fire for the group) and one children function over all checks (check c's sphere pairs,
        both links' frames recomputed, the arm with the fewer spheres held).  valid == no check whose
        bounding test and one of its children fire: the monolithic gen_pair_inter's OR, staged."""
        m = self.m
        dim = m["dimension"]
        nb = len(m["bounding"])
        spheres = m["spheres"]
        links = [b["link"] for b in m["bounding"]]
        checks = [(la, lb) for la in range(nb) for lb in range(nb)]
        args = ", ".join(f"{TY['f']} q{i}" for i in range(2 * dim))
        base_args = "float ax, float ay, float az, float bx, float by, float bz"

        def wc(E, c, pre):
            return [E.add(c[i], SV("var", name=f"{pre}{'xyz'[i]}")) for i in range(3)]

        out = [f"// GENERATED by tools/gen_kernels.py --pair-staged from model/{self.name}.json -- do not edit.",
               f"constexpr int {self.name}_pair_n_checks = {len(checks)};",
               f"constexpr int {self.name}_pair_chunk = {chunk};"]
        for k in range(0, len(checks), chunk):
            E = Emitter()
            fa, fb = self.Frames(self, E, 0), self.Frames(self, E, dim)
            bca, bcb = {}, {}
            E.raw("uint64_t mask = 0u;")
            for c in range(k, min(k + chunk, len(checks))):
                la, lb = checks[c]
                if la not in bca:
                    bca[la] = wc(E, fa.bound_center(la), "a")
                if lb not in bcb:
                    bcb[lb] = wc(E, fb.bound_center(lb), "b")
                A_, B_ = bca[la], bcb[lb]
                ra, rb = m["bounding"][la]["radius"], m["bounding"][lb]["radius"]
                E.raw(f"if (Grp::any(self_lane({A_[0].expr()}, {A_[1].expr()}, {A_[2].expr()}, {flit(ra)}, "
                      f"{B_[0].expr()}, {B_[1].expr()}, {B_[2].expr()}, {flit(rb)}))) mask |= 1ull << {c - k};"
                      f"  // {links[la]} (A) vs {links[lb]} (B)")
            E.raw("return mask;")
            out += ["template <class Grp>",
                    f"{TY['qual']} uint64_t {self.name}_pair_bound_mask_{k // chunk}(",
                    f"    {args},", f"    {base_args})", "{"] + E.lines + ["}", ""]
        # every chunk's bounding tests in ONE pass (vgpu_pair_staged.hip PairInterR<0>::bound_both): arm A's link
        # centres first, then arm B's links one at a time, each tested against all of A's -- both arms' FK once
        # instead of once per chunk, and only A's centres held.  Bit c of the group's mask = some lane's test fires
        # (Grp::any of each test, as in the chunked functions, taken as one OR over the group at the end)
        E = Emitter()
        fa, fb = self.Frames(self, E, 0), self.Frames(self, E, dim)
        nck = len(checks)
        E.raw("uint64_t mask[2] = {0u, 0u};")
        bca = {la: wc(E, fa.bound_center(la), "a") for la in range(nb)}
        for lb in range(nb):
            B_ = wc(E, fb.bound_center(lb), "b")
            rb = m["bounding"][lb]["radius"]
            for la in range(nb):
                c = la * nb + lb
                A_, ra = bca[la], m["bounding"][la]["radius"]
                E.raw(f"mask[{c // chunk}] |= (uint64_t)self_lane({A_[0].expr()}, {A_[1].expr()}, {A_[2].expr()}, "
                      f"{flit(ra)}, {B_[0].expr()}, {B_[1].expr()}, {B_[2].expr()}, {flit(rb)}) << {c % chunk};"
                      f"  // {links[la]} (A) vs {links[lb]} (B)")
        # per-lane bits, OR-ed over the group once at the end (not one group reduction per test)
        E.raw("m1 = vgpu::group_or64<Grp>(mask[1]);")
        E.raw("return vgpu::group_or64<Grp>(mask[0]);")
        assert nck <= 2 * chunk
        out += ["template <class Grp>",
                f"{TY['qual']} uint64_t {self.name}_pair_bound_both(",
                f"    {args},", f"    {base_args}, uint64_t& m1)", "{"] + E.lines + ["}", ""]
        body = []
        for c, (la, lb) in enumerate(checks):
            E = Emitter()
            E.indent = 2
            ga, gb = self.Frames(self, E, 0), self.Frames(self, E, dim)
            sa_ = [i for i, sp in enumerate(spheres) if sp["link"] == links[la]]
            sb_ = [j for j, sp in enumerate(spheres) if sp["link"] == links[lb]]
            for i in sa_:
                ga.rot(spheres[i]["frame"])
            for j in sb_:
                gb.rot(spheres[j]["frame"])
            hold_a = len(sa_) <= len(sb_)
            held, stream = (sa_, sb_) if hold_a else (sb_, sa_)
            gh, gs = (ga, gb) if hold_a else (gb, ga)
            ph, ps = ("a", "b") if hold_a else ("b", "a")
            E.raw(bdecl("h"))
            hc = {x: wc(E, gh.center(spheres[x]["frame"], spheres[x]["offset"]), ph) for x in held}
            CH = 6
            for ci in range(0, len(stream), CH):
                E.raw("{")
                E.indent += 1
                for y in stream[ci:ci + CH]:
                    cy = wc(E, gs.center(spheres[y]["frame"], spheres[y]["offset"]), ps)
                    for x in held:
                        (i, ci_), (j, cj_) = ((x, hc[x]), (y, cy)) if hold_a else ((y, cy), (x, hc[x]))
                        E.raw(f"h |= self_bits({ci_[0].expr()}, {ci_[1].expr()}, {ci_[2].expr()}, "
                              f"{flit(spheres[i]['radius'])}, {cj_[0].expr()}, {cj_[1].expr()}, {cj_[2].expr()}, "
                              f"{flit(spheres[j]['radius'])});")
                E.indent -= 1
                E.raw("}")
                if ci + CH < len(stream):
                    E.raw("if (Grp::any_bits(h)) return true;  // early exit (work only)")
            E.raw("return Grp::any_bits(h);")
            body += [f"    case {c}: {{  // {links[la]} (A) vs {links[lb]} (B): {len(sa_)} x {len(sb_)} sphere pairs"]
            body += E.lines + ["    }"]
        out += ["template <class Grp>",
                f"{TY['qual']} bool {self.name}_pair_children(int check,",
                f"    {args},", f"    {base_args})", "{", "    switch (check) {"] + body + \
               ["    default:", "        return false;", "    }", "}", ""]
        return "\n".join(out)

    def signature(self, ret, fname, extra="", mid=False):
        dim = self.m["dimension"]
        return [f"template <class Grp, bool EXT, bool MID = false>" if mid else f"template <class Grp, bool EXT>",
                f"{TY['qual']} {ret} {self.name}_{fname}(",
                f"    {extra}" + ", ".join(f"{TY['f']} q{i}" for i in range(dim)) + ",",
                "    const EnvView& env, float bx, float by, float bz)",
                "{"]

    def gen_fkcc(self, order=None, fname="fkcc", note=None, early=False) -> str:
        """Monolithic fkcc: FK emitted lazily in check order; per check the bounding test, and
        the children only when any lane of the group fires (Grp::any), early return.  `order`: a
        subset of the checks (the staged lead pass, `fname` "lead")."""
        E = Emitter()
        fr = self.Frames(self, E)
        m = self.m
        posed = False
        for o in (m["check_order"] if order is None else order):
            if REMAT:
                fr.R.clear()
            if o["kind"] in ("att", "attenv"):
                if not posed:  # Attachment::pose at the end-effector frame (set_attachment_pose)
                    f = m["ee_frame"]
                    fr.frame(f)
                    Qe, Pe = fr.Q[f], fr.P[f]
                    E.raw(f"const AttPose ap = att_pose(env, {Pe[0].expr()}, {Pe[1].expr()}, {Pe[2].expr()}, "
                          f"{Qe[1].expr()}, {Qe[2].expr()}, {Qe[3].expr()}, {Qe[0].expr()});")
                    posed = True
                self.emit_att_check(E, fr, o)
                continue
            if o["kind"] == "env":  # children frames first (short bounding->children gap)
                for kid in m["env_checks"][o["index"]]["children"]:
                    fr.rot(m["spheres"][kid["sphere"]]["frame"])
            else:
                for sa, sb in m["self_checks"][o["index"]]["children"]:
                    fr.rot(m["spheres"][sa]["frame"])
                    fr.rot(m["spheres"][sb]["frame"])
            kind, test, ck = self.bound_test(fr, o)
            label = ck["link"] if kind == "env" else " vs ".join(ck["links"])
            E.raw(f"// {kind}: {label} ({len(ck['children'])} children)")
            if kind == "env" and ck.get("leaf"):  # single-sphere link: its own hit is the collision
                E.raw(f"if (Grp::any_bits({test})) return false;")
                continue
            if kind == "env":
                E.raw(f"if (Grp::any_bits({test})) {{")
            else:
                E.raw(f"if (Grp::any({test})) {{")
            E.indent += 1
            self.emit_children(E, fr, kind, ck, "return false;", early, near_ok=(fname == "lead"))
            E.indent -= 1
            E.raw("}")
        E.raw("return true;")
        hdr = [f"// GENERATED by tools/gen_kernels.py from model/{self.name}.json -- do not edit.",
               "// Monolithic fkcc: checks follow the reference hierarchy (link-bounding sphere first,",
               "// children only when the group's bounding test fires)."] if note is None else note
        hdr = hdr + self.signature("bool", fname)
        return "\n".join(hdr + E.lines + ["}", ""])

    def emit_att_check(self, E, fr, o):
        """Checks of the attached spheres (interleaved_sphere_fk_attachment only), robot frame:
        "attenv" = every posed sphere vs the environment (validity.hh:251-266); "att" = the
        link's entity (its bounding sphere, or its single sphere) vs every posed sphere, then
        -- unless a leaf -- the link's spheres vs every posed sphere (validity.hh:269-293)."""
        m = self.m
        if o["kind"] == "attenv":
            E.raw("{  // attachment vs environment")
            E.raw("    " + bdecl("h"))
            E.raw("    for (int k = 0; k < env.n_att; ++k) {")
            E.raw("        " + xyzr_decl())
            E.raw("        att_sphere(env, ap, k, X, Y, Z, R);")
            E.raw("        h = env_bits<Grp, EXT>(env, X, Y, Z, R, h);")
            E.raw("    }")
            E.raw("    if (Grp::any_bits(h)) return false;")
            E.raw("}")
            return
        ck = m["att_checks"][o["index"]]
        c, r = self.self_ent(fr, ck["ent"])
        E.raw(f"{{  // attachment vs {ck['link']} ({len(ck['children'])} children)")
        E.indent += 1
        E.raw(bdecl("h"))
        E.raw("for (int k = 0; k < env.n_att; ++k) {")
        E.raw("    " + xyzr_decl())
        E.raw("    att_sphere(env, ap, k, X, Y, Z, R);")
        E.raw(f"    h |= self_bits({c[0].expr()}, {c[1].expr()}, {c[2].expr()}, {flit(r)}, X, Y, Z, R);")
        E.raw("}")
        if ck.get("leaf"):
            E.raw("if (Grp::any_bits(h)) return false;")
        else:
            E.raw("if (Grp::any_bits(h)) {")
            E.indent += 1
            E.raw(bdecl("hc"))
            spheres = m["spheres"]
            for sidx in ck["children"]:
                sp = spheres[sidx]
                cs = fr.center(sp["frame"], sp["offset"])
                E.raw("for (int k = 0; k < env.n_att; ++k) {")
                E.raw("    " + xyzr_decl())
                E.raw("    att_sphere(env, ap, k, X, Y, Z, R);")
                E.raw(f"    hc |= self_bits({cs[0].expr()}, {cs[1].expr()}, {cs[2].expr()}, {flit(sp['radius'])}, "
                      "X, Y, Z, R);")
                E.raw("}")
            E.raw("if (Grp::any_bits(hc)) return false;")
            E.indent -= 1
            E.raw("}")
        E.indent -= 1
        E.raw("}")

    def gen_staged(self) -> str:
        """Staged fkcc (same result, see DESIGN.md "Staged checks"):
        <robot>_bound_mask  FK + every bounding test, bit c set when check c's bounding test
                            fires for the group (no children, no early exit);
        <robot>_children    check c's children for one group (recomputing the frames it needs);
                            true when any child fires.
        valid == no check whose bounding test AND some child fire -- the reference's hierarchy
        evaluated check by check instead of in one divergent pass."""
        m = self.m
        order = m["check_order"]
        if len(order) > 64:
            return self.gen_staged_chunked()
        wide = len(order) > 32
        mt, one = ("uint64_t", "1ull") if wide else ("uint32_t", "1u")
        E = Emitter()
        fr = self.Frames(self, E)
        E.raw(f"{mt} mask = 0u;")
        if LANE_BITS:
            E.raw(f"{mt} lm = 0u;  // per-lane test bits, OR-ed over the group at the end")
        gate = self.load_gate()
        gated = {}
        if gate is not None:  # the wrist self checks' (q_a, q_b) gate table (tools/make_pair_gate.py)
            d0, d1 = gate["dofs"]
            E.raw(f"const uint32_t gate = Grp::or_bits({self.name}_gate(q{d0}, q{d1}));  // per group: checks that can fire")
            gated = {c: b for b, c in enumerate(gate["checks"])}
        members = CLUSTER.get(self.name, [])
        first = min([c for c, o in enumerate(order) if o["kind"] == "env" and
                     m["env_checks"][o["index"]]["link"] in members], default=-1)
        in_cluster = {c for c, o in enumerate(order) if o["kind"] == "env" and
                      m["env_checks"][o["index"]]["link"] in members}
        for c, o in enumerate(order):
            if c == first:  # E, then every member's bounding test at once (short live ranges of E and the centres)
                self.emit_cluster(E, fr, members)
                self.cluster_on = set(members)
                for cm in sorted(in_cluster):
                    self.emit_bound_check(E, fr, cm, order[cm], gated, one, mids_on=bool(MIDS), mt=mt)
                self.cluster_on = set()
            if c in in_cluster:
                continue
            self.emit_bound_check(E, fr, c, o, gated, one, mids_on=bool(MIDS), mt=mt)
        if LANE_BITS:
            E.raw(f"return mask | {self.group_or(mt, 'lm')};")
        else:
            E.raw("return mask;")
        env_bits = sum(1 << c for c, o in enumerate(order) if o["kind"] == "env")
        out = [f"// GENERATED by tools/gen_kernels.py from model/{self.name}.json -- do not edit.",
               f"constexpr int {self.name}_n_checks = {len(order)};",
               f"using {self.name}_mask_t = {mt};",
               f"constexpr {mt} {self.name}_env_check_bits = {env_bits:#x}{'ull' if wide else 'u'};  // environment checks"]
        if gate is not None:
            out += self.gate_function(gate)
        out += self.signature(mt, "bound_mask", mid=bool(MIDS)) + E.lines + ["}", ""]
        out += self.staged_children(order)
        lead = [c for c, o in enumerate(order) if o["kind"] == "env" and
                m["env_checks"][o["index"]]["link"] == LEAD.get(self.name)]
        if lead:
            c = lead[0]
            out += ["", f"constexpr int {self.name}_lead_check = {c};",
                    self.gen_fkcc([order[c]], "lead",
                                  [f"// staged lead pass: check {c} ({LEAD[self.name]} vs the environment) alone, "
                                   "monolithic -- true when it passes; a group leaves at its first child hit"],
                                  early=True)]

        return "\n".join(out)

    def emit_cluster(self, E, fr, members):
        """E: centred on the members' mean bounding centre, radius = the largest centre distance + radius, widened
        for float rounding (and infinite for a NaN centre); its near set nsE (primitive environments with near sets)"""
        m = self.m
        links = [b["link"] for b in m["bounding"]]
        cs = []
        for link in members:
            b = links.index(link)
            bd = m["bounding"][b]
            cs.append((self.world(fr.bound_center(b), bd["base"]), bd["radius"]))
        k = len(cs)
        E.raw(f"// cluster {', '.join(members)}: one near set for their bounding tests")
        for a in range(3):
            E.raw(f"const float e{'xyz'[a]} = (" + " + ".join(c[a] for c, _ in cs) + f") * {flit(1.0 / k)};")
        E.raw("float eR = 0.0f, enan = 0.0f;")
        for c, r in cs:
            E.raw(f"{{ const float dx = {c[0]} - ex, dy = {c[1]} - ey, dz = {c[2]} - ez; "
                  f"const float dd = __builtin_sqrtf(dx * dx + dy * dy + dz * dz) + {flit(r)}; "
                  "eR = dd > eR ? dd : eR; enan += dd; }")
        E.raw("eR = (eR + 2e-5f) * 1.00001f;")
        E.raw("if (enan != enan || !(eR < __builtin_inff())) eR = __builtin_inff();")
        E.raw("const NearSet nsE = (!EXT && env.near_ok) ? env_near<Grp>(env, ex, ey, ez, eR) : NearSet{0ull, 0ull};")

    @staticmethod
    def group_or(mt, v):
        """OR of a per-lane check mask over the lane's group (Grp::or_bits on 32-bit halves)"""
        if mt == "uint32_t":
            return f"Grp::or_bits({v})"
        return f"(((uint64_t)Grp::or_bits((uint32_t)({v} >> 32)) << 32) | (uint64_t)Grp::or_bits((uint32_t){v}))"

    def emit_bound_check(self, E, fr, c, o, gated, one, mids_on, mt="uint32_t"):
        """check c's bounding test in the staged bound stage: bit c of mask set when it fires for the group"""
        kind, test, ck = self.bound_test(fr, o)
        mids = self.mids_of(ck, kind) if (mids_on and c not in gated) else None
        lane = LANE_BITS and not TY["cpu"]
        if mids:
            self.emit_mid_check(E, fr, kind, test, ck, mids, c, one)
        elif kind == "env" and lane:  # per lane: the sign bit of the check's env bits (8-lane groups)
            E.raw(f"if constexpr (Grp::G == 1) {{ if (Grp::any_bits({test[:-1]}, 0u, {c}))) mask |= {one} << {c}; }}")
            E.raw(f"else {{ lm |= ({mt})({test[:-1]}, 0u, {c}) >> 31) << {c}; }}")
        elif kind == "env":  # the check's bit is its deferred-query tag (vgpu_device.hh capt_defer_*)
            E.raw(f"if (Grp::any_bits({test[:-1]}, 0u, {c}))) mask |= {one} << {c};")
        elif c in gated and lane:
            E.raw(f"if constexpr (Grp::G == 1) {{ if (((gate >> {gated[c]}) & 1u) && Grp::any({test})) mask |= {one} << {c}; }}")
            E.raw(f"else {{ if ((gate >> {gated[c]}) & 1u) lm |= ({mt})({test}) << {c}; }}")
        elif c in gated:
            E.raw(f"if (((gate >> {gated[c]}) & 1u) && Grp::any({test})) mask |= {one} << {c};")
        elif kind == "self" and ck.get("never_fires") and not TY["cpu"]:
            # tools/prove_self_checks.py: no child pair can fire while these joints stay in the proven box;
            # a group with every lane inside it gets no bit (the bounding test is not even evaluated)
            def inward(v, up):  # the float32 bound on the box's side of v
                f = F(v)
                if (up and float(f) < v) or (not up and float(f) > v):
                    f = np.nextafter(f, F(np.inf) if up else F(-np.inf))
                return flit(f)
            inside = " && ".join(f"q{d} >= {inward(lo, True)} && q{d} <= {inward(hi, False)}"
                                 for d, lo, hi in zip(ck["never_dofs"], ck["never_lo"], ck["never_hi"]))
            if lane:
                E.raw(f"if constexpr (Grp::G == 1) {{ if (Grp::any(!({inside})) && Grp::any({test})) mask |= {one} << {c}; }}")
                E.raw(f"else {{ if (Grp::any(!({inside}))) lm |= ({mt})({test}) << {c}; }}  // proven silent inside")
            else:
                E.raw(f"if (Grp::any(!({inside})) && Grp::any({test})) mask |= {one} << {c};  // proven silent inside")
        elif lane:
            E.raw(f"if constexpr (Grp::G == 1) {{ if (Grp::any({test})) mask |= {one} << {c}; }}")
            E.raw(f"else {{ lm |= ({mt})({test}) << {c}; }}")
        else:
            E.raw(f"if (Grp::any({test})) mask |= {one} << {c};")

    def side_spheres(self, ck, side):
        """sphere indices of one side of a self check's child pairs"""
        return sorted(set(p[side] for p in ck["children"]))

    def mids_of(self, ck, kind):
        """the mid spheres of a check ((frame, base flag, [(offset, radius)]) per side), or None"""
        S = self.m["spheres"]
        if kind == "env":
            if ck.get("leaf") or ck["link"] not in MID_ENV:
                return None
            kids = [k["sphere"] for k in ck["children"]]
            frames = {S[i]["frame"] for i in kids}
            bases = {k["base"] for k in ck["children"]}
            if len(frames) != 1 or len(bases) != 1:
                return None
            ms = mid_spheres([S[i]["offset"] for i in kids], [S[i]["radius"] for i in kids], MID_ENV[ck["link"]])
            return [(frames.pop(), bases.pop(), ms)]
        if tuple(ck["links"]) not in MID_SELF_CHECKS or ck.get("unreachable"):
            return None
        sides = []
        for side in (0, 1):
            ids = self.side_spheres(ck, side)
            frames = {S[i]["frame"] for i in ids}
            if len(frames) != 1:
                return None
            ms = mid_spheres([S[i]["offset"] for i in ids], [S[i]["radius"] for i in ids],
                             MID_SELF_LINKS.get(ck["links"][side], 1))
            sides.append((frames.pop(), False, ms))
        return sides

    def emit_mid_check(self, E, fr, kind, test, ck, mids, c, one):
        """bound test, then (MID instantiations: non-EXT environments / every self test) the mid spheres'
        conservative tests"""
        if kind == "env":
            E.raw(f"if (Grp::any_bits({test[:-1]}, 0u, {c}))) {{")
        else:
            E.raw(f"if (Grp::any({test})) {{")
        E.indent += 1
        if kind == "env":
            E.raw(f"if constexpr (EXT || !MID) {{ mask |= {one} << {c}; }} else {{")
            E.indent += 1
            frame, base, ms = mids[0]
            E.raw(bdecl("hm", "sign bit: a mid sphere may touch an obstacle"))
            for off, R in ms:
                w = self.world(fr.center(frame, off), base)
                E.raw(f"hm = mid_env_bits<Grp>(env, {w[0]}, {w[1]}, {w[2]}, {flit(R)}, hm);")
            E.raw(f"if (Grp::any_bits(hm)) mask |= {one} << {c};")
            E.indent -= 1
            E.raw("}")
        else:
            (fa, _, ma), (fb, _, mb) = mids
            ca = [fr.center(fa, off) for off, _ in ma]
            cb = [fr.center(fb, off) for off, _ in mb]
            terms = []
            for (oa, ra), xa in zip(ma, ca):
                for (ob, rb), xb in zip(mb, cb):
                    terms.append(f"self_lane({xa[0].expr()}, {xa[1].expr()}, {xa[2].expr()}, {flit(ra)}, "
                                 f"{xb[0].expr()}, {xb[1].expr()}, {xb[2].expr()}, {flit(rb)})")
            E.raw(f"if constexpr (!MID) {{ mask |= {one} << {c}; }} else {{")
            E.indent += 1
            E.raw("uint32_t hm = 0u;  // some mid pair overlaps")
            for t in terms:
                E.raw(f"hm |= (uint32_t){t};")
            E.raw(f"if (Grp::any(hm != 0u)) mask |= {one} << {c};")
            E.indent -= 1
            E.raw("}")
        E.indent -= 1
        E.raw("}")

    def staged_children(self, order):
        """<robot>_children(check, q..., env, base): check c's children, frames recomputed"""
        m = self.m
        body = []
        if self.name in NEAR_CHILDREN:  # a TU may compile the near-set children out (vgpu_staged.hip part 0)
            body += ["#ifndef VGPU_NEAR_CHILDREN", "#define VGPU_NEAR_CHILDREN 1", "#endif"]
        for c, o in enumerate(order):
            E = Emitter()
            E.indent = 2
            fr = self.Frames(self, E)
            kind = o["kind"]
            ck = m["env_checks"][o["index"]] if kind == "env" else m["self_checks"][o["index"]]
            label = ck["link"] if kind == "env" else " vs ".join(ck["links"])
            if kind == "env" and ck.get("leaf"):  # the bounding hit itself is the collision
                body += [f"    case {c}: {{  // env: {label} (leaf)", "        return true;", "    }"]
                continue
            # frames first, outside the chunk scopes of emit_children
            if kind == "env":
                for kid in ck["children"]:
                    fr.rot(m["spheres"][kid["sphere"]]["frame"])
            else:
                for sa, sb in ck["children"]:
                    fr.rot(m["spheres"][sa]["frame"])
                    fr.rot(m["spheres"][sb]["frame"])
            self.emit_children(E, fr, kind, ck, "return true;", "primitive" if self.name in EARLY_CHILDREN else False,
                               near_ok=(kind == "env" and self.name in NEAR_CHILDREN and
                                        len(ck["children"]) >= NEAR_CHILDREN[self.name]),
                               near_gate="VGPU_NEAR_CHILDREN")
            body += [f"    case {c}: {{  // {kind}: {label} ({len(ck['children'])} children)"] + E.lines + \
                    ["        return false;", "    }"]
        out = self.signature("bool", "children", "int check, ")
        out += ["    switch (check) {"] + body + ["    default:", "        return false;", "    }", "}", ""]
        return out

    def gen_staged_chunked(self, chunk=64) -> str:
        """Staged form of a robot with more than 64 checks (the Baxter: 388): the check list in chunks
        of <= 64, one bound function per chunk (only the frames its checks need, a u64 mask of the
        chunk's bounding tests) -- each chunk a chained staged pass over the same groups
        (vgpu_baxter_staged.hip) -- and one children function over all checks."""
        m = self.m
        order = m["check_order"]
        name = self.name
        out = [f"// GENERATED by tools/gen_kernels.py from model/{name}.json -- do not edit.",
               f"constexpr int {name}_n_checks = {len(order)};",
               f"constexpr int {name}_chunk = {chunk};",
               f"constexpr int {name}_n_chunks = {(len(order) + chunk - 1) // chunk};"]
        envs = []
        for k in range(0, len(order), chunk):
            E = Emitter()
            fr = self.Frames(self, E)
            E.raw("uint64_t mask = 0u;")
            for c in range(k, min(k + chunk, len(order))):
                kind, test, ck = self.bound_test(fr, order[c])
                if kind == "env" and LANE_BITS:
                    E.raw(f"mask |= (uint64_t)({test[:-1]}, 0u, {c - k}) >> 31) << {c - k};")
                elif kind == "env":  # the check's bit in the chunk mask is its deferred-query tag
                    E.raw(f"if (Grp::any_bits({test[:-1]}, 0u, {c - k}))) mask |= 1ull << {c - k};")
                elif LANE_BITS:
                    E.raw(f"mask |= (uint64_t)({test}) << {c - k};")
                else:
                    E.raw(f"if (Grp::any({test})) mask |= 1ull << {c - k};")
            E.raw(f"return {self.group_or('uint64_t', 'mask')};" if LANE_BITS else "return mask;")
            out += self.signature("uint64_t", f"bound_mask_{k // chunk}") + E.lines + ["}", ""]
            envs.append(sum(1 << (c - k) for c in range(k, min(k + chunk, len(order)))
                            if order[c]["kind"] == "env"))
        out.append(f"constexpr uint64_t {name}_env_check_bits_chunk[{len(envs)}] = {{" +
                   ", ".join(f"{e:#x}ull" for e in envs) + "};")
        out += self.staged_children(order)
        return "\n".join(out)


def gen_radii(paths) -> str:
    """Host-and-device table of every robot's collision-sphere radii (reference order, the
    Spheres<rake>::r of Robot::sphere_fk): used where a kernel needs the radii next to
    sphere_fk's centres (filter_robot_from_pointcloud, bindings/common.hh:36-87)."""
    out = ["// GENERATED by tools/gen_kernels.py --radii from model/*.json -- do not edit.", "#pragma once", ""]
    for path in paths:
        m = json.load(open(path))
        vals = ", ".join(flit(sp["radius"]) for sp in m["spheres"])
        out.append(f"constexpr int {m['robot']}_n_spheres_table = {len(m['spheres'])};")
        out.append(f"constexpr float {m['robot']}_sphere_radii[{len(m['spheres'])}] = {{{vals}}};")
    return "\n".join(out) + "\n"


def main():
    global REMAT, TY, HOLD, GATE, MIDS, LANE_BITS, NEAR, CLUSTER
    if "--radii" in sys.argv:  # tools/gen_kernels.py --radii OUT model/a.json model/b.json ...
        args = [a for a in sys.argv[1:] if a != "--radii"]
        open(args[0], "w").write(gen_radii(args[1:]))
        print(f"wrote {args[0]}")
        return
    if "--no-remat" in sys.argv:
        REMAT = False
        sys.argv.remove("--no-remat")
    if "--cpu" in sys.argv:
        TY = TY_CPU
    if "--no-hold" in sys.argv:
        HOLD = False
        sys.argv.remove("--no-hold")
    if "--no-gate" in sys.argv:
        GATE = False
        sys.argv.remove("--no-gate")
    if "--no-lane-bits" in sys.argv:
        LANE_BITS = False
        sys.argv.remove("--no-lane-bits")
    if "--mids" in sys.argv:
        MIDS = True
        sys.argv.remove("--mids")
    if "--cluster" in sys.argv:
        CLUSTER = CLUSTER_LINKS
        sys.argv.remove("--cluster")
    if "--no-near" in sys.argv:
        NEAR = False
        sys.argv.remove("--no-near")
    argv = [a for a in sys.argv if not a.startswith("--")]
    sys.argv[1:3] = argv[1:3]
    model = json.load(open(sys.argv[1]))
    g = RobotGen(model)
    name = g.name
    consts = [f"// Robot::scale_configuration q * s_m + s_a (one fma per joint, pinned by ref_probe \"scale\")"]
    for key in ("s_m", "s_a"):
        vals = ", ".join(f"{float(np.float32(v)).hex()}f" for v in model[key])
        consts.append(f"__device__ constexpr float {name}_{key}[{len(model[key])}] = {{{vals}}};")
    out = "\n".join(consts) + "\n\n" + g.gen_sphere_fk() + "\n" + g.gen_fkcc()
    if TY["cpu"]:  # CPU restatement: scale constants, sphere_fk + monolithic fkcc (one rake block per call)
        vals = ", ".join(f"{float(np.float32(v)).hex()}f" for v in model["d_m"])
        consts.append(f"constexpr float {name}_d_m[{len(model['d_m'])}] = {{{vals}}};  // descale (q - s_a) * d_m")
        out = "\n".join(consts).replace("__device__ constexpr", "constexpr") + "\n\n" + g.gen_sphere_fk() + "\n" + g.gen_fkcc()
        if "att_checks" in model:
            out = g.gen_fkcc()
    elif "att_checks" in model:  # the attachment variant: its fkcc only (first rake block)
        out = g.gen_fkcc()
    else:  # check masks: 32-bit up to 32 checks, 64-bit up to 64, chunks of 64 beyond
        out += "\n" + g.gen_staged()
    if "--pair" in sys.argv:  # the composite's inter-robot check, as its own include
        out = g.gen_pair_inter()
    if "--pair-staged" in sys.argv:  # its staged form (vgpu_pair_staged.hip)
        out = g.gen_pair_staged()
    open(sys.argv[2], "w").write(out)
    print(f"wrote {sys.argv[2]} ({len(out.splitlines())} lines)")


if __name__ == "__main__":
    main()
