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
        self.lines.append("    " * self.indent + f"const float {name} = {expr};")
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
                d = fr["dof"]
                if d >= 0:
                    h = E.tmp(f"q{d} * 0.5f")
                    c = E.tmp(f"vamp_cos({h.name})")
                    s = E.tmp(f"vamp_sin({h.name})")
                    E.flops += 2 * 16
                    Q[f] = qmul(E, A, (c, SV.zero(), SV.zero(), s))
                else:
                    Q[f] = A
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
            f"__device__ __forceinline__ void {self.name}_sphere_fk_store(",
            "    " + ", ".join(f"float q{i}" for i in range(dim)) + ",",
            "    float bx, float by, float bz, float* __restrict__ out, size_t ld)",
            "{",
        ]
        return "\n".join(hdr + E.lines + ["}", ""])

    def gen_fkcc(self) -> str:
        """fkcc with lazily emitted frames (short live ranges -> fewer VGPRs) and the
        reference's group semantics per check: a bounding test fires for the group if any
        lane fires (Grp::any); the children's per-lane hits are OR-ed and reduced once, which
        equals the reference's per-child `return false` (any lane, any child)."""
        E = Emitter()
        m = self.m
        dim = m["dimension"]
        frames = m["frames"]
        spheres, bounding = m["spheres"], m["bounding"]
        links = [b["link"] for b in bounding]
        Q, P, R = {}, {}, {}

        def ensure_frame(f):
            if f in Q:
                return
            fr = frames[f]
            qf = tuple(SV.const(v) for v in fr["qf"])
            if fr["parent"] < 0:
                Q[f] = qf
                P[f] = [SV.const(v) for v in fr["t"]]
                return
            p = fr["parent"]
            ensure_R(p)
            ident = list(fr["qf"]) == [1.0, 0.0, 0.0, 0.0]
            A = Q[p] if ident else qmul(E, Q[p], qf)
            d = fr["dof"]
            if d >= 0:
                h = E.tmp(f"q{d} * 0.5f")
                c = E.tmp(f"vamp_cos({h.name})")
                sn = E.tmp(f"vamp_sin({h.name})")
                E.flops += 2 * 16
                Q[f] = qmul(E, A, (c, SV.zero(), SV.zero(), sn))
            else:
                Q[f] = A
            P[f] = xform(E, R[p], P[p], fr["t"])

        # Rotation matrices live only within one check: a frame needed again by a later check
        # keeps its quaternion (4 values) + origin (3) and rebuilds R (9) from an opaque copy
        # of the quaternion (bit-identical values, ~20 flops) instead of holding 12 registers
        # across the whole hierarchy.
        built = set()

        def ensure_R(f):
            ensure_frame(f)
            if f not in R:
                if f in built and REMAT:
                    R[f] = qmat(E, tuple(E.opaque(v) for v in Q[f]))
                else:
                    R[f] = qmat(E, Q[f])
                    built.add(f)

        bc = {}

        def bound_center(b):
            if b not in bc:
                ensure_R(bounding[b]["frame"])
                bc[b] = self.center(E, R, P, bounding[b]["frame"], bounding[b]["offset"])
            return bc[b]

        def world(c, base):
            if not base:
                return [x.expr() for x in c]
            return [f"({c[i].expr()} + {('bx', 'by', 'bz')[i]})" if c[i].kind != "zero" else ("bx", "by", "bz")[i]
                    for i in range(3)]

        for o in m["check_order"]:
            if REMAT:
                R.clear()
            if o["kind"] == "env":
                ck = m["env_checks"][o["index"]]
                b = links.index(ck["link"])
                bd = bounding[b]
                for kid in ck["children"]:
                    ensure_R(spheres[kid["sphere"]]["frame"])
                w = world(bound_center(b), bd["base"])
                E.raw(f"// env: {ck['link']} bounding sphere r={bd['radius']} (+{len(ck['children'])} children)")
                E.raw(f"if (Grp::any_bits(env_bits<Grp, EXT>(env, {w[0]}, {w[1]}, {w[2]}, {flit(bd['radius'])}))) {{")
                E.indent += 1
                E.raw("uint32_t h = 0u;  // sign bit: this lane hit (a hit lane keeps no obstacle loop alive)")
                for kid in ck["children"]:
                    sp = spheres[kid["sphere"]]
                    c = self.center(E, R, P, sp["frame"], sp["offset"])
                    cw = world(c, kid["base"])
                    E.raw(f"h = env_bits<Grp, EXT>(env, {cw[0]}, {cw[1]}, {cw[2]}, {flit(sp['radius'])}, h);")
                E.raw("if (Grp::any_bits(h)) return false;")
                E.indent -= 1
                E.raw("}")
            else:
                ck = m["self_checks"][o["index"]]

                def ent(e):
                    if "sphere" in e:
                        sp = spheres[e["sphere"]]
                        ensure_R(sp["frame"])
                        return self.center(E, R, P, sp["frame"], sp["offset"]), sp["radius"]
                    bi = links.index(e["bound"])
                    return bound_center(bi), bounding[bi]["radius"]

                for sa, sb in ck["children"]:
                    ensure_R(spheres[sa]["frame"])
                    ensure_R(spheres[sb]["frame"])
                (ca, ra), (cb, rb) = ent(ck["a"]), ent(ck["b"])
                E.raw(f"// self: {ck['links'][0]} vs {ck['links'][1]} ({len(ck['children'])} children)")
                E.raw(f"if (Grp::any(self_lane({ca[0].expr()}, {ca[1].expr()}, {ca[2].expr()}, {flit(ra)}, "
                      f"{cb[0].expr()}, {cb[1].expr()}, {cb[2].expr()}, {flit(rb)}))) {{")
                E.indent += 1
                E.raw("uint32_t h = 0u;  // OR of the children's test-value bits: sign bit = any child fired")
                # Evaluate the child pairs in chunks of CH distinct b-spheres: the chunk's b
                # centres stay in registers while each a-sphere centre is recomputed per chunk,
                # bounding the live set (the OR is order-independent).
                CH = 6
                pairs = ck["children"]
                bs = sorted(set(p[1] for p in pairs))
                nchunks = (len(bs) + CH - 1) // CH
                for ci in range(nchunks):
                    chunk = bs[ci * CH:(ci + 1) * CH]
                    E.raw("{")
                    E.indent += 1
                    bcen = {}
                    for sb in chunk:
                        sp = spheres[sb]
                        bcen[sb] = self.center(E, R, P, sp["frame"], sp["offset"])
                    for sa in sorted(set(p[0] for p in pairs if p[1] in bcen)):
                        sp = spheres[sa]
                        a_ = self.center(E, R, P, sp["frame"], sp["offset"])
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
                        E.raw("if (Grp::any_bits(h)) return false;  // early exit (work only)")
                E.raw("if (Grp::any_bits(h)) return false;")
                E.indent -= 1
                E.raw("}")
        E.raw("return true;")
        hdr = [
            f"// GENERATED by tools/gen_kernels.py from model/{self.name}.json -- do not edit.",
            "// FK emitted lazily in check order; checks follow the reference hierarchy",
            "// (link-bounding sphere first, children only when the group's bounding test fires).",
            "template <class Grp, bool EXT>",
            f"__device__ __forceinline__ bool {self.name}_fkcc(",
            "    " + ", ".join(f"float q{i}" for i in range(dim)) + ",",
            "    const EnvView& env, float bx, float by, float bz)",
            "{",
        ]
        return "\n".join(hdr + E.lines + ["}", ""])


def main():
    global REMAT
    if "--no-remat" in sys.argv:
        REMAT = False
        sys.argv.remove("--no-remat")
    model = json.load(open(sys.argv[1]))
    g = RobotGen(model)
    name = g.name
    consts = [f"// Robot::scale_configuration q * s_m + s_a (one fma per joint, pinned by ref_probe \"scale\")"]
    for key in ("s_m", "s_a"):
        vals = ", ".join(f"{float(np.float32(v)).hex()}f" for v in model[key])
        consts.append(f"__device__ constexpr float {name}_{key}[{len(model[key])}] = {{{vals}}};")
    out = "\n".join(consts) + "\n\n" + g.gen_sphere_fk() + "\n" + g.gen_fkcc()
    open(sys.argv[2], "w").write(out)
    print(f"wrote {sys.argv[2]} ({len(out.splitlines())} lines)")


if __name__ == "__main__":
    main()
