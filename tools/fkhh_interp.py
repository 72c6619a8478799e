"""Interpreter for the reference's *generated* forward-kinematics headers.

FIXTURE GENERATION / MODEL EXTRACTION ONLY -- runs in the build container (where
/root/reference exists), never on the GPU box, never imported by the product.

Why this exists
---------------
The reference hot path (``/root/reference/src/impl/vamp/robots/panda/fk.hh``) cannot be
compiled in this image: ``fk.hh`` includes ``collision/environment.hh`` -> ``shapes.hh`` ->
``<Eigen/Geometry>`` and ``capt.hh`` -> ``<pdqsort.h>``, neither of which is installed, and
the task forbids stand-in headers.  The generated FK is, however, a straight-line
expression DAG in a tiny C++ subset:

    auto NAME = A op B;   auto NAME = -A;   auto NAME = q[i];   auto NAME = A.sin();
    out.x[i] = expr;      if (sphere_environment_in_collision(environment, x, y, z, r)) { ... }
    if (sphere_sphere_self_collision<decltype(q[0])>(ax, ay, az, ar, bx, by, bz, br)) { ... }
    return false;         return true;

This module parses that text and evaluates it lane-vectorised with numpy, following the
C++ type rules of the reference's vector layer (vector/interface.hh:565-815): vector (op)
scalar broadcasts the scalar as float; scalar literals are ``double``; ``float base_x``.
Two numeric modes:

* ``ref32``  float32, with FloatVector::sin()/cos() evaluated exactly as the reference's
  release build computes them (Horner form with FMAs, pinned bit-exact against
  oracle/_ref/ref_probe built from the reference's own vector layer; see
  tests/test_ref_pin.py).  Everything else is evaluated in source order without
  contraction: the reference build contracts/reassociates FK arithmetic
  (-ffp-contract=fast -fassociative-math, cmake/CompilerSettings.cmake:12-15), which moves
  sphere centres by ~1e-7 relative -- inside the 1e-5 FK tolerance, and the reason the
  mask comparison is margin-filtered.
* ``exact64`` float64 with exact trig -- used only to *extract* the kinematic model
  (which frame each sphere rides on, the link-bounding spheres and the self-collision
  pair hierarchy) as data; no arithmetic of this mode ends up in the product.

The collision predicates used while evaluating ``interleaved_sphere_fk`` are restated in
numpy from collision/validity.hh:13-150 and sphere_*.hh (see ``EnvNP``).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

F32 = np.float32

# --------------------------------------------------------------------------------------
# tokenizer / parser
# --------------------------------------------------------------------------------------
_TOK = re.compile(
    r"\s+|//[^\n]*|/\*.*?\*/"
    r"|(?P<num>\d+\.\d*(?:[eE][-+]?\d+)?f?|\d+(?:[eE][-+]?\d+)?f?)"
    r"|(?P<id>[A-Za-z_][A-Za-z_0-9]*(?:::[A-Za-z_][A-Za-z_0-9]*)*)"
    r"|(?P<op>[-+*/(){}\[\],;.=<>&!])",
    re.S,
)


def tokenize(src: str) -> List[Tuple[str, str]]:
    out = []
    pos = 0
    while pos < len(src):
        m = _TOK.match(src, pos)
        if not m:
            raise SyntaxError(f"cannot tokenize near: {src[pos:pos + 40]!r}")
        pos = m.end()
        if m.lastgroup is None:
            continue
        out.append((m.lastgroup, m.group(m.lastgroup)))
    return out


def function_body(src: str, head_regex: str) -> str:
    """Return the text between the braces of the first function whose head matches."""
    m = re.search(head_regex, src)
    if not m:
        raise KeyError(head_regex)
    i = src.index("{", m.end())
    depth = 0
    for j in range(i, len(src)):
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                return src[i + 1:j]
    raise SyntaxError("unbalanced braces")


# AST node kinds (tuples):
#   ('num', text)  ('var', name)  ('q', idx)  ('neg', e)  ('bin', op, a, b)  ('call1', fn, e)
#   stmt: ('decl', name, e) ('out', field, idx, e) ('if', call, body) ('ret', bool) ('fdecl', name, e)
#   call: ('env', [x, y, z, r])  ('self', [ax..br])  ('att', [...])


class Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else ("eof", "")

    def take(self, val=None):
        tok = self.t[self.i]
        if val is not None and tok[1] != val:
            raise SyntaxError(f"expected {val!r} got {tok!r} at {self.i}")
        self.i += 1
        return tok

    def stmts(self):
        body = []
        while self.i < len(self.t) and self.peek()[1] != "}":
            body.append(self.stmt())
        return body

    def stmt(self):
        kind, v = self.peek()
        if v == "auto":
            self.take()
            name = self.take()[1]
            self.take("=")
            e = self.expr()
            self.take(";")
            return ("decl", name, e)
        if v == "float":
            self.take()
            name = self.take()[1]
            self.take("=")
            e = self.expr()
            self.take(";")
            return ("fdecl", name, e)
        if v == "out":
            self.take()
            self.take(".")
            fld = self.take()[1]
            self.take("[")
            idx = int(self.take()[1])
            self.take("]")
            self.take("=")
            e = self.expr()
            self.take(";")
            return ("out", fld, idx, e)
        if v == "if":
            self.take()
            self.take("(")
            call = self.call()
            self.take(")")
            self.take("{")
            body = self.stmts()
            self.take("}")
            return ("if", call, body)
        if v == "set_attachment_pose":  # set_attachment_pose(environment, tx, ty, tz, rx, ry, rz, rw);
            self.take()
            self.take("(")
            self.take("environment")
            args = []
            while self.peek()[1] == ",":
                self.take()
                args.append(self.expr())
            self.take(")")
            self.take(";")
            return ("setpose", args)
        if v == "return":
            self.take()
            b = self.take()[1]
            self.take(";")
            return ("ret", b == "true")
        if v == "q":  # in-place scale blocks: q[i] = ...
            raise SyntaxError("unsupported statement q[...] =")
        raise SyntaxError(f"unsupported statement starting {self.peek()} at {self.i}")

    def call(self):
        fn = self.take()[1]
        if fn == "attachment_environment_collision":  # (environment)
            self.take("(")
            self.take("environment")
            self.take(")")
            return ("attenv", [])
        if fn.startswith("sphere_sphere_self_collision") or fn.startswith("attachment_sphere_collision"):
            # template args: <decltype(q[0])>
            self.take("<")
            depth = 1
            while depth:
                v = self.take()[1]
                if v == "<":
                    depth += 1
                elif v == ">":
                    depth -= 1
        self.take("(")
        args = []
        if self.peek()[1] == "environment":
            self.take()
            self.take(",")
        while True:
            args.append(self.expr())
            if self.peek()[1] == ",":
                self.take()
                continue
            break
        self.take(")")
        if fn == "sphere_environment_in_collision":
            return ("env", args)
        if fn.startswith("sphere_sphere_self_collision"):
            return ("self", args)
        if fn.startswith("attachment_sphere_collision"):
            return ("att", args)
        raise SyntaxError(f"unknown call {fn}")

    def expr(self):
        e = self.term()
        while self.peek()[1] in ("+", "-"):
            op = self.take()[1]
            e = ("bin", op, e, self.term())
        return e

    def term(self):
        e = self.unary()
        while self.peek()[1] in ("*", "/"):
            op = self.take()[1]
            e = ("bin", op, e, self.unary())
        return e

    def unary(self):
        if self.peek()[1] == "-":
            self.take()
            return ("neg", self.unary())
        return self.primary()

    def primary(self):
        kind, v = self.peek()
        if kind == "num":
            self.take()
            return ("num", v)
        if v == "(":
            self.take()
            e = self.expr()
            self.take(")")
            return e
        if v == "static_cast":
            self.take()
            self.take("<")
            ty = self.take()[1]
            self.take(">")
            self.take("(")
            e = self.expr()
            self.take(")")
            return ("cast", ty, e)
        if v == "q":
            self.take()
            self.take("[")
            idx = int(self.take()[1])
            self.take("]")
            return ("q", idx)
        if v in ("std::sin", "std::cos"):
            self.take()
            self.take("(")
            e = self.expr()
            self.take(")")
            return ("call1", v[5:], e)
        if kind == "id":
            self.take()
            if self.peek()[1] == "." and self.peek(1)[1] in ("sin", "cos"):
                self.take()
                fn = self.take()[1]
                self.take("(")
                self.take(")")
                return ("call1", fn, ("var", v))
            return ("var", v)
        raise SyntaxError(f"bad primary {self.peek()} at {self.i}")


def parse_function(src: str, head_regex: str):
    body = function_body(src, head_regex)
    return Parser(tokenize(body)).stmts()


# --------------------------------------------------------------------------------------
# numerics
# --------------------------------------------------------------------------------------
def fma32(a, b, c):
    """float32 fma emulated in float64 (exact product; single double rounding of the sum)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(F32)


SIN_C1 = F32(-0.478637850138)
SIN_C2 = F32(1.503684069359)
SIN_C3 = F32(0.011596870476)
SIN_C4 = F32(0.140024078368)
SIN_C5 = F32(0.665200679751)
PI_F = F32(3.14159265359)
HALF_PI_F = F32(float(PI_F) / 2.0)
TWO_PI_F = F32(2 * PI_F)


def ref_sin(x):
    """FloatVector::sin() (vector/interface.hh:438-456) as the reference release build
    evaluates it (GCC -O3 -fassociative-math -ffp-contract=fast factors it into Horner form
    with FMAs; pinned bit-exact by tests/test_ref_pin.py)."""
    x = np.asarray(x, F32)
    p = x * fma32(np.abs(x), SIN_C1, SIN_C2)
    ap = np.abs(p)
    return (p * fma32(ap, fma32(ap, SIN_C3, SIN_C4), SIN_C5)).astype(F32)


def ref_cos(x):
    """FloatVector::cos() (vector/interface.hh:458-469)."""
    x = np.asarray(x, F32)
    v = (x + HALF_PI_F).astype(F32)
    v = (v - np.where(v >= PI_F, TWO_PI_F, F32(0))).astype(F32)
    return ref_sin(v)


@dataclass
class Val:
    kind: str  # 'vec' | 'dbl' | 'flt' | 'int'
    v: Any


class Evaluator:
    """Evaluates an FK AST over N lanes.  mode: 'ref32' or 'exact64'."""

    def __init__(self, q: np.ndarray, base100=(0, 0, 0), mode="ref32"):
        self.mode = mode
        self.vt = F32 if mode == "ref32" else np.float64
        self.q = np.asarray(q, self.vt)  # (N, dof)
        self.N = self.q.shape[0]
        self.env: Dict[str, Val] = {}
        self.base100 = base100
        self.out: Dict[str, Dict[int, np.ndarray]] = {"x": {}, "y": {}, "z": {}, "r": {}}

    # ---- expression evaluation ----
    def num(self, text):
        if text.endswith("f"):
            return Val("flt", F32(float(text[:-1])) if self.mode == "ref32" else float(text[:-1]))
        if "." in text or "e" in text or "E" in text:
            return Val("dbl", float(text))
        return Val("int", int(text))

    def to_vec(self, a: Val):
        if a.kind == "vec":
            return a.v
        # scalar broadcast to FloatVector: implicit conversion to float (ScalarT)
        s = self.vt(a.v) if self.mode == "exact64" else F32(a.v)
        return np.full(self.N, s, self.vt)

    def binop(self, op, a: Val, b: Val) -> Val:
        if a.kind == "vec" or b.kind == "vec":
            x, y = self.to_vec(a), self.to_vec(b)
            if op == "+":
                r = x + y
            elif op == "-":
                r = x - y
            elif op == "*":
                r = x * y
            else:
                r = x / y
            return Val("vec", r.astype(self.vt))
        # scalar (op) scalar -- C++ usual arithmetic conversions
        if self.mode == "exact64":
            x, y = float(a.v), float(b.v)
            kind = "dbl"
        elif "dbl" in (a.kind, b.kind):
            x, y = float(a.v), float(b.v)
            kind = "dbl"
        elif "flt" in (a.kind, b.kind):
            x, y = F32(a.v), F32(b.v)
            kind = "flt"
        else:
            x, y = int(a.v), int(b.v)
            kind = "int"
        r = {"+": lambda: x + y, "-": lambda: x - y, "*": lambda: x * y, "/": lambda: x / y}[op]()
        if kind == "flt":
            r = F32(r)
        return Val(kind, r)

    def ev(self, e) -> Val:
        k = e[0]
        if k == "num":
            return self.num(e[1])
        if k == "var":
            name = e[1]
            if name in self.env:
                return self.env[name]
            raise KeyError(name)
        if k == "q":
            return Val("vec", self.q[:, e[1]].astype(self.vt))
        if k == "neg":
            a = self.ev(e[1])
            if a.kind == "vec":
                return Val("vec", (-a.v).astype(self.vt))
            return Val(a.kind, -a.v)
        if k == "bin":
            return self.binop(e[1], self.ev(e[2]), self.ev(e[3]))
        if k == "cast":
            a = self.ev(e[2])
            if e[1] == "float":
                return Val("flt", F32(a.v) if self.mode == "ref32" else float(a.v))
            return a
        if k == "call1":
            a = self.ev(e[2])
            x = self.to_vec(a)
            if self.mode == "exact64":
                r = np.sin(x) if e[1] == "sin" else np.cos(x)
            else:
                r = ref_sin(x) if e[1] == "sin" else ref_cos(x)
            return Val("vec", r.astype(self.vt))
        raise ValueError(k)

    def arg(self, e) -> np.ndarray:
        """static_cast<DataT>(arg): vectors pass, scalars convert through float."""
        return self.to_vec(self.ev(e))

    def bind_base(self):
        bx, by, bz = self.base100
        for name, val in (("base_x100", bx), ("base_y100", by), ("base_z100", bz)):
            self.env[name] = Val("int", val)


# --------------------------------------------------------------------------------------
# collision predicates (numpy restatement of collision/validity.hh + sphere_*.hh)
# --------------------------------------------------------------------------------------
def signbit(x):
    return np.signbit(np.asarray(x, F32))


class RsqrtHost:
    """rsqrt as `_mm256_rsqrt_ps` of THIS host: a (parity, top-K mantissa bits) table,
    probed by oracle/vamp_oracle.c (vo_rsqrt_probe) and passed in."""

    def __init__(self, lut: np.ndarray, kbits: int):
        self.lut = np.asarray(lut, np.uint32)
        self.k = kbits

    def sqrt_approx(self, v):
        from_bits = lambda b: np.asarray(b, np.uint32).view(F32)
        v = np.asarray(v, F32)
        bits = v.view(np.uint32).astype(np.int64)
        e = (bits >> 23) & 0xFF
        mant = bits & 0x7FFFFF
        parity = e & 1
        idx = (parity << self.k) | (mant >> (23 - self.k))
        t = self.lut[idx].astype(np.int64)  # rsqrt of m * 2^(parity ? -1 : 0) ... see oracle
        # table entries are rsqrt bit patterns for inputs with exponent field (126 + parity);
        # rsqrt(x * 4^k) = rsqrt(x) * 2^-k  ->  exponent shift by -(e - (126+parity)) / 2
        shift = (e - (126 + parity)) // 2
        rb = t - (shift << 23)
        r = from_bits(rb.astype(np.uint32))
        out = (v * r).astype(F32)
        # zero / denormal input: rsqrt = +inf, v * inf = NaN (x86 default NaN has the sign bit)
        small = e == 0
        out = np.where(small, from_bits(np.uint32(0xFFC00000)), out).astype(F32)
        return out


@dataclass
class EnvNP:
    """Environment<float> (collision/environment.hh:12-66) as SoA numpy arrays, each
    obstacle list sorted ascending by min_distance (environment.hh:40-66)."""

    spheres: np.ndarray = field(default_factory=lambda: np.zeros((0, 5), F32))   # x y z r mind
    capsules: np.ndarray = field(default_factory=lambda: np.zeros((0, 9), F32))  # x1 y1 z1 xv yv zv r rdv mind
    zcapsules: np.ndarray = field(default_factory=lambda: np.zeros((0, 9), F32))
    cuboids: np.ndarray = field(default_factory=lambda: np.zeros((0, 16), F32))  # x y z a1(3) a2(3) a3(3) r1 r2 r3 mind
    zcuboids: np.ndarray = field(default_factory=lambda: np.zeros((0, 16), F32))


def _dot3(ax, ay, az, bx, by, bz):
    return ((ax * bx) + (ay * by)) + (az * bz)


def env_tests(env: EnvNP, sx, sy, sz, sr):
    """Yield (kind, min_distance[M], values[M, N]) per obstacle type, in the order
    validity.hh:61-127 visits them (spheres, capsules, z-capsules, cuboids, z-cuboids)."""
    sr = F32(sr)
    if len(env.spheres):
        S = env.spheres
        dx = sx[None] - S[:, 0:1]
        dy = sy[None] - S[:, 1:2]
        dz = sz[None] - S[:, 2:3]
        rs = (S[:, 3:4] + sr).astype(F32)
        vals = (_dot3(dx, dy, dz, dx, dy, dz) - rs * rs).astype(F32)
        yield "sphere", S[:, 4], vals
    for kind, C in (("capsule", env.capsules), ("zcapsule", env.zcapsules)):
        if not len(C):
            continue
        x1, y1, z1, xv, yv, zv, r, rdv = (C[:, i:i + 1] for i in range(8))
        if kind == "capsule":
            dot = _dot3(sx[None] - x1, sy[None] - y1, sz[None] - z1, xv, yv, zv)
            cdf = np.minimum(np.maximum(dot * rdv, F32(0)), F32(1)).astype(F32)
            px, py, pz = x1 + xv * cdf, y1 + yv * cdf, z1 + zv * cdf
        else:
            dot = (sz[None] - z1) * zv
            cdf = np.minimum(np.maximum(dot * rdv, F32(0)), F32(1)).astype(F32)
            px, py, pz = np.broadcast_to(x1, dot.shape), np.broadcast_to(y1, dot.shape), z1 + zv * cdf
        dx, dy, dz = sx[None] - px, sy[None] - py, sz[None] - pz
        rs = (sr + r).astype(F32)
        vals = (_dot3(dx, dy, dz, dx, dy, dz) - rs * rs).astype(F32)
        yield kind, C[:, 8], vals
    rsq = F32(sr * sr)
    for kind, C in (("cuboid", env.cuboids), ("zcuboid", env.zcuboids)):
        if not len(C):
            continue
        cx, cy, cz = C[:, 0:1], C[:, 1:2], C[:, 2:3]
        xs, ys, zs = sx[None] - cx, sy[None] - cy, sz[None] - cz
        if kind == "cuboid":
            d1 = _dot3(C[:, 3:4], C[:, 4:5], C[:, 5:6], xs, ys, zs)
            d2 = _dot3(C[:, 6:7], C[:, 7:8], C[:, 8:9], xs, ys, zs)
            d3 = _dot3(C[:, 9:10], C[:, 10:11], C[:, 11:12], xs, ys, zs)
        else:
            d1 = (C[:, 3:4] * xs) + (C[:, 4:5] * ys)
            d2 = (C[:, 6:7] * xs) + (C[:, 7:8] * ys)
            d3 = zs
        a1 = np.maximum(np.abs(d1) - C[:, 12:13], F32(0)).astype(F32)
        a2 = np.maximum(np.abs(d2) - C[:, 13:14], F32(0)).astype(F32)
        a3 = np.maximum(np.abs(d3) - C[:, 14:15], F32(0)).astype(F32)
        vals = (_dot3(a1, a2, a3, a1, a2, a3) - rsq).astype(F32)
        yield kind, C[:, 15], vals


class CheckStats:
    def __init__(self, N):
        self.test_margin = np.full(N, np.inf, np.float64)
        self.cull_margin = np.full(N, np.inf, np.float64)


def group_any(x, G):
    if G == 1:
        return x
    return np.repeat(x.reshape(-1, G).any(1), G)


def group_all(x, G):
    if G == 1:
        return x
    return np.repeat(x.reshape(-1, G).all(1), G)


def env_in_collision(env: EnvNP, rs: RsqrtHost, sx, sy, sz, sr, G, active, stats: CheckStats):
    """sphere_environment_in_collision (validity.hh:46-150), lanes grouped by G
    (G=8: one reference rake block; G=1: a broadcast single configuration)."""
    sx, sy, sz = (np.asarray(a, F32) for a in (sx, sy, sz))
    N = sx.shape[0]
    # dot_3 as the release build evaluates it: fma(x, x, fma(z, z, y*y)) (pinned, test_ref_pin)
    d3 = fma32(sx, sx, fma32(sz, sz, (sy * sy).astype(F32)))
    me = (rs.sqrt_approx(d3) + F32(sr)).astype(F32)
    hit = np.zeros(N, bool)
    for kind, mind, vals in env_tests(env, sx, sy, sz, sr):
        M = len(mind)
        live = active.copy()  # lanes (groups) still scanning this type
        for j in range(M):
            diff = (F32(mind[j]) - me).astype(F32)
            cull = ~signbit(diff)
            stop = group_all(cull, G)
            stats.cull_margin = np.where(live, np.minimum(stats.cull_margin, np.abs(diff)), stats.cull_margin)
            live = live & ~stop
            if not live.any():
                break
            v = vals[j]
            stats.test_margin = np.where(live, np.minimum(stats.test_margin, np.abs(v)), stats.test_margin)
            h = group_any(signbit(v) & live, G) & live
            hit |= h
            live = live & ~h
    return hit


def self_collision(ax, ay, az, ar, bx, by, bz, br, G, active, stats: CheckStats):
    """sphere_sphere_self_collision (validity.hh:13-44 + sphere_sphere.hh:10-22)."""
    dx, dy, dz = ax - bx, ay - by, az - bz
    rsum = (ar + br).astype(F32)
    v = (_dot3(dx, dy, dz, dx, dy, dz) - rsum * rsum).astype(F32)
    stats.test_margin = np.where(active, np.minimum(stats.test_margin, np.abs(v)), stats.test_margin)
    return group_any(signbit(v) & active, G) & active


def run_sphere_fk(ast, q, base100, mode="ref32"):
    ev = Evaluator(q, base100, mode)
    ev.bind_base()
    for st in ast:
        if st[0] == "fdecl":
            ev.env[st[1]] = ev.ev(st[2])
        elif st[0] == "decl":
            ev.env[st[1]] = ev.ev(st[2])
        elif st[0] == "out":
            ev.out[st[1]][st[2]] = ev.arg(st[3])
        else:
            raise ValueError(st[0])
    n = len(ev.out["r"])
    xyz = np.stack([np.stack([ev.out[c][i] for i in range(n)]) for c in "xyz"])  # (3, S, N)
    r = np.array([float(ev.out["r"][i][0]) for i in range(n)])
    return xyz, r


def pose_attachment(att, p):
    """Attachment::pose (collision/attachments.hh:75-122) in float32, left to right: the
    end-effector pose p = (tx, ty, tz, rx, ry, rz, rw) (lane vectors) composed with the
    attachment's relative frame att["tf"] = (tx, ty, tz, rx, ry, rz, rw), then every relative
    sphere centre att["spheres"][k] = (x, y, z, r) rotated and translated.  Returns (x, y, z)
    arrays of shape (K, N) and the radii (K,)."""
    f = F32
    p_tx, p_ty, p_tz, p_rx, p_ry, p_rz, p_rw = (np.asarray(a, f) for a in p)
    t_tx, t_ty, t_tz, t_rx, t_ry, t_rz, t_rw = (f(v) for v in att["tf"])
    two, one = f(2.0), f(1.0)
    rx = p_rw * t_rx + p_rx * t_rw + p_ry * t_rz - p_rz * t_ry
    ry = p_rw * t_ry - p_rx * t_rz + p_ry * t_rw + p_rz * t_rx
    rz = p_rw * t_rz + p_rx * t_ry - p_ry * t_rx + p_rz * t_rw
    rw = p_rw * t_rw - p_rx * t_rx - p_ry * t_ry - p_rz * t_rz
    x0 = p_ry * t_tz - p_rz * t_ty
    x1 = p_rx * t_ty - p_ry * t_tx
    x2 = p_rx * t_tz - p_rz * t_tx
    tx = p_tx + two * (p_rw * x0 + p_ry * x1 + p_rz * x2) + t_tx
    ty = p_ty + two * (-p_rw * x2 - p_rx * x1 + p_rz * x0) + t_ty
    tz = p_tz + two * (p_rw * x1 - p_rx * x2 - p_ry * x0) + t_tz
    bx0, bx1, bx2, bx3 = ry * ry, rz * rz, rw * rz, rw * ry
    bx4, bx5, bx6, bx7, bx8 = rx * rx, rw * rx, rx * ry, rx * rz, ry * rz
    b_xx = -two * (bx0 + bx1) + one
    b_xy = two * (bx6 + bx2)
    b_xz = two * (bx7 - bx3)
    b_yx = two * (bx6 - bx2)
    b_yy = -two * (bx1 + bx4) + one
    b_yz = two * (bx8 + bx5)
    b_zx = two * (bx7 + bx3)
    b_zy = two * (bx8 - bx5)
    b_zz = -two * (bx0 + bx4) + one
    sp = np.asarray(att["spheres"], f).reshape(-1, 4)
    X = np.stack([sx * b_xx + sy * b_yx + sz * b_zx + tx for sx, sy, sz, _ in sp]).astype(f)
    Y = np.stack([sx * b_xy + sy * b_yy + sz * b_zy + ty for sx, sy, sz, _ in sp]).astype(f)
    Z = np.stack([sx * b_xz + sy * b_yz + sz * b_zz + tz for sx, sy, sz, _ in sp]).astype(f)
    return X, Y, Z, sp[:, 3].copy()


def run_fkcc(ast, q, base100, env: EnvNP, rs: RsqrtHost, G=1, att=None):
    """Evaluate interleaved_sphere_fk (or interleaved_sphere_fk_attachment, with `att` =
    {"tf": 7 floats, "spheres": K x 4}) over N lanes grouped by G. Returns (valid[N], stats)."""
    q = np.asarray(q, F32)
    N = q.shape[0]
    assert N % G == 0
    ev = Evaluator(q, base100, "ref32")
    ev.bind_base()
    stats = CheckStats(N)
    alive = np.ones(N, bool)
    posed = {}

    def run(stmts, active):
        nonlocal alive
        for st in stmts:
            k = st[0]
            if k in ("decl", "fdecl"):
                ev.env[st[1]] = ev.ev(st[2])
            elif k == "setpose":
                posed["s"] = pose_attachment(att, [ev.arg(a) for a in st[1]])
            elif k == "if":
                call = st[1]
                act = active & alive
                if call[0] == "env":
                    a = [ev.arg(x) for x in call[1]]
                    c = env_in_collision(env, rs, a[0], a[1], a[2], F32(a[3][0]), G, act, stats)
                elif call[0] == "self":
                    a = [ev.arg(x) for x in call[1]]
                    c = self_collision(*a, G, act, stats)
                elif call[0] == "att":  # attachment_sphere_collision (validity.hh:269-293)
                    a = [ev.arg(x) for x in call[1]]
                    X, Y, Z, R = posed["s"]
                    c = np.zeros(N, bool)
                    for kk in range(len(R)):
                        c |= self_collision(a[0], a[1], a[2], F32(a[3][0]), X[kk], Y[kk], Z[kk], F32(R[kk]), G, act,
                                            stats)
                elif call[0] == "attenv":  # attachment_environment_collision (validity.hh:251-266)
                    X, Y, Z, R = posed["s"]
                    c = np.zeros(N, bool)
                    for kk in range(len(R)):
                        c |= env_in_collision(env, rs, X[kk], Y[kk], Z[kk], F32(R[kk]), G, act & ~c, stats)
                else:
                    raise NotImplementedError(call[0])
                run(st[2], act & c)
            elif k == "ret":
                if not st[1]:
                    alive &= ~active
                return
            else:
                raise ValueError(k)

    run(ast, np.ones(N, bool))
    return alive, stats


# --------------------------------------------------------------------------------------
# hierarchy extraction (structure of interleaved_sphere_fk as data)
# --------------------------------------------------------------------------------------
def hierarchy(ast):
    """Return the ordered list of top-level checks of interleaved_sphere_fk:
    ('env', bounding_args_ast, [child_args_ast...]) or ('self', pair_args_ast, [child_pair_args...])."""
    out = []
    for st in ast:
        if st[0] != "if":
            continue
        call, body = st[1], st[2]
        kids = []
        for b in body:
            if b[0] == "if":
                kids.append(b[1][1])
        out.append((call[0], call[1], kids))
    return out


def load_panda(ref_root="/root/reference"):
    src = open(f"{ref_root}/src/impl/vamp/robots/panda/fk.hh").read()
    fk = parse_function(src, r"inline void sphere_fk\(")
    cc = parse_function(src, r"inline bool interleaved_sphere_fk\(")
    return fk, cc
