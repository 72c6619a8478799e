"""ctypes view of the C restatement (oracle/_build/libvamp_oracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  Never part of the product path.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "libvamp_oracle.so")

F32P = C.POINTER(C.c_float)
U8P = C.POINTER(C.c_uint8)
I32P = C.POINTER(C.c_int32)
U32P = C.POINTER(C.c_uint32)


class VoHeightfield(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("xs", C.c_float), ("ys", C.c_float),
                ("zs", C.c_float), ("xd", C.c_int), ("yd", C.c_int), ("data", F32P)]


class VoCapt(C.Structure):
    _fields_ = [("nlog2", C.c_int), ("r_min", C.c_float), ("r_max", C.c_float), ("r_point", C.c_float),
                ("aabb_top", C.c_float * 6), ("tests", F32P), ("aabbs", F32P), ("aff_starts", U32P),
                ("aff", F32P), ("n_aff", C.c_size_t)]


class VoEnv(C.Structure):
    _fields_ = [
        ("n_spheres", C.c_int), ("n_capsules", C.c_int), ("n_zcapsules", C.c_int), ("n_cuboids", C.c_int),
        ("n_zcuboids", C.c_int),
        ("spheres", F32P), ("capsules", F32P), ("zcapsules", F32P), ("cuboids", F32P), ("zcuboids", F32P),
        ("n_heightfields", C.c_int), ("n_pointclouds", C.c_int),
        ("heightfields", C.POINTER(VoHeightfield)), ("pointclouds", C.POINTER(VoCapt)),
    ]


class VoAttachment(C.Structure):
    _fields_ = [("tf", C.c_float * 7), ("n", C.c_int), ("spheres", F32P)]


class VoStats(C.Structure):
    _fields_ = [("test_margin", C.c_double), ("cull_margin", C.c_double), ("flops", C.c_double)]


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.vo_sin.restype = C.c_float
        L.vo_sin.argtypes = [C.c_float]
        L.vo_cos.restype = C.c_float
        L.vo_cos.argtypes = [C.c_float]
        L.vo_max_extent.restype = C.c_float
        L.vo_max_extent.argtypes = [C.c_float] * 4
        L.vo_l2_norm7.restype = C.c_float
        L.vo_l2_norm7.argtypes = [F32P]
        L.vo_rsqrt_probe.restype = C.c_int
        L.vo_rsqrt_probe.argtypes = [U32P, C.POINTER(C.c_int)]
        L.vo_sqrt_lut.restype = C.c_float
        L.vo_sqrt_lut.argtypes = [C.c_float, U32P, C.c_int]
        L.vo_rsqrt_native.restype = C.c_float
        L.vo_rsqrt_native.argtypes = [C.c_float]
        L.vo_sphere_min_distance.restype = C.c_float
        L.vo_sphere_min_distance.argtypes = [C.c_float] * 4
        L.vo_cuboid_min_distance.restype = C.c_float
        L.vo_cuboid_min_distance.argtypes = [F32P]
        L.vo_capsule_min_distance.restype = C.c_float
        L.vo_capsule_min_distance.argtypes = [F32P]
        L.vo_panda_sphere_fk.argtypes = [F32P, C.c_int, C.c_int, C.c_int, F32P]
        L.vo_panda_fkcc_block.restype = C.c_int
        L.vo_panda_fkcc_block.argtypes = [C.POINTER(VoEnv), F32P, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(VoStats)]
        L.vo_panda_validate_motion.restype = C.c_int
        L.vo_panda_validate_motion.argtypes = [C.POINTER(VoEnv), F32P, F32P, C.c_int, C.c_int, C.c_int,
                                               C.POINTER(C.c_int), C.POINTER(VoStats)]
        L.vo_panda_validate_motion_split.restype = C.c_int
        L.vo_panda_validate_motion_split.argtypes = [C.POINTER(VoEnv), F32P, F32P, C.c_int, C.c_int, C.c_int,
                                                     C.POINTER(C.c_int), C.POINTER(VoStats), C.POINTER(VoStats)]
        L.vo_panda_fkcc_configs.argtypes = [C.POINTER(VoEnv), F32P, C.c_size_t, C.c_int, C.c_int, C.c_int, U8P,
                                            C.c_int]
        L.vo_panda_validate_motions.argtypes = [C.POINTER(VoEnv), F32P, F32P, C.c_size_t, C.c_int, C.c_int,
                                                C.c_int, U8P, I32P, C.c_int]
        L.vo_halton.argtypes = [C.c_int, C.c_uint64, F32P]
        L.vo_sphere_heightfield.restype = C.c_float
        L.vo_sphere_heightfield.argtypes = [C.POINTER(VoHeightfield), C.c_float, C.c_float, C.c_float, C.c_float,
                                            C.POINTER(C.c_int)]
        L.vo_sql2_3.restype = C.c_float
        L.vo_sql2_3.argtypes = [C.c_float] * 6
        for fn in ("vo_capt_box_vec", "vo_capt_vol_distsq", "vo_capt_vol_ball"):
            getattr(L, fn).restype = C.c_float
            getattr(L, fn).argtypes = [F32P, F32P, F32P]
        L.vo_capt_build.restype = C.c_int
        L.vo_capt_build.argtypes = [F32P, C.c_size_t, C.c_float, C.c_float, C.c_float, C.POINTER(VoCapt)]
        L.vo_capt_free.argtypes = [C.POINTER(VoCapt)]
        L.vo_capt_collides_batch.argtypes = [C.POINTER(VoCapt), F32P, F32P, C.c_size_t, C.c_int, U8P,
                                             C.POINTER(C.c_double)]
        L.vo_panda_scale.argtypes = [F32P]
        L.vo_robot_scale.argtypes = [C.c_int, F32P]
        L.vo_robot_sphere_fk.argtypes = [C.c_int, F32P, C.c_int, C.c_int, C.c_int, F32P]
        L.vo_robot_fkcc_block.restype = C.c_int
        L.vo_robot_fkcc_block.argtypes = [C.c_int, C.POINTER(VoEnv), F32P, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(VoStats)]
        L.vo_robot_validate_motion.restype = C.c_int
        L.vo_robot_validate_motion.argtypes = [C.c_int, C.POINTER(VoEnv), F32P, F32P, C.c_int, C.c_int, C.c_int,
                                               C.POINTER(C.c_int), C.POINTER(VoStats)]
        L.vo_robot_validate_vector.restype = C.c_int
        L.vo_robot_validate_vector.argtypes = [C.c_int, C.POINTER(VoEnv), F32P, F32P, C.c_float, C.c_int, C.c_int,
                                               C.c_int, C.POINTER(C.c_int)]
        L.vo_robot_fkcc_configs.argtypes = [C.c_int, C.POINTER(VoEnv), F32P, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                            U8P, C.c_int]
        L.vo_robot_validate_motions.argtypes = [C.c_int, C.POINTER(VoEnv), F32P, F32P, C.c_size_t, C.c_int,
                                                C.c_int, C.c_int, U8P, I32P, C.c_int]
        I3 = C.c_int * 3
        L.vo_pair_fkcc_block.restype = C.c_int
        L.vo_pair_fkcc_block.argtypes = [C.POINTER(VoEnv), F32P, C.c_int, I3, I3, C.POINTER(VoStats)]
        L.vo_pair_validate_motion.restype = C.c_int
        L.vo_pair_validate_motion.argtypes = [C.POINTER(VoEnv), F32P, F32P, I3, I3, C.POINTER(C.c_int),
                                              C.POINTER(VoStats)]
        L.vo_pair_fkcc_configs.argtypes = [C.POINTER(VoEnv), F32P, C.c_size_t, I3, I3, U8P, C.c_int]
        L.vo_pair_validate_motions.argtypes = [C.POINTER(VoEnv), F32P, F32P, C.c_size_t, I3, I3, U8P, I32P,
                                               C.c_int]
        AP = C.POINTER(VoAttachment)
        L.vo_robot_fkcc_attach_block.restype = C.c_int
        L.vo_robot_fkcc_attach_block.argtypes = [C.c_int, C.POINTER(VoEnv), AP, F32P, C.c_int, C.c_int, C.c_int,
                                                 C.c_int, C.POINTER(VoStats)]
        L.vo_robot_fkcc_attach_configs.argtypes = [C.c_int, C.POINTER(VoEnv), AP, F32P, C.c_size_t, C.c_int,
                                                   C.c_int, C.c_int, U8P, C.c_int]
        L.vo_robot_validate_motions_att.argtypes = [C.c_int, C.POINTER(VoEnv), AP, F32P, F32P, C.c_size_t,
                                                    C.c_int, C.c_int, C.c_int, U8P, I32P, C.c_int]
        L.vo_l2_norm.restype = C.c_float
        L.vo_l2_norm.argtypes = [F32P, C.c_int]
        _lib = L
    return _lib


def fp(a):
    return a.ctypes.data_as(F32P)


class Env:
    """Host environment in the oracle's layout, built like the reference's
    Environment::add_* (bindings/environment.cc:107-146): min_distance from the shape
    constructors, cuboids with axis_3_z == 1 and capsules with xv == yv == 0 routed to the
    z-aligned lists, every list sorted by min_distance (environment.hh:40-66)."""

    def __init__(self):
        self.spheres, self.capsules, self.zcapsules, self.cuboids, self.zcuboids = [], [], [], [], []
        self.heightfields, self.pointclouds = [], []

    def add_sphere(self, center, r):
        x, y, z = (float(np.float32(v)) for v in center)
        md = lib().vo_sphere_min_distance(x, y, z, float(np.float32(r)))
        self.spheres.append([x, y, z, r, md])
        return self

    def add_cuboid_axes(self, center, a1, a2, a3, half):
        c = np.array(list(center) + list(a1) + list(a2) + list(a3) + list(half), np.float32)
        md = lib().vo_cuboid_min_distance(fp(c))
        row = list(c) + [md]
        (self.zcuboids if c[11] == 1.0 else self.cuboids).append(row)
        return self

    def add_capsule_endpoints(self, p1, p2, r):
        p1 = np.array(p1, np.float32)
        p2 = np.array(p2, np.float32)
        v = (p2 - p1).astype(np.float32)
        dot = np.float32((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
        rdv = np.float32(1.0 / float(dot))  # factory.hh:120-121 (double reciprocal, cast)
        c = np.array(list(p1) + list(v) + [r, rdv], np.float32)
        md = lib().vo_capsule_min_distance(fp(c))
        row = list(c) + [md]
        (self.zcapsules if (v[0] == 0 and v[1] == 0) else self.capsules).append(row)
        return self

    def add_heightfield(self, center, scale, xd, yd, data):
        """factory::heightfield::flat (factory.hh:365-386): stores 1/scale."""
        d = np.ascontiguousarray(data, np.float32).ravel()
        assert d.size == xd * yd
        self.heightfields.append(((np.float32(center[0]), np.float32(center[1]), np.float32(center[2]),
                                   np.float32(1.0) / np.float32(scale[0]), np.float32(1.0) / np.float32(scale[1]),
                                   np.float32(1.0) / np.float32(scale[2]), int(xd), int(yd)), d))
        return self

    def add_pointcloud(self, points, r_min, r_max, r_point):
        self.pointclouds.append(Capt(points, r_min, r_max, r_point))
        return self

    def arrays(self):
        out = {}
        for name, width in (("spheres", 5), ("capsules", 9), ("zcapsules", 9), ("cuboids", 16), ("zcuboids", 16)):
            rows = getattr(self, name)
            a = np.array(rows, np.float32).reshape(-1, width)
            if len(a):
                a = a[np.argsort(a[:, -1], kind="stable")]
            out[name] = np.ascontiguousarray(a)
        return out

    def c(self):
        arrs = self.arrays()
        self._keep = arrs
        e = VoEnv()
        for name in arrs:
            setattr(e, "n_" + name, len(arrs[name]))
            setattr(e, name, fp(arrs[name]) if len(arrs[name]) else None)
        if self.heightfields:
            hf = (VoHeightfield * len(self.heightfields))()
            for i, (h, d) in enumerate(self.heightfields):
                hf[i] = VoHeightfield(*h, fp(d))
            e.n_heightfields = len(self.heightfields)
            e.heightfields = hf
            self._keep_hf = hf
        if self.pointclouds:
            pc = (VoCapt * len(self.pointclouds))()
            for i, t in enumerate(self.pointclouds):
                pc[i] = t.t
            e.n_pointclouds = len(self.pointclouds)
            e.pointclouds = pc
            self._keep_pc = pc
        return e


class Capt:
    """CAPT::CAPT (collision/capt.hh:327-398) built by the C restatement."""

    def __init__(self, points, r_min, r_max, r_point):
        p = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
        self.t = VoCapt()
        lib().vo_capt_build(fp(p), p.shape[0], r_min, r_max, r_point, C.byref(self.t))

    def arrays(self):
        t = self.t
        m = 1 << t.nlog2
        return {
            "nlog2": t.nlog2,
            "tests": np.ctypeslib.as_array(t.tests, (max(m - 1, 1),))[: m - 1].copy(),
            "aabbs": np.ctypeslib.as_array(t.aabbs, (m * 6,)).reshape(m, 6).copy(),
            "aff_starts": np.ctypeslib.as_array(t.aff_starts, (m + 1,)).copy(),
            "aff": (np.ctypeslib.as_array(t.aff, (t.n_aff * 24,)).reshape(-1, 3, 8).copy() if t.n_aff
                    else np.zeros((0, 3, 8), np.float32)),
            "aabb_top": np.array(t.aabb_top[:], np.float32),
        }

    def collides(self, centers, radii, simd=False, margin=False):
        c = np.ascontiguousarray(centers, np.float32).reshape(-1, 3)
        r = np.ascontiguousarray(radii, np.float32).ravel()
        out = np.zeros(c.shape[0], np.uint8)
        m = np.zeros(c.shape[0], np.float64)
        lib().vo_capt_collides_batch(C.byref(self.t), fp(c), fp(r), c.shape[0], int(simd), out.ctypes.data_as(U8P),
                                     m.ctypes.data_as(C.POINTER(C.c_double)))
        return (out.astype(bool), m) if margin else out.astype(bool)

    def __del__(self):
        try:
            lib().vo_capt_free(C.byref(self.t))
        except Exception:
            pass


def sphere_cage_env():
    """The 14-sphere cage of scripts/cpp/benchmark_collision_checks.cc:33-51 (r = 0.2)."""
    centers = [(0.55, 0, 0.25), (0.35, 0.35, 0.25), (0, 0.55, 0.25), (-0.55, 0, 0.25), (-0.35, -0.35, 0.25),
               (0, -0.55, 0.25), (0.35, -0.35, 0.25), (0.35, 0.35, 0.8), (0, 0.55, 0.8), (-0.35, 0.35, 0.8),
               (-0.55, 0, 0.8), (-0.35, -0.35, 0.8), (0, -0.55, 0.8), (0.35, -0.35, 0.8)]
    e = Env()
    for c in centers:
        e.add_sphere(c, np.float32(0.2))
    return e


def sphere_fk(q, base100=(0, 0, 0)):
    q = np.ascontiguousarray(q, np.float32).reshape(-1, 7)
    out = np.zeros((q.shape[0], 59, 3), np.float32)
    L = lib()
    for i in range(q.shape[0]):
        L.vo_panda_sphere_fk(fp(q[i]), *base100, fp(out[i]))
    return out


def fkcc(env: Env, q, base100=(0, 0, 0), G=1, stats=False):
    q = np.ascontiguousarray(q, np.float32).reshape(-1, 7)
    N = q.shape[0]
    assert N % G == 0
    ce = env.c()
    L = lib()
    res = np.zeros(N // G, bool)
    tm = np.zeros(N // G)
    cm = np.zeros(N // G)
    fl = np.zeros(N // G)
    for i in range(N // G):
        st = VoStats(np.inf, np.inf, 0.0)
        res[i] = L.vo_panda_fkcc_block(C.byref(ce), fp(q[i * G:(i + 1) * G]), G, *base100, C.byref(st))
        tm[i], cm[i], fl[i] = st.test_margin, st.cull_margin, st.flops
    if stats:
        return res, tm, cm, fl
    return res


def fkcc_threads(env: Env, q, base100=(0, 0, 0), threads=8):
    q = np.ascontiguousarray(q, np.float32).reshape(-1, 7)
    out = np.zeros(q.shape[0], np.uint8)
    ce = env.c()
    lib().vo_panda_fkcc_configs(C.byref(ce), fp(q), q.shape[0], *base100, out.ctypes.data_as(U8P), threads)
    return out.astype(bool)


def validate_motions(env: Env, starts, goals, base100=(0, 0, 0), threads=8):
    s = np.ascontiguousarray(starts, np.float32).reshape(-1, 7)
    g = np.ascontiguousarray(goals, np.float32).reshape(-1, 7)
    ok = np.zeros(s.shape[0], np.uint8)
    n = np.zeros(s.shape[0], np.int32)
    ce = env.c()
    lib().vo_panda_validate_motions(C.byref(ce), fp(s), fp(g), s.shape[0], *base100, ok.ctypes.data_as(U8P),
                                    n.ctypes.data_as(I32P), threads)
    return ok.astype(bool), n


def rsqrt_probe():
    lut = np.zeros(2 << 16, np.uint32)
    k = C.c_int(0)
    rc = lib().vo_rsqrt_probe(lut.ctypes.data_as(U32P), C.byref(k))
    if rc != 0:
        raise RuntimeError(f"rsqrt probe failed ({rc})")
    return lut[: 2 << k.value].copy(), k.value


def halton(dim, ks):
    out = np.zeros((len(ks), dim), np.float32)
    for i, k in enumerate(ks):
        lib().vo_halton(dim, int(k), fp(out[i]))
    return out


def scale(q):
    q = np.ascontiguousarray(q, np.float32).reshape(-1, 7).copy()
    for i in range(q.shape[0]):
        lib().vo_panda_scale(fp(q[i]))
    return q


def validate_flops(env: Env, starts, goals, base100=(0, 0, 0), threads=8):
    """Executed float ops of validate_motion per edge (reference semantics, early exit),
    split into the first rake block and the back-steps (edges in parallel chunks: ctypes calls
    release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    ce = env.c()
    L = lib()
    starts = np.ascontiguousarray(starts, np.float32).reshape(len(starts), -1)
    goals = np.ascontiguousarray(goals, np.float32).reshape(len(goals), -1)
    head = np.zeros(len(starts))
    tail = np.zeros(len(starts))

    def run(lo, hi):
        for i in range(lo, hi):
            h = VoStats(np.inf, np.inf, 0.0)
            t = VoStats(np.inf, np.inf, 0.0)
            n = C.c_int()
            L.vo_panda_validate_motion_split(C.byref(ce), fp(starts[i]), fp(goals[i]), *base100, C.byref(n),
                                             C.byref(h), C.byref(t))
            head[i], tail[i] = h.flops, t.flops

    chunks = np.linspace(0, len(starts), max(1, threads) + 1).astype(int)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        list(ex.map(lambda k: run(chunks[k], chunks[k + 1]), range(len(chunks) - 1)))
    return head, tail


# ---- robot-generic views (robot = "panda" | "fetch"; ids match VGPU_ROBOT_*) ----
ROBOTS = {"panda": (1, 7, 59), "fetch": (2, 8, 111), "ur5": (4, 6, 36), "baxter": (5, 14, 75)}
RESOLUTION = {"panda": 32, "fetch": 32, "ur5": 32, "baxter": 64}  # Robot::resolution


def robot_scale(robot, u):
    rid, dim, _ = ROBOTS[robot]
    q = np.ascontiguousarray(u, np.float32).reshape(-1, dim).copy()
    for i in range(q.shape[0]):
        lib().vo_robot_scale(rid, fp(q[i]))
    return q


def robot_sphere_fk(robot, q, base100=(0, 0, 0)):
    rid, dim, ns = ROBOTS[robot]
    q = np.ascontiguousarray(q, np.float32).reshape(-1, dim)
    out = np.zeros((q.shape[0], ns, 3), np.float32)
    for i in range(q.shape[0]):
        lib().vo_robot_sphere_fk(rid, fp(q[i]), *base100, fp(out[i]))
    return out


def robot_filter_pointcloud(robot, env: Env, q, pc, point_radius, base100=(0, 0, 0)):
    """filter_robot_from_pointcloud (bindings/common.hh:36-87): keep mask [n] (oracle/vamp_oracle.c)"""
    rid, dim, _ = ROBOTS[robot]
    q = np.ascontiguousarray(q, np.float32).reshape(dim)
    pc = np.ascontiguousarray(pc, np.float32).reshape(-1, 3)
    keep = np.zeros(pc.shape[0], np.uint8)
    ce = env.c()
    L = lib()
    L.vo_robot_filter_pointcloud.argtypes = [C.c_int, C.c_void_p, F32P, C.c_int, C.c_int, C.c_int, F32P, C.c_size_t,
                                             C.c_float, U8P]
    L.vo_robot_filter_pointcloud(rid, C.byref(ce), fp(q), *base100, fp(pc), pc.shape[0], float(point_radius),
                                 keep.ctypes.data_as(U8P))
    return keep.astype(bool)


def robot_fkcc(robot, env: Env, q, base100=(0, 0, 0), G=1, stats=False):
    rid, dim, _ = ROBOTS[robot]
    q = np.ascontiguousarray(q, np.float32).reshape(-1, dim)
    N = q.shape[0]
    assert N % G == 0
    ce = env.c()
    res = np.zeros(N // G, bool)
    tm = np.zeros(N // G)
    cm = np.zeros(N // G)
    fl = np.zeros(N // G)
    for i in range(N // G):
        st = VoStats(np.inf, np.inf, 0.0)
        res[i] = lib().vo_robot_fkcc_block(rid, C.byref(ce), fp(q[i * G:(i + 1) * G]), G, *base100, C.byref(st))
        tm[i], cm[i], fl[i] = st.test_margin, st.cull_margin, st.flops
    return (res, tm, cm, fl) if stats else res


def robot_fkcc_threads(robot, env: Env, q, base100=(0, 0, 0), threads=8):
    rid, dim, _ = ROBOTS[robot]
    q = np.ascontiguousarray(q, np.float32).reshape(-1, dim)
    out = np.zeros(q.shape[0], np.uint8)
    ce = env.c()
    lib().vo_robot_fkcc_configs(rid, C.byref(ce), fp(q), q.shape[0], *base100, out.ctypes.data_as(U8P), threads)
    return out.astype(bool)


def robot_validate_vector(robot, env_c, start, vector, distance, base100=(0, 0, 0)):
    """validate_vector<Robot, 8, res>(start, vector, distance) (planning/validate.hh:23-65); env_c is
    Env.c() (kept alive by the caller across calls)"""
    rid = ROBOTS[robot][0]
    s = np.ascontiguousarray(start, np.float32)
    v = np.ascontiguousarray(vector, np.float32)
    return bool(lib().vo_robot_validate_vector(rid, C.byref(env_c), fp(s), fp(v), float(distance), *base100, None))


def robot_validate_motions(robot, env: Env, starts, goals, base100=(0, 0, 0), threads=8):
    rid, dim, _ = ROBOTS[robot]
    s = np.ascontiguousarray(starts, np.float32).reshape(-1, dim)
    g = np.ascontiguousarray(goals, np.float32).reshape(-1, dim)
    ok = np.zeros(s.shape[0], np.uint8)
    n = np.zeros(s.shape[0], np.int32)
    ce = env.c()
    lib().vo_robot_validate_motions(rid, C.byref(ce), fp(s), fp(g), s.shape[0], *base100, ok.ctypes.data_as(U8P),
                                    n.ctypes.data_as(I32P), threads)
    return ok.astype(bool), n


def robot_validate_flops(robot, env: Env, starts, goals, base100=(0, 0, 0), threads=8):
    """Executed float ops of validate_motion per edge (reference semantics, early exit) for any robot, counted
    by the instrumented restatement (vo_robot_validate_motion's vo_stats.flops); edges in parallel chunks"""
    from concurrent.futures import ThreadPoolExecutor
    rid, dim, _ = ROBOTS[robot]
    ce = env.c()
    L = lib()
    s = np.ascontiguousarray(starts, np.float32).reshape(-1, dim)
    g = np.ascontiguousarray(goals, np.float32).reshape(-1, dim)
    fl = np.zeros(len(s))

    def run(lo, hi):
        for i in range(lo, hi):
            st = VoStats(np.inf, np.inf, 0.0)
            n = C.c_int()
            L.vo_robot_validate_motion(rid, C.byref(ce), fp(s[i]), fp(g[i]), *base100, C.byref(n), C.byref(st))
            fl[i] = st.flops

    chunks = np.linspace(0, len(s), max(1, threads) + 1).astype(int)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        list(ex.map(lambda k: run(chunks[k], chunks[k + 1]), range(len(chunks) - 1)))
    return fl


def mbm_env(scene: dict) -> Env:
    """A MotionBenchMaker scene (resources/<robot>/problems.tar.bz2 scene*.yaml) as an
    environment: boxes -> cuboids by the RESOLVED axes of the pose quaternion (columns of its
    rotation matrix, float64 -> float32), half extents = dimensions / 2; cylinders -> capsules by
    endpoints centre -+ axis_z * length / 2 (src/vamp/__init__.py:135-184 routes cylinders to
    capsules and boxes to cuboids; its Euler -> Eigen axes step is restated, parity unpinned,
    which is why fixtures carry the resolved rows)."""
    e = Env()
    for obj in scene["world"]["collision_objects"]:
        for prim, pose in zip(obj["primitives"], obj["primitive_poses"]):
            x, y, z, w = pose["orientation"]
            R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                          [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                          [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
            c = np.array(pose["position"], np.float64)
            if prim["type"] == "box":
                h = np.array(prim["dimensions"], np.float64) / 2
                e.add_cuboid_axes(c, R[:, 0], R[:, 1], R[:, 2], h)
            elif prim["type"] == "cylinder":
                length, radius = prim["dimensions"]
                a = R[:, 2] * (length / 2)
                e.add_capsule_endpoints(c - a, c + a, np.float32(radius))
            elif prim["type"] == "sphere":
                e.add_sphere(c, np.float32(prim["dimensions"][0]))
    return e


# ---- two-Panda composite (BASELINE configs[4]) ----
def _i3(b):
    return (C.c_int * 3)(*[int(v) for v in b])


def pair_fkcc(env: Env, q, ba=(0, 0, 0), bb=(100, 0, 0), G=1, stats=False):
    q = np.ascontiguousarray(q, np.float32).reshape(-1, 14)
    N = q.shape[0]
    ce = env.c()
    res = np.zeros(N // G, bool)
    fl = np.zeros(N // G)
    for i in range(N // G):
        st = VoStats(np.inf, np.inf, 0.0)
        res[i] = lib().vo_pair_fkcc_block(C.byref(ce), fp(q[i * G:(i + 1) * G]), G, _i3(ba), _i3(bb), C.byref(st))
        fl[i] = st.flops
    return (res, fl) if stats else res


def pair_fkcc_threads(env: Env, q, ba=(0, 0, 0), bb=(100, 0, 0), threads=8):
    q = np.ascontiguousarray(q, np.float32).reshape(-1, 14)
    out = np.zeros(q.shape[0], np.uint8)
    ce = env.c()
    lib().vo_pair_fkcc_configs(C.byref(ce), fp(q), q.shape[0], _i3(ba), _i3(bb), out.ctypes.data_as(U8P), threads)
    return out.astype(bool)


def pair_validate_motions(env: Env, starts, goals, ba=(0, 0, 0), bb=(100, 0, 0), threads=8):
    s = np.ascontiguousarray(starts, np.float32).reshape(-1, 14)
    g = np.ascontiguousarray(goals, np.float32).reshape(-1, 14)
    ok = np.zeros(s.shape[0], np.uint8)
    n = np.zeros(s.shape[0], np.int32)
    ce = env.c()
    lib().vo_pair_validate_motions(C.byref(ce), fp(s), fp(g), s.shape[0], _i3(ba), _i3(bb), ok.ctypes.data_as(U8P),
                                   n.ctypes.data_as(I32P), threads)
    return ok.astype(bool), n


def pair_validate_vector(env_c, start, vector, distance, ba=(0, 0, 0), bb=(100, 0, 0)):
    """validate_vector<Composite, 8, 32>(start, vector, distance) (planning/validate.hh:23-65, oracle
    vo_pair_validate_vector); env_c is Env.c() (kept alive by the caller across calls)"""
    s = np.ascontiguousarray(start, np.float32)
    v = np.ascontiguousarray(vector, np.float32)
    L = lib()
    L.vo_pair_validate_vector.argtypes = [C.c_void_p, F32P, F32P, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p]
    return bool(L.vo_pair_validate_vector(C.byref(env_c), fp(s), fp(v), float(distance), _i3(ba), _i3(bb), None,
                                          None))


def pair_scale(u):
    """the composite's scale_configuration: each arm's seven joints by the Panda's limits"""
    u = np.ascontiguousarray(u, np.float32).reshape(-1, 14)
    return np.concatenate([robot_scale("panda", u[:, :7]), robot_scale("panda", u[:, 7:])], axis=1)


def pair_scene() -> Env:
    """Config-5 scene: a table surface under both arms plus three spheres between them."""
    e = Env()
    e.add_cuboid_axes((0.5, 0.0, -0.15), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1.3, 0.8, 0.05))
    for c in ((0.5, 0.55, 0.35), (0.5, -0.55, 0.35), (0.5, 0.0, 1.05)):
        e.add_sphere(c, np.float32(0.1))
    return e


def pair_validate_flops(env: Env, starts, goals, ba=(0, 0, 0), bb=(100, 0, 0)):
    """executed float ops of the composite validate_motion per edge (reference semantics)"""
    ce = env.c()
    out = np.zeros(len(starts))
    for i in range(len(starts)):
        st = VoStats(np.inf, np.inf, 0.0)
        n = C.c_int()
        lib().vo_pair_validate_motion(C.byref(ce), fp(np.ascontiguousarray(starts[i], np.float32)),
                                      fp(np.ascontiguousarray(goals[i], np.float32)), _i3(ba), _i3(bb), C.byref(n),
                                      C.byref(st))
        out[i] = st.flops
    return out


# ---- attachments (collision/attachments.hh; Robot::fkcc_attach) ----
class Attachment:
    """Attachment(center, quaternion_xyzw) + add_sphere (bindings/environment.cc:197-249)."""

    def __init__(self, center, quaternion_xyzw):
        self.tf = np.array(list(center) + list(quaternion_xyzw), np.float32)
        self.spheres = []

    def add_sphere(self, center, r):
        self.spheres.append([float(np.float32(v)) for v in center] + [float(np.float32(r))])
        return self

    def c(self):
        self._keep = np.ascontiguousarray(np.array(self.spheres, np.float32).reshape(-1, 4))
        a = VoAttachment()
        for i in range(7):
            a.tf[i] = float(self.tf[i])
        a.n = len(self.spheres)
        a.spheres = fp(self._keep)
        return a

    def as_dict(self):
        return {"tf": self.tf.copy(), "spheres": np.array(self.spheres, np.float32).reshape(-1, 4)}


def held_object():
    """A bar held 10-25 cm along the hand's z axis (four spheres, r 3 cm), turned 45 degrees."""
    a = Attachment((0.0, 0.0, 0.1), (0.0, 0.0, 0.38268343, 0.92387953))
    for z in (0.0, 0.05, 0.1, 0.15):
        a.add_sphere((0.03, 0.0, z), 0.03)
    return a


def robot_fkcc_attach_threads(robot, env: Env, att: Attachment, q, base100=(0, 0, 0), threads=8):
    rid, dim, _ = ROBOTS[robot]
    q = np.ascontiguousarray(q, np.float32).reshape(-1, dim)
    out = np.zeros(q.shape[0], np.uint8)
    ce, ca = env.c(), att.c()
    lib().vo_robot_fkcc_attach_configs(rid, C.byref(ce), C.byref(ca), fp(q), q.shape[0], *base100,
                                       out.ctypes.data_as(U8P), threads)
    return out.astype(bool)


def robot_validate_motions_att(robot, env: Env, att: Attachment, starts, goals, base100=(0, 0, 0), threads=8):
    rid, dim, _ = ROBOTS[robot]
    s = np.ascontiguousarray(starts, np.float32).reshape(-1, dim)
    g = np.ascontiguousarray(goals, np.float32).reshape(-1, dim)
    ok = np.zeros(s.shape[0], np.uint8)
    n = np.zeros(s.shape[0], np.int32)
    ce, ca = env.c(), att.c()
    lib().vo_robot_validate_motions_att(rid, C.byref(ce), C.byref(ca), fp(s), fp(g), s.shape[0], *base100,
                                        ok.ctypes.data_as(U8P), n.ctypes.data_as(I32P), threads)
    return ok.astype(bool), n


# ---- PRM roadmap edge stage (planning/prm.hh:235-283) ----
# Robot::space_measure() returns float (panda/fk.hh:88-91)
SPACE_MEASURE = {r: float(np.float32(json.load(open(os.path.join(ROOT, "model", f"{r}.json")))["space_measure"]))
                 for r in ("panda", "fetch", "ur5", "baxter")}


def prm_max_neighbors(dim, n):
    L = lib()
    L.vo_prm_max_neighbors.restype = C.c_size_t
    L.vo_prm_max_neighbors.argtypes = [C.c_int, C.c_size_t]
    return int(L.vo_prm_max_neighbors(dim, n))


def prm_neighbor_radius(dim, space_measure, gamma, n):
    L = lib()
    L.vo_prm_neighbor_radius.restype = C.c_float
    L.vo_prm_neighbor_radius.argtypes = [C.c_int, C.c_double, C.c_double, C.c_size_t]
    return np.float32(L.vo_prm_neighbor_radius(dim, space_measure, gamma, n))


def roadmap_knn(V, space_measure, gamma=2.0, kmax=None, threads=8):
    """The neighbour lists build_roadmap queries for each vertex (nearest first)."""
    V = np.ascontiguousarray(V, np.float32)
    n, dim = V.shape
    kmax = kmax or max(1, prm_max_neighbors(dim, max(n - 1, 2)))
    nbr = np.zeros((n, kmax), np.uint32)
    dist = np.zeros((n, kmax), np.float32)
    cnt = np.zeros(n, np.uint32)
    L = lib()
    L.vo_roadmap_knn.argtypes = [C.c_int, F32P, C.c_size_t, C.c_double, C.c_double, C.c_uint32,
                                 C.POINTER(C.c_uint32), F32P, C.POINTER(C.c_uint32), C.c_int]
    U32P_ = C.POINTER(C.c_uint32)
    L.vo_roadmap_knn(dim, fp(V), n, space_measure, gamma, kmax, nbr.ctypes.data_as(U32P_), fp(dist),
                     cnt.ctypes.data_as(U32P_), threads)
    return nbr, dist, cnt


def build_roadmap_edges(robot, env: Env, V, base100=(0, 0, 0), gamma=2.0, threads=8):
    """Roadmap::build_roadmap's graph (prm.hh:235-299) for the vertex sequence V (start, goal,
    valid samples in draw order): per vertex, its valid neighbours in query order (nearest
    first), then the later vertices that connected to it, ascending -- the order the reference
    appends them (prm.hh:268-276).  The kNN does not depend on edge validity, so every candidate
    edge is validated in one parallel batch (validate_motion(neighbor, new vertex))."""
    V = np.ascontiguousarray(V, np.float32)
    n, dim = V.shape
    nbr, dist, cnt = roadmap_knn(V, SPACE_MEASURE[robot], gamma, threads=threads)
    qi = np.repeat(np.arange(n), cnt.astype(np.int64))
    qm = np.concatenate([np.arange(c) for c in cnt]) if n else np.zeros(0, np.int64)
    cand = nbr[qi, qm].astype(np.int64)
    ok, _ = robot_validate_motions(robot, env, V[cand], V[qi], base100, threads)
    edges = [[] for _ in range(n)]
    for i, j, good in zip(qi.tolist(), cand.tolist(), ok.tolist()):
        if good:
            edges[i].append(j)
            edges[j].append(i)
    return edges, (nbr, dist, cnt, ok)


def components(n, edges):
    """Connected components by union-find: the smallest vertex index of each vertex's component."""
    parent = list(range(n))

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a
    for i, lst in enumerate(edges):
        for j in lst:
            a, b = find(i), find(j)
            if a != b:
                parent[max(a, b)] = min(a, b)
    return np.array([find(i) for i in range(n)], np.uint32)


def morton_encode(x, y, z):
    L = lib()
    L.vo_morton_encode.restype = C.c_uint32
    L.vo_morton_encode.argtypes = [C.c_uint32] * 3
    return L.vo_morton_encode(x, y, z)


def remap_point(x, mn, mx):
    L = lib()
    L.vo_remap_point.restype = C.c_uint32
    L.vo_remap_point.argtypes = [C.c_float] * 3
    return L.vo_remap_point(x, mn, mx)


def filter_pointcloud(pc, min_dist, max_range, origin, ws_min, ws_max, cull=True):
    """filter_pointcloud (collision/filter.hh:175-268): kept point indices in the final order."""
    L = lib()
    L.vo_filter_pointcloud.restype = C.c_size_t
    L.vo_filter_pointcloud.argtypes = [F32P, C.c_size_t, C.c_float, C.c_float, F32P, F32P, F32P, C.c_int, U32P]
    pc = np.ascontiguousarray(pc, np.float32).reshape(-1, 3)
    out = np.zeros(max(pc.shape[0], 1), np.uint32)
    o, a, b = (np.ascontiguousarray(v, np.float32) for v in (origin, ws_min, ws_max))
    k = L.vo_filter_pointcloud(fp(pc), pc.shape[0], min_dist, max_range, fp(o), fp(a), fp(b), int(cull),
                               out.ctypes.data_as(U32P))
    return out[:k].copy()
