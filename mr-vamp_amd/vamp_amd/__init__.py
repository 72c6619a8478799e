"""vamp_amd -- MI355X (gfx950) implementation of VAMP's motion-validation rake.

Host-side mirror of the reference's Python surface for this path
(``vamp.Environment``/``Sphere``/``Cuboid``/``Cylinder`` and ``vamp.<robot>.fk``/``validate``;
reference src/impl/vamp/bindings/environment.cc:18-146 and bindings/common.hh:132-182,586-725),
plus the batch entry points the GPU path exists for.  Every call goes through the C ABI
(include/vamp_gpu.h) into libvampgpu.so; nothing here computes collision results on the CPU.

    import vamp_amd as vamp
    env = vamp.Environment()
    env.add_sphere(vamp.Sphere([0.5, 0.0, 0.3], 0.2))
    vamp.panda.validate(q, env)                      # one configuration (bindings/common.hh:172-190)
    ok, n = vamp.panda_0_0.validate_batch(starts, goals, env)   # N edges, validate_motion each
"""
from __future__ import annotations

import ctypes as C
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import VgpuError, check, load

__all__ = [
    "Context", "context", "Environment", "Attachment", "Sphere", "Cuboid", "Cylinder", "HeightField", "make_heightfield", "Robot", "halton", "compact_device",
    "PandaBase", "panda", "panda_0_0", "VgpuError",
]


def _f3(v) -> C.Array:
    a = (C.c_float * 3)(*[float(np.float32(x)) for x in v])
    return a


class Context:
    """One HIP device + stream (vgpu_ctx).  Probes the host rsqrt approximation on creation."""

    def __init__(self, device: int = 0):
        lib = load()
        h = C.c_void_p()
        rc = lib.vgpu_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise VgpuError(f"vgpu_ctx_create(device={device}) failed: {_lib.ERRORS.get(rc, rc)}")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            load().vgpu_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(load().vgpu_sync(self.h), self.h)

    def set_stream(self, stream_handle: Optional[int]):
        check(load().vgpu_ctx_set_stream(self.h, C.c_void_p(stream_handle or 0)), self.h)

    def set_profiling(self, enable: bool):
        check(load().vgpu_ctx_set_profiling(self.h, int(bool(enable))), self.h)

    def phase_times(self) -> dict:
        """Accumulated ms of vgpu_validate_motions phases since the last call (then reset)."""
        out = (C.c_float * 4)()
        check(load().vgpu_phase_times(self.h, out), self.h)
        return {"head_ms": out[0], "scan_ms": out[1], "tail_ms": out[2], "calls": int(out[3])}

    def rsqrt_table(self) -> Tuple[np.ndarray, int]:
        k = C.c_int()
        p = _lib.U32P()
        check(load().vgpu_rsqrt_table(self.h, C.byref(k), C.byref(p)), self.h)
        n = 2 << k.value
        return np.ctypeslib.as_array(p, shape=(n,)).copy(), k.value

    def set_rsqrt_table(self, table: np.ndarray, kbits: int):
        t = np.ascontiguousarray(table, np.uint32)
        check(load().vgpu_rsqrt_table_set(self.h, t.ctypes.data_as(_lib.U32P), int(kbits)), self.h)


_contexts: Dict[int, Context] = {}


def context(device: int = 0) -> Context:
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]


# ---- shapes (collision/shapes.hh, factory.hh) ---------------------------------------------
class Sphere:
    """vamp.Sphere(center, radius) (bindings/environment.cc:20-25)."""

    def __init__(self, center: Sequence[float], radius: float):
        self.center = [float(c) for c in center]
        self.r = float(radius)
        self.name = ""

    @property
    def x(self):
        return self.center[0]

    @property
    def y(self):
        return self.center[1]

    @property
    def z(self):
        return self.center[2]

    @property
    def position(self):
        return list(self.center)

    def __repr__(self):
        return f"Sphere({self.center}, {self.r})"


class Cuboid:
    """vamp.Cuboid(center, euler_xyz, half_extents) (bindings/environment.cc:70-76); use
    Cuboid.from_axes for resolved axes (the Euler->axes step of factory.hh:26-60 goes through
    Eigen in the reference and is restated here without bit-parity)."""

    def __init__(self, center, euler_xyz=None, half_extents=None, axes=None):
        self.center = [float(c) for c in center]
        self.euler = None if euler_xyz is None else [float(e) for e in euler_xyz]
        self.half = [float(h) for h in half_extents]
        self.axes = axes
        self.name = ""

    @classmethod
    def from_axes(cls, center, axis_1, axis_2, axis_3, half_extents):
        return cls(center, None, half_extents, axes=[list(axis_1), list(axis_2), list(axis_3)])


class Cylinder:
    """vamp.Cylinder(center, euler_xyz, radius, length) or vamp.Cylinder(endpoint1, endpoint2,
    radius) (bindings/environment.cc:37-52); added to environments as capsules."""

    def __init__(self, a, b, radius, length=None):
        if length is None:
            self.p1, self.p2, self.r = [float(v) for v in a], [float(v) for v in b], float(radius)
            self.center = None
        else:
            self.center, self.euler, self.r, self.length = ([float(v) for v in a], [float(v) for v in b],
                                                            float(radius), float(length))
        self.name = ""


class HeightField:
    """collision::HeightField<float> as made by vamp.make_heightfield(center, scale,
    dimensions, data) (bindings/environment.cc:96-105, factory.hh:365-423): reciprocal scales
    xs/ys/zs = 1/scale, data row-major with dimensions (xd, yd)."""

    def __init__(self, center, scale, dimensions, data):
        self.center = [float(v) for v in center]
        self.scale = [float(v) for v in scale]
        self.xd, self.yd = int(dimensions[0]), int(dimensions[1])
        self.data = np.ascontiguousarray(data, np.float32).ravel()
        if self.data.size != self.xd * self.yd:
            raise ValueError("heightfield data must hold dimensions[0] * dimensions[1] values")
        self.x, self.y, self.z = (np.float32(v) for v in self.center)
        self.xs, self.ys, self.zs = (np.float32(1.0) / np.float32(v) for v in self.scale)


def make_heightfield(center, scale, dimensions, data) -> HeightField:
    return HeightField(center, scale, dimensions, data)


class _PointCloud:
    def __init__(self, points, r_min, r_max, r_point):
        self.points = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
        self.r_min, self.r_max, self.r_point = float(r_min), float(r_max), float(r_point)


class Attachment:
    """collision::Attachment<float> (collision/attachments.hh:14-123; bindings/environment.cc:197-249):
    spheres rigidly attached at a frame relative to the end effector."""

    def __init__(self, center: Sequence[float], quaternion_xyzw: Sequence[float]):
        self.tf = np.array(list(center) + list(quaternion_xyzw), np.float32)
        if self.tf.shape != (7,):
            raise ValueError("center[3] and quaternion_xyzw[4]")
        self.spheres: List[Sphere] = []
        self.posed_spheres: List[Sphere] = []

    @property
    def relative_frame(self):
        return (self.tf[:3].tolist(), self.tf[3:].tolist())

    def add_sphere(self, sphere: Sphere):
        self.spheres.append(sphere)

    def add_spheres(self, spheres: Sequence[Sphere]):
        self.spheres.extend(spheres)

    def set_ee_pose(self, position: Sequence[float], quaternion_xyzw: Sequence[float]):
        """Attachment::pose (attachments.hh:75-122) on the host, float32 left to right (the
        kernels' att_pose / att_sphere): fills posed_spheres."""
        F = np.float32
        ptx, pty, ptz = (F(v) for v in position)
        prx, pry, prz, prw = (F(v) for v in quaternion_xyzw)
        ttx, tty, ttz, trx, try_, trz, trw = (F(v) for v in self.tf)
        two, one = F(2.0), F(1.0)
        with np.errstate(all="ignore"):
            rx = prw * trx + prx * trw + pry * trz - prz * try_
            ry = prw * try_ - prx * trz + pry * trw + prz * trx
            rz = prw * trz + prx * try_ - pry * trx + prz * trw
            rw = prw * trw - prx * trx - pry * try_ - prz * trz
            x0, x1, x2 = pry * ttz - prz * tty, prx * tty - pry * ttx, prx * ttz - prz * ttx
            tx = ptx + two * (prw * x0 + pry * x1 + prz * x2) + ttx
            ty = pty + two * (-prw * x2 - prx * x1 + prz * x0) + tty
            tz = ptz + two * (prw * x1 - prx * x2 - pry * x0) + ttz
            b0, b1, b2, b3, b4 = ry * ry, rz * rz, rw * rz, rw * ry, rx * rx
            b5, b6, b7, b8 = rw * rx, rx * ry, rx * rz, ry * rz
            xx, xy, xz = -two * (b0 + b1) + one, two * (b6 + b2), two * (b7 - b3)
            yx, yy, yz = two * (b6 - b2), -two * (b1 + b4) + one, two * (b8 + b5)
            zx, zy, zz = two * (b7 + b3), two * (b8 - b5), -two * (b0 + b4) + one
            self.posed_spheres = []
            for s in self.spheres:
                x, y, z = (F(v) for v in s.center)
                self.posed_spheres.append(Sphere((x * xx + y * yx + z * zx + tx, x * xy + y * yy + z * zy + ty,
                                                  x * xz + y * yz + z * zz + tz), s.r))

    def _rows(self) -> np.ndarray:
        return np.array([list(s.center) + [s.r] for s in self.spheres], np.float32).reshape(-1, 4)


_ENVS = weakref.WeakSet()  # live environments (the debug build's bounds-check fixture reads their copies)


class Environment:
    """collision::Environment<float> (environment.hh:12-82) realised lazily per Context."""

    def __init__(self):
        _ENVS.add(self)
        self._ops: List[Tuple[str, object]] = []
        self._handles: Dict[int, C.c_void_p] = {}
        self._host: Optional[C.c_void_p] = None  # host-only twin holding the built CAPTs
        self._n_clouds = 0  # point clouds in the twin (built once; realised by copying their arrays)

    def _changed(self):
        """Drop every realised copy (the next use re-creates it from the op list)."""
        for dev, h in list(self._handles.items()):
            load().vgpu_env_destroy(h)
        self._handles.clear()

    def _apply_live(self, op):
        """Apply one op to every realised copy in place: the library re-sends only the section it touches
        (vgpu_env_upload: obstacles / attachment in the blob's tail; the point clouds and their cell grids
        stay on the device unless a cloud is added)."""
        lib = load()
        for key, h in list(self._handles.items()):
            self._apply(lib, h, None, op)

    def _push(self, op):
        """Apply op to every realised copy, then record it.  If it fails on some copy (an invalid shape),
        every copy is dropped and the op is not recorded: the copies cannot diverge, and later contexts
        realise the environment without it."""
        try:
            self._apply_live(op)
        except Exception:
            self._changed()
            raise
        self._ops.append(op)

    def add_sphere(self, s: Sphere):
        self._push(("sphere", s))

    def add_cuboid(self, c: Cuboid):
        self._push(("cuboid", c))

    def add_capsule(self, c: Cylinder):
        self._push(("capsule", c))

    def add_heightfield(self, h: HeightField):
        self._push(("heightfield", h))

    def attach(self, a: Attachment):
        """Environment.attach (bindings/environment.cc:161-162): validate_motion then checks its
        first rake block through Robot::fkcc_attach (planning/validate.hh:43)."""
        self._ops = [op for op in self._ops if op[0] != "attach"]
        self._push(("attach", (a.tf.copy(), a._rows())))

    def detach(self):
        """Environment.detach (bindings/environment.cc:163)."""
        self._ops = [op for op in self._ops if op[0] != "attach"]
        self._apply_live(("detach", None))

    def upload_stats(self, ctx: Optional["Context"] = None) -> dict:
        """vgpu_env_upload_stats of the copy on ctx: whole-blob uploads, tail-only uploads, cell-grid builds."""
        ctx = ctx or context()
        out = (C.c_uint64 * 3)()
        check(load().vgpu_env_upload_stats(self.handle(ctx), out), ctx.h)
        return {"full": int(out[0]), "tail": int(out[1]), "grids": int(out[2])}

    @property
    def attached(self) -> bool:
        return any(op[0] == "attach" for op in self._ops)

    def _host_env(self):
        if self._host is None:
            h = C.c_void_p()
            check(load().vgpu_env_create(None, C.byref(h)))
            self._host = h
        return self._host

    def add_pointcloud(self, points, r_min: float, r_max: float, r_point: float) -> int:
        """Environment::add_pointcloud (bindings/environment.cc:148-158): builds a CAPT once (host
        twin) and returns the build time in nanoseconds; device environments copy its arrays."""
        pc = _PointCloud(points, r_min, r_max, r_point)
        host = self._host_env()
        ns = C.c_int64()
        check(load().vgpu_env_add_pointcloud(host, pc.points.ctypes.data_as(_lib.F32P), pc.points.shape[0],
                                             pc.r_min, pc.r_max, pc.r_point, C.byref(ns)))
        self._n_clouds += 1
        self._push(("pointcloud", self._n_clouds - 1))
        return int(ns.value)

    def add_pointcloud_device(self, points_ptr: int, n: int, r_min: float, r_max: float, r_point: float,
                              ctx: Optional[Context] = None) -> int:
        """Environment::add_pointcloud with the CAPT built on the GPU (vgpu_capt_build.hip) from
        DEVICE points (n x 3 float32, e.g. a filtered cloud already in HBM); the same arrays as
        add_pointcloud.  The built arrays are kept in the host twin, so the points need not stay
        alive and every context's environment copies them (no rebuild).  Returns the build time in ns."""
        ctx = ctx or context()
        host = self._host_env()
        ns = C.c_int64()
        args = (C.c_void_p(int(points_ptr)), int(n), float(r_min), float(r_max), float(r_point))
        check(load().vgpu_env_add_pointcloud_device(ctx.h, host, *args, C.byref(ns)), ctx.h)
        self._n_clouds += 1
        self._push(("pointcloud", self._n_clouds - 1))
        return int(ns.value)

    def pointcloud_arrays(self, index: int = 0) -> dict:
        """The built CAPT's arrays (tests, aabbs, aff_starts, affordances [n][3][8], top box)."""
        lib = load()
        n2, na, top = C.c_int32(), C.c_size_t(), (C.c_float * 6)()
        check(lib.vgpu_env_pointcloud_info(self._host, index, C.byref(n2), C.byref(na), top))
        m = 1 << n2.value
        tests = np.zeros(max(m - 1, 0), np.float32)
        aabbs = np.zeros((m, 6), np.float32)
        starts = np.zeros(m + 1, np.uint32)
        aff = np.zeros((na.value, 3, 8), np.float32)
        check(lib.vgpu_env_pointcloud_arrays(self._host, index, tests.ctypes.data_as(_lib.F32P),
                                             aabbs.ctypes.data_as(_lib.F32P), starts.ctypes.data_as(_lib.U32P),
                                             aff.ctypes.data_as(_lib.F32P)))
        return {"nlog2": n2.value, "tests": tests, "aabbs": aabbs, "aff_starts": starts, "aff": aff,
                "aabb_top": np.array(top[:], np.float32)}

    def pointcloud_collides(self, centers, radii, index: int = 0, simd: bool = False,
                            ctx: Optional[Context] = None) -> np.ndarray:
        """Raw sphere queries on the GPU: CAPT::collides (capt.hh:403-443), or with simd=True
        one lane of CAPT::collides_simd (capt.hh:457-541)."""
        ctx = ctx or context()
        c = np.ascontiguousarray(centers, np.float32).reshape(-1, 3)
        r = np.ascontiguousarray(radii, np.float32).ravel()
        if r.shape[0] != c.shape[0]:
            raise ValueError("one radius per centre")
        out = np.zeros(c.shape[0], np.uint8)
        check(load().vgpu_pointcloud_collides_host(ctx.h, self.handle(ctx), index, c.ctypes.data_as(_lib.F32P),
                                                   r.ctypes.data_as(_lib.F32P), c.shape[0], int(simd),
                                                   out.ctypes.data_as(_lib.U8P)), ctx.h)
        return out.astype(bool)

    def pointcloud_collides_device(self, centers_ptr: int, radii_ptr: int, n: int, out_ptr: int, index: int = 0,
                                   simd: bool = False, ctx: Optional[Context] = None):
        ctx = ctx or context()
        check(load().vgpu_pointcloud_collides(ctx.h, self.handle(ctx), index, centers_ptr, radii_ptr, n, int(simd),
                                              out_ptr), ctx.h)

    def handle(self, ctx: Context) -> C.c_void_p:
        """This environment realised on ctx (one device copy per context, rebuilt after a change)."""
        key = ctx.h.value  # per context: two contexts may share a device
        if key in self._handles:
            return self._handles[key]
        lib = load()
        h = C.c_void_p()
        check(lib.vgpu_env_create(ctx.h, C.byref(h)), ctx.h)
        self._realise(lib, h, ctx.h)
        check(lib.vgpu_env_upload(h), ctx.h)
        self._handles[key] = h
        return h

    def host_handle(self) -> C.c_void_p:
        """A host-only twin (no context) for the CPU rake (vgpu_cpu_*)."""
        if "cpu" in self._handles:
            return self._handles["cpu"]
        lib = load()
        h = C.c_void_p()
        check(lib.vgpu_env_create(None, C.byref(h)))
        self._realise(lib, h, None)
        self._handles["cpu"] = h
        return h

    def _realise(self, lib, h, ctx_h):
        for op in self._ops:
            self._apply(lib, h, ctx_h, op)

    def _apply(self, lib, h, ctx_h, op):
        kind, s = op
        if kind == "detach":
            rc = lib.vgpu_env_detach(h)
        elif kind == "sphere":
            rc = lib.vgpu_env_add_sphere(h, _f3(s.center), float(np.float32(s.r)))
        elif kind == "cuboid":
            if s.axes is not None:
                rc = lib.vgpu_env_add_cuboid_axes(h, _f3(s.center), _f3(s.axes[0]), _f3(s.axes[1]),
                                                  _f3(s.axes[2]), _f3(s.half))
            else:
                rc = lib.vgpu_env_add_cuboid_euler(h, _f3(s.center), _f3(s.euler), _f3(s.half))
        elif kind == "heightfield":
            rc = lib.vgpu_env_add_heightfield(h, _f3(s.center), _f3(s.scale), s.xd, s.yd,
                                              s.data.ctypes.data_as(_lib.F32P))
        elif kind == "attach":
            tf, rows = s
            rows = np.ascontiguousarray(rows, np.float32)
            rc = lib.vgpu_env_attach(h, tf.ctypes.data_as(_lib.F32P), rows.ctypes.data_as(_lib.F32P),
                                     rows.shape[0])
        elif kind == "pointcloud":  # s = index of the cloud in the host twin
            rc = lib.vgpu_env_copy_pointcloud(h, self._host, int(s))
        else:
            if s.center is None:
                rc = lib.vgpu_env_add_capsule_endpoints(h, _f3(s.p1), _f3(s.p2), float(np.float32(s.r)))
            else:
                rc = lib.vgpu_env_add_capsule_euler(h, _f3(s.center), _f3(s.euler), float(np.float32(s.r)),
                                                    float(np.float32(s.length)))
        check(rc, ctx_h)

    def counts(self, ctx: Optional[Context] = None) -> List[int]:
        ctx = ctx or context()
        out = (C.c_int32 * 5)()
        check(load().vgpu_env_counts(self.handle(ctx), out), ctx.h)
        return list(out)

    def __del__(self):
        try:
            self._changed()
            if self._host is not None:
                load().vgpu_env_destroy(self._host)
                self._host = None
        except Exception:
            pass


# ---- sampling ---------------------------------------------------------------------------------
def filter_pointcloud_indices(pc, min_dist: float, max_range: float, origin, workspace_min, workspace_max,
                              cull: bool = True, ctx: Optional[Context] = None) -> np.ndarray:
    """Indices of the points vamp.filter_pointcloud keeps (collision/filter.hh:175-268), in its
    final space-filling-curve order, computed on the GPU (vgpu_filter.hip)."""
    ctx = ctx or context()
    pc = np.ascontiguousarray(pc, np.float32).reshape(-1, 3)
    out = np.zeros(max(pc.shape[0], 1), np.uint32)
    cnt = C.c_size_t(0)
    o, lo, up = (np.ascontiguousarray(v, np.float32).reshape(3) for v in (origin, workspace_min, workspace_max))
    check(load().vgpu_filter_pointcloud_host(ctx.h, pc.ctypes.data_as(_lib.F32P), pc.shape[0], float(min_dist),
                                             float(max_range), o.ctypes.data_as(_lib.F32P),
                                             lo.ctypes.data_as(_lib.F32P), up.ctypes.data_as(_lib.F32P), int(cull),
                                             out.ctypes.data_as(_lib.U32P), C.byref(cnt)), ctx.h)
    return out[:cnt.value].copy()


def filter_pointcloud(pc, min_dist: float, max_range: float, origin, workspace_min, workspace_max,
                      cull: bool = True, ctx: Optional[Context] = None) -> np.ndarray:
    """vamp.filter_pointcloud (bindings/common.hh, collision/filter.hh:175-268): the kept points."""
    pc = np.ascontiguousarray(pc, np.float32).reshape(-1, 3)
    return pc[filter_pointcloud_indices(pc, min_dist, max_range, origin, workspace_min, workspace_max, cull, ctx)]


def halton(dim: int, first: int, n: int, ctx: Optional[Context] = None) -> np.ndarray:
    """rng::Halton<dim>::next draws first .. first+n-1 (1-based) of a fresh sampler, on the GPU."""
    ctx = ctx or context()
    out = np.empty((n, dim), np.float32)
    check(load().vgpu_halton_host(ctx.h, dim, first, n, out.ctypes.data_as(_lib.F32P)), ctx.h)
    return out


def compact_device(rows_ptr: int, valid_ptr: int, n: int, dim: int, rows_out_ptr: int, index_out_ptr: int,
                   ctx: Optional[Context] = None) -> int:
    """Stream compaction on the device (selected row indices ascending); returns the count."""
    ctx = ctx or context()
    cnt = C.c_size_t()
    check(load().vgpu_compact(ctx.h, C.c_void_p(rows_ptr or 0), C.c_void_p(valid_ptr), n, dim,
                              C.c_void_p(rows_out_ptr or 0), C.c_void_p(index_out_ptr), C.byref(cnt)), ctx.h)
    return int(cnt.value)


# ---- planning (RRT-Connect on the CPU rake: BASELINE configs[0]) -------------------------------
class RRTCSettings:
    """vamp::planning::RRTCSettings (planning/rrtc_settings.hh:5-20), same field names/defaults."""

    def __init__(self, **kw):
        self.range = 2.0
        self.dynamic_domain = True
        self.radius = 4.0
        self.alpha = 0.0001
        self.min_radius = 1.0
        self.balance = True
        self.tree_ratio = 1.0
        self.max_iterations = 100000
        self.max_samples = 100000
        self.start_tree_first = True
        for k, v in kw.items():
            if not hasattr(self, k):
                raise AttributeError(k)
            setattr(self, k, v)

    def c(self) -> _lib.VgpuRrtcSettings:
        return _lib.VgpuRrtcSettings(float(self.range), int(self.dynamic_domain), float(self.radius),
                                     float(self.alpha), float(self.min_radius), int(self.balance),
                                     float(self.tree_ratio), int(self.max_iterations), int(self.max_samples),
                                     int(self.start_tree_first))


class Halton:
    """rng::Halton<dim> (random/halton.hh) as the planners consume it: vamp.<robot>.halton() with
    reset() / skip(n) / next(); the state is the 1-based index of the next draw."""

    def __init__(self, dim: int):
        self.dim = dim
        self.index = 1

    def reset(self):
        self.index = 1

    def skip(self, n: int):
        self.index += int(n)


class PRMNeighborParams:
    """vamp.PRMNeighborParams(dim, space_measure) = planning::PRMStarNeighborParams (roadmap.hh:42-77,
    bindings/settings.cc:38-44): PRM* k(n) = ceil((e + e/dim) ln n), r(n) from the space measure,
    gamma_scale 2.0."""

    def __init__(self, dim: int, space_measure: float):
        self.dim = int(dim)
        self.space_measure = float(space_measure)
        self.gamma_scale = 2.0

    def _kr(self, num_states: int):
        from .roadmap import prm_neighbor_params
        k, r = prm_neighbor_params(self.dim, self.space_measure, int(num_states) + 1, self.gamma_scale)
        return int(k[num_states]), float(r[num_states])

    def max_neighbors(self, num_states: int) -> int:
        return self._kr(num_states)[0]

    def neighbor_radius(self, num_states: int) -> float:
        return self._kr(num_states)[1]


class PRMSettings:
    """vamp.PRMSettings(neighbor_params) = RoadmapSettings<PRMStarNeighborParams> (roadmap.hh:150-171,
    bindings/settings.cc:46-53): max_iterations = max_samples = 100000 by default."""

    def __init__(self, neighbor_params: PRMNeighborParams):
        self.neighbor_params = neighbor_params
        self.max_iterations = 100000
        self.max_samples = 100000

    def max_neighbors(self, num_states: int) -> int:
        return self.neighbor_params.max_neighbors(num_states)

    def neighbor_radius(self, num_states: int) -> float:
        return self.neighbor_params.neighbor_radius(num_states)


class PlanningResult:
    """vamp::planning::PlanningResult (planning/plan.hh): path, cost, iterations, size, nanoseconds."""

    def __init__(self, path, cost, iterations, size, nanoseconds, solved):
        self.path, self.cost, self.iterations = path, cost, iterations
        self.size, self.nanoseconds, self.solved = size, nanoseconds, solved


# ---- robots -----------------------------------------------------------------------------------
# Robot::space_measure of each robot: the reference's generated constant returned as float
# (panda/fk.hh:88-91 "-> float"), values as extracted into model/<robot>.json; the composite is
# two Pandas (product)
_SPACE_MEASURE = {k: float(np.float32(v)) for k, v in {
    _lib.VGPU_ROBOT_PANDA: 878819.1112640093, _lib.VGPU_ROBOT_FETCH: 269832.2635954135,
    _lib.VGPU_ROBOT_UR5: 700852.7173113511, _lib.VGPU_ROBOT_BAXTER: 89641415145.821,
    _lib.VGPU_ROBOT_PANDA_PAIR: 878819.1112640093 ** 2}.items()}


class Robot:
    """Python face of a vamp::robots robot: PandaBase<X100, Y100, Z100>
    (robots/panda_base.hh:15-75) or Fetch (robots/fetch.hh:8-48)."""

    # scale_configuration q * s_m + s_a, descale (q - s_a) * d_m (panda/fk.hh:14-62, fetch/fk.hh:20-97)
    _SCALE = {
        _lib.VGPU_ROBOT_PANDA: (
            [5.9342, 3.6652, 5.9342, 3.2289, 5.9342, 3.9095999999999997, 5.9342],
            [-2.9671, -1.8326, -2.9671, -3.1416, -2.9671, -0.0873, -2.9671],
            [0.1685147113342995, 0.2728364072901888, 0.1685147113342995, 0.30970299482796, 0.1685147113342995,
             0.25578064252097404, 0.1685147113342995]),
        _lib.VGPU_ROBOT_UR5: (
            [6.2831853, 6.2831853, 6.2831853, 6.2831853, 6.2831853, 6.2831853],
            [-3.14159265, -3.14159265, -3.14159265, -3.14159265, -3.14159265, -3.14159265],
            [0.15915494327375637, 0.15915494327375637, 0.15915494327375637, 0.15915494327375637, 0.15915494327375637, 0.15915494327375637]),
        _lib.VGPU_ROBOT_BAXTER: (
            [3.40335987756, 3.194, 6.10835987756, 2.6679999999999997, 6.118, 3.66479632679, 6.118, 3.40335987756, 3.194, 6.10835987756, 2.6679999999999997, 6.118, 3.66479632679, 6.118],
            [-1.70167993878, -2.147, -3.05417993878, -0.05, -3.059, -1.57079632679, -3.059, -1.70167993878, -2.147, -3.05417993878, -0.05, -3.059, -1.57079632679, -3.059],
            [0.2938272871445316, 0.31308703819661865, 0.16371006621166082, 0.37481259370314846, 0.16345210853220005, 0.2728664599148137, 0.16345210853220005, 0.2938272871445316, 0.31308703819661865, 0.16371006621166082, 0.37481259370314846, 0.16345210853220005, 0.2728664599148137, 0.16345210853220005]),
        _lib.VGPU_ROBOT_FETCH: (
            [0.38615, 3.2112, 2.739, 6.28318, 4.502, 6.28318, 4.32, 6.28318],
            [0.0, -1.6056, -1.221, -3.14159, -2.251, -3.14159, -2.16, -3.14159],
            [2.589667227761233, 0.31141006477329347, 0.36509675063891933, 0.15915507752443828,
             0.22212350066637052, 0.15915507752443828, 0.23148148148148145, 0.15915507752443828]),
    }

    def __init__(self, name: str, base_x100: int, base_y100: int, base_z100: int, kind: int = _lib.VGPU_ROBOT_PANDA,
                 base2=(0, 0, 0)):
        self.name = name
        self.c_robot = _lib.VgpuRobot(kind, base_x100, base_y100, base_z100, *base2)
        self._info = None
        self.kind = kind
        if kind == _lib.VGPU_ROBOT_PANDA_PAIR:  # both arms' scaling, concatenated
            sm, sa, dm = (a + a for a in self._SCALE[_lib.VGPU_ROBOT_PANDA])
        else:
            sm, sa, dm = self._SCALE[kind]
        self.S_M = np.array(sm, np.float32)
        self.S_A = np.array(sa, np.float32)
        self.D_M = np.array(dm, np.float32)
        self.radii = {_lib.VGPU_ROBOT_PANDA: _PANDA_RADII, _lib.VGPU_ROBOT_FETCH: _FETCH_RADII,
                      _lib.VGPU_ROBOT_UR5: _UR5_RADII, _lib.VGPU_ROBOT_BAXTER: _BAXTER_RADII}.get(
            kind, np.concatenate([_PANDA_RADII, _PANDA_RADII]))

    def _meta(self):
        if self._info is None:
            dim, res, ns = C.c_int32(), C.c_int32(), C.c_int32()
            check(load().vgpu_robot_info(self.kind, C.byref(dim), C.byref(res), C.byref(ns)))
            self._info = (dim.value, res.value, ns.value)
        return self._info

    def dimension(self) -> int:
        return self._meta()[0]

    def resolution(self) -> int:
        return self._meta()[1]

    def space_measure(self) -> float:
        """Robot::space_measure (robots/panda_base.hh:22 -> panda/fk.hh; fetch.hh:14): the product
        of the joint ranges, the PRMNeighborParams input (src/vamp/__init__.py:91)."""
        return _SPACE_MEASURE[self.kind]

    def n_spheres(self) -> int:
        return self._meta()[2]

    @property
    def base(self):
        r = self.c_robot
        return (np.float32(r.base_x100) / np.float32(100), np.float32(r.base_y100) / np.float32(100),
                np.float32(r.base_z100) / np.float32(100))

    # --- scaling (robots/panda/fk.hh:34-62) ---
    def scale_configuration(self, u):
        u = np.asarray(u, np.float32)
        return (u.astype(np.float64) * self.S_M + self.S_A).astype(np.float32)

    def descale_configuration(self, q):
        q = np.asarray(q, np.float32)
        return ((q - self.S_A) * self.D_M).astype(np.float32)

    # --- reference-named single calls: the CPU rake (host AVX2, csrc/cpu/), as the reference's
    # single-edge entry points stay on the CPU (a GPU launch costs far more than one edge) ---
    def fk(self, configuration) -> List[Sphere]:
        """vamp.<robot>.fk(q) (bindings/common.hh:132-152): the collision spheres."""
        q = np.asarray(configuration, np.float32).reshape(self.dimension())
        xyz = self.cpu_sphere_fk_block(np.repeat(q[:, None], 8, axis=1))[:, :, 0].T
        radii = self.radii
        return [Sphere(xyz[s], float(radii[s])) for s in range(xyz.shape[0])]

    def validate(self, configuration, environment: Environment) -> bool:
        """vamp.<robot>.validate(q, env) (bindings/common.hh:172-190): bounds check in the
        descaled unit box, then validate_motion<Robot, rake, 1>(q, q, env) -- one broadcast block,
        through fkcc_attach when the environment has an attachment (validate.hh:43)."""
        q = np.asarray(configuration, np.float32).reshape(self.dimension())
        d = self.descale_configuration(q)
        if not ((d <= 1.0).all() and (d >= 0.0).all()):
            return False
        return self.validate_motion(q, q, environment)

    def filter_from_pointcloud(self, pointcloud, configuration, environment: Environment, point_radius: float,
                               ctx: Optional[Context] = None) -> np.ndarray:
        """vamp.<robot>.filter_from_pointcloud(pointcloud, configuration, environment, point_radius)
        (bindings/common.hh:36-87,713): the points that neither overlap the robot's spheres at
        `configuration` nor collide with the environment, in input order, as float32 [m][3] -- on
        the GPU (sphere_fk + one lane per point, vgpu_filter_robot_pointcloud_host)."""
        ctx = ctx or context()
        pc = np.ascontiguousarray(pointcloud, np.float32).reshape(-1, 3)
        q = np.ascontiguousarray(configuration, np.float32).reshape(self.dimension())
        out = np.empty((max(pc.shape[0], 1), 3), np.float32)
        cnt = C.c_size_t(0)
        check(load().vgpu_filter_robot_pointcloud_host(ctx.h, C.byref(self.c_robot), environment.handle(ctx),
                                                       q.ctypes.data_as(_lib.F32P), pc.ctypes.data_as(_lib.F32P),
                                                       pc.shape[0], float(point_radius), out.ctypes.data_as(_lib.F32P),
                                                       C.byref(cnt)), ctx.h)
        return out[:cnt.value].copy()

    def filter_from_pointcloud_device(self, pc_ptr: int, n: int, configuration, environment: Environment,
                                      point_radius: float, keep_ptr: int, ctx: Optional[Context] = None):
        """Device form: pc[n][3] (device) -> keep[n] (device uint8, 1 = kept), stream-ordered."""
        ctx = ctx or context()
        q = np.ascontiguousarray(configuration, np.float32).reshape(self.dimension())
        check(load().vgpu_filter_robot_pointcloud(ctx.h, C.byref(self.c_robot), environment.handle(ctx),
                                                  q.ctypes.data_as(_lib.F32P), C.c_void_p(pc_ptr), int(n),
                                                  float(point_radius), C.c_void_p(keep_ptr)), ctx.h)

    def validate_motion(self, start, goal, environment: Environment) -> bool:
        """planning::validate_motion<Robot, 8, resolution> (planning/validate.hh:67-75)."""
        s = np.ascontiguousarray(start, np.float32).reshape(self.dimension())
        g = np.ascontiguousarray(goal, np.float32).reshape(self.dimension())
        v = C.c_int()
        check(load().vgpu_cpu_validate_motion(C.byref(self.c_robot), environment.host_handle(),
                                              s.ctypes.data_as(_lib.F32P), g.ctypes.data_as(_lib.F32P), C.byref(v)))
        return bool(v.value)

    def eefk(self, configuration):
        """vamp.<robot>.eefk(q) (bindings/common.hh:342-352): (position [3], quaternion x y z w [4])."""
        p = self.eefk_batch(np.asarray(configuration, np.float32)[None])[0]
        return p[:3].copy(), p[3:].copy()

    def eefk_batch(self, q) -> np.ndarray:
        """Robot::eefk of each q[n][dim]: [n][7] (x y z, qx qy qz qw), robot frame."""
        q = np.ascontiguousarray(q, np.float32).reshape(-1, self.dimension())
        out = np.empty((q.shape[0], 7), np.float32)
        check(load().vgpu_cpu_eefk(C.byref(self.c_robot), q.ctypes.data_as(_lib.F32P), q.shape[0],
                                   out.ctypes.data_as(_lib.F32P)))
        return out

    def halton(self) -> Halton:
        """vamp.<robot>.halton(): a fresh Halton<dimension> sampler."""
        return Halton(self.dimension())

    def rrtc(self, start, goals, environment: Environment, settings: Optional[RRTCSettings] = None,
             rng: Optional[Halton] = None) -> PlanningResult:
        """vamp.<robot>.rrtc(start, goal(s), env, settings, rng) (bindings/common.hh:191-200 ->
        planning/rrtc.hh:33-248) on the CPU rake; rng advances by the draws taken."""
        dim = self.dimension()
        s = np.ascontiguousarray(start, np.float32).reshape(dim)
        g = np.ascontiguousarray(goals, np.float32).reshape(-1, dim)
        settings = settings or RRTCSettings()
        rng = rng or self.halton()
        idx = C.c_uint64(rng.index)
        res = _lib.VgpuPlanResult()
        cap = 4096
        while True:
            path = np.empty((cap, dim), np.float32)
            i0 = C.c_uint64(idx.value)
            rc = load().vgpu_cpu_rrtc(C.byref(self.c_robot), environment.host_handle(), s.ctypes.data_as(_lib.F32P),
                                      g.ctypes.data_as(_lib.F32P), g.shape[0], C.byref(settings.c()), C.byref(i0),
                                      path.ctypes.data_as(_lib.F32P), cap, C.byref(res))
            if rc == _lib.VGPU_OK or res.path_len <= cap:
                check(rc)
                idx = i0
                break
            cap = int(res.path_len)
        rng.index = int(idx.value)
        return PlanningResult(path[:res.path_len].copy(), float(res.cost), int(res.iterations),
                              (int(res.size[0]), int(res.size[1])), int(res.nanoseconds), bool(res.solved))

    def roadmap(self, start, goal, environment: Environment, settings: Optional[PRMSettings] = None,
                rng: Optional[Halton] = None, ctx: Optional[Context] = None):
        """vamp.<robot>.roadmap(start, goal, environment, settings, rng) (bindings/common.hh:312-321,667 ->
        PRM::build_roadmap, planning/prm.hh:197-299) on the GPU: the sampler's draws rng.index ..
        rng.index + max_iterations - 1 through the fused Halton -> scale -> fkcc kernel (sharded over
        the ranks when torch.distributed is initialised), the vertex sequence start, goal, valid samples
        in draw order cut at max_samples, then every vertex's PRM* neighbour query and validate_motion
        of its candidates, adjacency in the reference's append order.  Returns a Roadmap with
        vertices, edges, nanoseconds and iterations (= draws taken + 1, the reference loop's count);
        rng advances by the draws taken."""
        import time

        from . import roadmap as _rm
        settings = settings or PRMSettings(PRMNeighborParams(self.dimension(), self.space_measure()))
        rng = rng or self.halton()
        dim = self.dimension()
        s = np.ascontiguousarray(start, np.float32).reshape(dim)
        g = np.ascontiguousarray(goal, np.float32).reshape(dim)
        t0 = time.perf_counter_ns()
        max_it, max_s = int(settings.max_iterations), int(settings.max_samples)
        rows, draws = _rm.roadmap_vertices(self, environment, max_it, rng.index, s, g, max(max_s, 2), ctx)
        draws = draws.cpu().numpy()
        taken = max_it
        if max_s <= 2:  # the loop never draws (nodes.size() < max_samples fails at once)
            taken = 0
        elif len(draws) >= max_s:  # the last vertex's draw ends the loop
            taken = int(draws[max_s - 1]) - rng.index + 1
        rm = _rm.build_roadmap_edges(self, environment, rows.cpu().numpy(),
                                     settings.neighbor_params.gamma_scale, settings.neighbor_params.space_measure,
                                     ctx)
        rng.skip(taken)
        rm.nanoseconds = time.perf_counter_ns() - t0
        rm.iterations = taken + 1
        return rm

    def cpu_validate_vector(self, start, vector, distance: float, environment: Environment) -> bool:
        """planning::validate_vector<Robot, 8, resolution>(start, vector, distance, env)."""
        s = np.ascontiguousarray(start, np.float32).reshape(self.dimension())
        v = np.ascontiguousarray(vector, np.float32).reshape(self.dimension())
        ok = C.c_int()
        check(load().vgpu_cpu_validate_vector(C.byref(self.c_robot), environment.host_handle(),
                                              s.ctypes.data_as(_lib.F32P), v.ctypes.data_as(_lib.F32P),
                                              float(np.float32(distance)), C.byref(ok)))
        return bool(ok.value)

    # --- CPU rake batches and blocks (host numpy in/out; threads <= 0: every hardware thread) ---
    def cpu_fkcc_block(self, block, environment: Environment, attach: bool = False) -> bool:
        """Robot::fkcc<8>(env, block) / fkcc_attach<8>: block = ConfigurationBlock<8> [dim][8]."""
        b = np.ascontiguousarray(block, np.float32).reshape(self.dimension(), 8)
        v = C.c_int()
        fn = load().vgpu_cpu_fkcc_attach_block if attach else load().vgpu_cpu_fkcc_block
        check(fn(C.byref(self.c_robot), environment.host_handle(), b.ctypes.data_as(_lib.F32P), C.byref(v)))
        return bool(v.value)

    def cpu_sphere_fk_block(self, block) -> np.ndarray:
        """Robot::sphere_fk<8>(block): [3][n_spheres][8] world-frame centres."""
        b = np.ascontiguousarray(block, np.float32).reshape(self.dimension(), 8)
        out = np.empty((3, self.n_spheres(), 8), np.float32)
        check(load().vgpu_cpu_sphere_fk_block(C.byref(self.c_robot), b.ctypes.data_as(_lib.F32P),
                                              out.ctypes.data_as(_lib.F32P)))
        return out

    def cpu_fkcc_batch(self, q, environment: Environment, threads: int = 0, attach: bool = False) -> np.ndarray:
        q = np.ascontiguousarray(q, np.float32).reshape(-1, self.dimension())
        out = np.empty(q.shape[0], np.uint8)
        fn = load().vgpu_cpu_fkcc_attach if attach else load().vgpu_cpu_fkcc
        check(fn(C.byref(self.c_robot), environment.host_handle(), q.ctypes.data_as(_lib.F32P), q.shape[0],
                 out.ctypes.data_as(_lib.U8P), int(threads)))
        return out.astype(bool)

    def cpu_validate_mask(self, starts, goals, environment: Environment, threads: int = 0):
        """Full-mask validate on the CPU rake: (ok, n_e, block_ok [sum n_e], block offsets [n+1])."""
        s = np.ascontiguousarray(starts, np.float32).reshape(-1, self.dimension())
        g = np.ascontiguousarray(goals, np.float32).reshape(-1, self.dimension())
        n = s.shape[0]
        ok = np.empty(n, np.uint8)
        nb = np.empty(n, np.int32)
        tot = C.c_size_t()
        lib = load()
        args = (C.byref(self.c_robot), environment.host_handle(), s.ctypes.data_as(_lib.F32P),
                g.ctypes.data_as(_lib.F32P), n, ok.ctypes.data_as(_lib.U8P), nb.ctypes.data_as(_lib.I32P))
        rc = lib.vgpu_cpu_validate_motions_mask(*args, None, 0, C.byref(tot), int(threads))
        if rc != _lib.VGPU_OK and tot.value == 0 and n:
            check(rc)
        blk = np.empty(max(tot.value, 1), np.uint8)
        check(lib.vgpu_cpu_validate_motions_mask(*args, blk.ctypes.data_as(_lib.U8P), blk.size, C.byref(tot),
                                                 int(threads)))
        off = np.concatenate([[0], np.cumsum(nb.astype(np.int64))])
        return ok.astype(bool), nb, blk[:tot.value].astype(bool), off

    def cpu_validate_batch(self, starts, goals, environment: Environment, threads: int = 0):
        """validate_motion of every edge on the CPU rake: (ok, n_e, blocks evaluated)."""
        s = np.ascontiguousarray(starts, np.float32).reshape(-1, self.dimension())
        g = np.ascontiguousarray(goals, np.float32).reshape(-1, self.dimension())
        if s.shape != g.shape:
            raise ValueError("starts and goals differ in shape")
        ok = np.empty(s.shape[0], np.uint8)
        nb = np.empty(s.shape[0], np.int32)
        ne = np.empty(s.shape[0], np.int32)
        check(load().vgpu_cpu_validate_motions(C.byref(self.c_robot), environment.host_handle(),
                                               s.ctypes.data_as(_lib.F32P), g.ctypes.data_as(_lib.F32P), s.shape[0],
                                               ok.ctypes.data_as(_lib.U8P), nb.ctypes.data_as(_lib.I32P),
                                               ne.ctypes.data_as(_lib.I32P), int(threads)))
        return ok.astype(bool), nb, ne

    # --- batches (host numpy in/out) ---
    def sphere_fk_batch(self, q, ctx: Optional[Context] = None) -> np.ndarray:
        ctx = ctx or context()
        q = np.ascontiguousarray(q, np.float32).reshape(-1, self.dimension())
        n = q.shape[0]
        ns = self.n_spheres()
        out = np.empty((3, ns, n), np.float32)
        check(load().vgpu_sphere_fk_host(ctx.h, C.byref(self.c_robot), q.ctypes.data_as(_lib.F32P), n,
                                         out.ctypes.data_as(_lib.F32P)), ctx.h)
        return np.ascontiguousarray(out.transpose(2, 1, 0))

    def fkcc_batch(self, q, environment: Environment, ctx: Optional[Context] = None) -> np.ndarray:
        ctx = ctx or context()
        q = np.ascontiguousarray(q, np.float32).reshape(-1, self.dimension())
        out = np.empty(q.shape[0], np.uint8)
        check(load().vgpu_fkcc_host(ctx.h, C.byref(self.c_robot), environment.handle(ctx),
                                    q.ctypes.data_as(_lib.F32P), q.shape[0], out.ctypes.data_as(_lib.U8P)), ctx.h)
        return out.astype(bool)

    def fkcc_attach_batch(self, q, environment: Environment, ctx: Optional[Context] = None) -> np.ndarray:
        """Robot::fkcc_attach per configuration (robots/panda_base.hh:61-65): the environment's
        attachment posed at each configuration's end effector."""
        ctx = ctx or context()
        q = np.ascontiguousarray(q, np.float32).reshape(-1, self.dimension())
        out = np.empty(q.shape[0], np.uint8)
        check(load().vgpu_fkcc_attach_host(ctx.h, C.byref(self.c_robot), environment.handle(ctx),
                                           q.ctypes.data_as(_lib.F32P), q.shape[0], out.ctypes.data_as(_lib.U8P)),
              ctx.h)
        return out.astype(bool)

    def validate_batch(self, starts, goals, environment: Environment, ctx: Optional[Context] = None):
        ctx = ctx or context()
        s = np.ascontiguousarray(starts, np.float32).reshape(-1, self.dimension())
        g = np.ascontiguousarray(goals, np.float32).reshape(-1, self.dimension())
        if s.shape != g.shape:
            raise ValueError("starts and goals differ in shape")
        ok = np.empty(s.shape[0], np.uint8)
        nb = np.empty(s.shape[0], np.int32)
        check(load().vgpu_validate_motions_host(ctx.h, C.byref(self.c_robot), environment.handle(ctx),
                                                s.ctypes.data_as(_lib.F32P), g.ctypes.data_as(_lib.F32P),
                                                s.shape[0], ok.ctypes.data_as(_lib.U8P),
                                                nb.ctypes.data_as(_lib.I32P)), ctx.h)
        return ok.astype(bool), nb

    # --- batches on device memory (raw pointers, e.g. torch tensor.data_ptr()) ---
    def sphere_fk_device(self, q_ptr: int, n: int, out_ptr: int, ld: int, ctx: Optional[Context] = None):
        ctx = ctx or context()
        check(load().vgpu_sphere_fk(ctx.h, C.byref(self.c_robot), C.c_void_p(q_ptr), n, C.c_void_p(out_ptr), ld),
              ctx.h)

    def sample_fkcc(self, first: int, n: int, environment: Environment, ctx: Optional[Context] = None):
        """Halton<dimension> draws first .. first+n-1 -> scale_configuration -> fkcc, fused on the
        GPU (the PRM sampling stage, prm.hh:236-251).  Returns (q [n, dim], valid [n])."""
        ctx = ctx or context()
        q = np.empty((n, self.dimension()), np.float32)
        ok = np.empty(n, np.uint8)
        check(load().vgpu_sample_fkcc_host(ctx.h, C.byref(self.c_robot), environment.handle(ctx), first, n,
                                           q.ctypes.data_as(_lib.F32P), ok.ctypes.data_as(_lib.U8P)), ctx.h)
        return q, ok.astype(bool)

    def sample_fkcc_device(self, first: int, n: int, environment: Environment, q_ptr: int, valid_ptr: int,
                           ctx: Optional[Context] = None):
        ctx = ctx or context()
        check(load().vgpu_sample_fkcc(ctx.h, C.byref(self.c_robot), environment.handle(ctx), first, n,
                                      C.c_void_p(q_ptr or 0), C.c_void_p(valid_ptr)), ctx.h)

    def fkcc_device(self, q_ptr: int, n: int, environment: Environment, valid_ptr: int,
                    ctx: Optional[Context] = None):
        ctx = ctx or context()
        check(load().vgpu_fkcc(ctx.h, C.byref(self.c_robot), environment.handle(ctx), C.c_void_p(q_ptr), n,
                               C.c_void_p(valid_ptr)), ctx.h)

    def validate_mask_device(self, starts_ptr: int, goals_ptr: int, n: int, environment: Environment, ok_ptr: int,
                             nblocks_ptr: int, block_ok_ptr: int, block_cap: int, ctx: Optional[Context] = None) -> int:
        """Full-mask validate (every rake block evaluated, each block's result kept): returns the
        number of blocks written to block_ok (edge-major, block 0 .. n_e - 1)."""
        ctx = ctx or context()
        total = C.c_size_t()
        check(load().vgpu_validate_motions_mask(ctx.h, C.byref(self.c_robot), environment.handle(ctx),
                                                C.c_void_p(starts_ptr), C.c_void_p(goals_ptr), n, C.c_void_p(ok_ptr),
                                                C.c_void_p(nblocks_ptr or 0), C.c_void_p(block_ok_ptr), block_cap,
                                                C.byref(total)), ctx.h)
        return int(total.value)

    def validate_device(self, starts_ptr: int, goals_ptr: int, n: int, environment: Environment, ok_ptr: int,
                        nblocks_ptr: int = 0, ctx: Optional[Context] = None):
        ctx = ctx or context()
        check(load().vgpu_validate_motions(ctx.h, C.byref(self.c_robot), environment.handle(ctx),
                                           C.c_void_p(starts_ptr), C.c_void_p(goals_ptr), n, C.c_void_p(ok_ptr),
                                           C.c_void_p(nblocks_ptr or 0)), ctx.h)


# robots/panda/fk.hh:113-171 sphere radii (reference order)
_PANDA_RADII = np.array(
    [0.08] + [0.06] * 9 + [0.05, 0.055, 0.055, 0.06, 0.055, 0.055, 0.055, 0.06, 0.06, 0.06, 0.05] + [0.025] * 8 +
    [0.05, 0.05, 0.052, 0.05, 0.025, 0.025, 0.02, 0.02] + [0.028] * 6 + [0.026] * 6 + [0.024] * 6 + [0.012] * 4,
    np.float32)


# robots/fetch/fk.hh:118-228 sphere radii (reference order)
_FETCH_RADII = np.array(
    [0.24, 0.066, 0.22] + [0.066] * 5 + [0.22] + [0.066] * 5 + [0.15] * 6 + [0.07, 0.15] + [0.05] * 5 + [0.03] * 22 +
    [0.055] * 4 + [0.04] * 4 + [0.055] * 6 + [0.03] * 4 + [0.055] + [0.03] * 4 + [0.055] * 3 + [0.03] * 6 +
    [0.055] * 2 + [0.03] * 4 + [0.055] * 2 + [0.05] * 4 + [0.012] * 12 + [0.12] * 6, np.float32)
assert _FETCH_RADII.shape == (111,)


# robots/ur5/fk.hh and robots/baxter/fk.hh sphere radii (reference order)
_UR5_RADII = np.array([0.08, 0.08, 0.08, 0.08, 0.08, 0.08, 0.08, 0.08, 0.06, 0.06, 0.06, 0.06, 0.04, 0.04, 0.04, 0.04, 0.04, 0.04, 0.04, 0.04, 0.04, 0.04, 0.02, 0.015, 0.015, 0.015, 0.02, 0.02, 0.02, 0.02, 0.02, 0.02, 0.02, 0.015, 0.015, 0.015], np.float32)
_BAXTER_RADII = np.array([0.25, 0.25, 0.23, 0.2, 0.1, 0.1, 0.1, 0.08, 0.08, 0.08, 0.1, 0.08, 0.08, 0.08, 0.07, 0.07, 0.07, 0.08, 0.05, 0.1, 0.1, 0.1, 0.08, 0.08, 0.08, 0.1, 0.08, 0.08, 0.08, 0.07, 0.07, 0.07, 0.08, 0.05, 0.5, 0.04, 0.04, 0.015, 0.015, 0.012, 0.012, 0.012, 0.014, 0.014, 0.014, 0.014, 0.015, 0.015, 0.012, 0.012, 0.012, 0.014, 0.014, 0.014, 0.014, 0.04, 0.04, 0.015, 0.015, 0.012, 0.012, 0.012, 0.014, 0.014, 0.014, 0.014, 0.015, 0.015, 0.012, 0.012, 0.012, 0.014, 0.014, 0.014, 0.014], np.float32)


def PandaBase(base_x100: int, base_y100: int, base_z100: int, name: Optional[str] = None) -> Robot:
    """vamp::robots::PandaBase<X100, Y100, Z100> (robots/panda_base.hh:15)."""
    return Robot(name or f"panda_{base_x100}_{base_y100}_{base_z100}", base_x100, base_y100, base_z100)


# robots/panda_grid.hh:10-41 -- including this fork's default Panda at base (2, 2, 0)
panda = PandaBase(200, 200, 0, "panda")
for _i in range(3):
    for _j in range(3):
        globals()[f"panda_{_i}_{_j}"] = PandaBase(100 * _i, 100 * _j, 0, f"panda_{_i}_{_j}")
        __all__.append(f"panda_{_i}_{_j}")


# robots/fetch.hh: vamp::robots::Fetch (8 dof, no base offset)
fetch = Robot("fetch", 0, 0, 0, kind=_lib.VGPU_ROBOT_FETCH)
__all__.append("fetch")


def PandaPair(a100=(0, 0, 0), b100=(100, 0, 0), name: Optional[str] = None) -> Robot:
    """The two-Panda composite of BASELINE configs[4] (14 dof: arm A = PandaBase<a100> on joints
    0..6, arm B = PandaBase<b100> on joints 7..13).  No reference counterpart: validity is
    fkcc_A && fkcc_B && no A-B sphere overlap (oracle/vamp_oracle.c vo_pair_*)."""
    return Robot(name or f"panda_pair_{a100}_{b100}", *a100, kind=_lib.VGPU_ROBOT_PANDA_PAIR, base2=tuple(b100))


panda_pair = PandaPair((0, 0, 0), (100, 0, 0), "panda_pair")
__all__ += ["PandaPair", "panda_pair"]

# robots/ur5.hh (6 dof) and robots/baxter.hh (14-dof dual arm): no base offset
ur5 = Robot("ur5", 0, 0, 0, kind=_lib.VGPU_ROBOT_UR5)
baxter = Robot("baxter", 0, 0, 0, kind=_lib.VGPU_ROBOT_BAXTER)
__all__ += ["ur5", "baxter", "RRTCSettings", "Halton", "PlanningResult", "PRMNeighborParams", "PRMSettings"]
