"""Timing of the GPU point-cloud filter (vgpu_filter.hip, reference collision/filter.hh:175-268).

Input resident in HBM (torch allocation), vgpu_filter_pointcloud on the device pointers; the
call is synchronous, so wall time per call is the whole filter (6 passes: keys, radix sort,
next-farther scan, pointer doubling, compaction, plus one count read-back per pass).  The
oracle restatement (tests/oracle_py.py, one core) is timed on the same cloud for reference.
Cloud: points on the 14 cage spheres (SURVEY §8d config 3 style) plus uniform clutter.
Usage: python tools/bench_filter.py [n_points] [reps]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import vamp_amd  # noqa: E402
from vamp_amd import _lib  # noqa: E402

CAGE = np.array([[0.55, 0, 0.25], [0.35, 0.35, 0.25], [0, 0.55, 0.25], [-0.55, 0, 0.25], [-0.35, -0.35, 0.25],
                 [0, -0.55, 0.25], [0.35, -0.35, 0.25], [0.35, 0.35, 0.8], [0, 0.55, 0.8], [-0.35, 0.35, 0.8],
                 [-0.55, 0, 0.8], [-0.35, -0.35, 0.8], [0, -0.55, 0.8], [0.35, -0.35, 0.8]], np.float32)


def cloud(n, seed=1):
    rng = np.random.default_rng(seed)
    m = n * 7 // 8
    d = rng.normal(size=(m, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pts = CAGE[rng.integers(0, len(CAGE), m)] + 0.2 * d
    clutter = rng.uniform([-1, -1, 0], [1, 1, 1.2], size=(n - m, 3))
    return np.concatenate([pts, clutter]).astype(np.float32)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    args = (0.005, 1.5, [0.0, 0.0, 0.5], [-1.2, -1.2, -0.1], [1.2, 1.2, 1.4], 1)
    pc = cloud(n)
    ctx = vamp_amd.context(0)
    d_pc = torch.from_numpy(pc).cuda()
    d_out = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    o, lo, up = (np.ascontiguousarray(v, np.float32) for v in args[2:5])
    cnt = C.c_size_t(0)
    lib = _lib.load()

    def run():
        _lib.check(lib.vgpu_filter_pointcloud(ctx.h, d_pc.data_ptr(), n, args[0], args[1],
                                              o.ctypes.data_as(_lib.F32P), lo.ctypes.data_as(_lib.F32P),
                                              up.ctypes.data_as(_lib.F32P), args[5], d_out.data_ptr(),
                                              C.byref(cnt)), ctx.h)

    run()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        times.append(time.perf_counter() - t0)
    gpu_ms = 1e3 * float(np.median(times))
    got = d_out[:cnt.value].cpu().numpy().view(np.uint32)

    import oracle_py as O  # the checker and the CPU leg only
    t0 = time.perf_counter()
    want = O.filter_pointcloud(pc, *args[:5], cull=bool(args[5]))
    cpu_ms = 1e3 * (time.perf_counter() - t0)
    line = {"workload": "filter_pointcloud", "points": n, "kept": int(cnt.value),
            "parity": bool(np.array_equal(got, want)), "gpu_ms": gpu_ms, "gpu_points_per_s": n / gpu_ms * 1e3,
            "cpu_oracle_ms": cpu_ms, "cpu_cores": 1, "min_dist": args[0], "reps": reps}
    print(json.dumps(line))
    return 0 if line["parity"] else 1


if __name__ == "__main__":
    sys.exit(main())
