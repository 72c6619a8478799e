#!/usr/bin/env python3
"""CAPT build timing on one GPU (development tool): host build (vgpu_capt.cpp) vs the device build
(vgpu_capt_build.hip) of the same cloud, points on the cage spheres (tests/scenes.py), arrays
compared bit for bit.  Wall clock around each call (both are synchronous), best of 3.

    python tools/bench_capt_build.py [n ...]      (default 10000 100000 1000000)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import vamp_amd as vamp
    from scenes import R_MAX, R_MIN, R_POINT, cage_points

    ctx = vamp.context(0)
    for n in [int(x) for x in sys.argv[1:]] or [10000, 100000, 1000000]:
        pts = cage_points(n, 1)
        d = torch.from_numpy(pts).to("cuda:0")
        torch.cuda.synchronize()
        th, td = [], []
        for _ in range(3):
            eh, ed = vamp.Environment(), vamp.Environment()
            t0 = time.perf_counter()
            eh.add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
            t1 = time.perf_counter()
            ed.add_pointcloud_device(d.data_ptr(), n, R_MIN, R_MAX, R_POINT, ctx)
            t2 = time.perf_counter()
            th.append(t1 - t0)
            td.append(t2 - t1)
        a, b = eh.pointcloud_arrays(), ed.pointcloud_arrays()
        same = all(np.array_equal(np.atleast_1d(a[k]).view(np.uint8), np.atleast_1d(b[k]).view(np.uint8))
                   for k in ("tests", "aabbs", "aff_starts", "aff", "aabb_top"))
        print(json.dumps({"n": n, "host_ms": min(th) * 1e3, "device_ms": min(td) * 1e3,
                          "affordance_vectors": int(a["aff"].shape[0]), "identical": same}), flush=True)
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
