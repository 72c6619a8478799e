#!/usr/bin/env python3
"""CAPT A/B timing on one GPU (development tool): BASELINE configs[2]'s per-configuration fkcc of
2^20 Panda configurations against the 10k-point cloud, and 2^20 raw collides_simd queries.

    VAMP_AMD_LIB=mr-vamp_amd/vamp_amd/libvampgpu_<v>.so python tools/kbench_capt.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
import scenes  # noqa: E402


def main():
    import torch

    import vamp_amd as vamp
    tag = os.path.basename(os.environ.get("VAMP_AMD_LIB", "default"))
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.Stream(dev)
    ctx.set_stream(st.cuda_stream)
    env = vamp.Environment()
    env.add_pointcloud(scenes.cage_points(10000, seed=1), scenes.R_MIN, scenes.R_MAX, scenes.R_POINT)
    n = 1 << 20
    with torch.cuda.stream(st):
        g = torch.Generator(device=dev)
        g.manual_seed(2)
        q = torch.addcmul(torch.tensor(bench.S_A, device=dev), torch.rand((n, 7), generator=g, device=dev),
                          torch.tensor(bench.S_M, device=dev)).contiguous()
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        c, r = scenes.raw_queries(n)
        cd, rd = torch.from_numpy(c).to(dev), torch.from_numpy(r).to(dev)
        out = torch.empty(n, dtype=torch.uint8, device=dev)

        def timeit(fn, reps=10):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                fn()
            e1.record(st)
            torch.cuda.synchronize(dev)
            return e0.elapsed_time(e1) / reps

        ms = timeit(lambda: vamp.panda_0_0.fkcc_device(q.data_ptr(), n, env, ok.data_ptr(), ctx))
        print(json.dumps({"tag": tag, "kernel": "capt_fkcc", "ms": ms, "configs_per_s": n / ms * 1e3,
                          "valid": ok.float().mean().item()}))
        ms = timeit(lambda: env.pointcloud_collides_device(cd.data_ptr(), rd.data_ptr(), n, out.data_ptr(), simd=True,
                                                           ctx=ctx))
        print(json.dumps({"tag": tag, "kernel": "capt_raw_simd", "ms": ms, "queries_per_s": n / ms * 1e3,
                          "hit": out.float().mean().item()}))


if __name__ == "__main__":
    main()
