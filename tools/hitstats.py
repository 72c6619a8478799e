#!/usr/bin/env python3
"""Children hit statistics of the Panda staged pass (development tool; needs the VGPU_HITSTATS variant:
make -C mr-vamp_amd VARIANT=hs DEFS=-DVGPU_HITSTATS).  For one validate call on set B, one on set A and
one CAPT fkcc call: per (source kind, check) the children items run and how many of them hit -- the share of
children work that only confirms a bounding hit that is no collision.

    VAMP_AMD_LIB=mr-vamp_amd/vamp_amd/libvampgpu_hs.so python tools/hitstats.py > gpurun_out/hitstats.json
    VAMP_AMD_LIB=... python tools/hitstats.py --fetch   # the Fetch: configs[3]'s sampler (4M draws) and the
                                                        # edge stage at 100k vertices
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402


def fetch_main():
    import torch

    import vamp_amd as vamp
    from vamp_amd import roadmap
    from vamp_amd._lib import load
    lib = load()
    fn = lib.vgpu_fetch_hitstats
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_uint32), C.c_int]
    buf = (C.c_uint32 * (5 * 64 * 2))()
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    env, _ = bench.fetch_scene(vamp)
    env.handle(ctx)
    out = {}

    def grab(tag):
        torch.cuda.synchronize(dev)
        assert fn(buf, 1) == 0
        a = np.frombuffer(buf, np.uint32).reshape(5, 64, 2).copy()
        out[tag] = {f"kind{k}_check{c}": {"items": int(a[k, c, 0]), "hits": int(a[k, c, 1]),
                                          "hit_rate": int(a[k, c, 1]) / int(a[k, c, 0])}
                    for k in range(5) for c in range(64) if a[k, c, 0]}

    fn(buf, 1)
    rows, _, cnt = roadmap.sample_valid_shard(torch, vamp.fetch, env, 1, 4_000_000, ctx, dev)
    grab("fetch_sampler_4M")
    V = rows[:min(100_000, cnt)].contiguous()
    comm = roadmap.Comm(ctx, 0, 1, roadmap.Comm.unique_id())
    fn(buf, 1)
    roadmap.build_roadmap_edges_comm(torch, vamp.fetch, env, V, comm)
    grab("fetch_edges_100k")
    print(json.dumps(out))


def main():
    if "--fetch" in sys.argv:
        return fetch_main()
    import torch

    import vamp_amd as vamp
    from vamp_amd._lib import load
    lib = load()
    fn = lib.vgpu_panda_hitstats
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_uint32), C.c_int]
    buf = (C.c_uint32 * (5 * 64 * 2))()
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    env = vamp.Environment()
    for c in bench.CAGE:
        env.add_sphere(vamp.Sphere(c, 0.2))
    robot = vamp.panda_0_0
    E = 1 << 20
    out = {}

    def grab(tag):
        torch.cuda.synchronize(dev)
        assert fn(buf, 1) == 0
        a = np.frombuffer(buf, np.uint32).reshape(5, 64, 2).copy()
        rec = {}
        for kind in range(5):
            for c in range(64):
                items, hits = int(a[kind, c, 0]), int(a[kind, c, 1])
                if items:
                    rec[f"kind{kind}_check{c}"] = {"items": items, "hits": hits, "hit_rate": hits / items}
        out[tag] = rec

    fn(buf, 1)
    for edge_set in ("B", "A"):
        s, g = bench.make_edges(torch, vamp, env, robot, E, bench.shard_seed(0), dev, edge_set=edge_set)
        ok = torch.empty(E, dtype=torch.uint8, device=dev)
        nb = torch.empty(E, dtype=torch.int32, device=dev)
        fn(buf, 1)  # the edge generation's fkcc passes are not counted
        robot.validate_device(s.data_ptr(), g.data_ptr(), E, env, ok.data_ptr(), nb.data_ptr(), ctx)
        grab(f"validate_set{edge_set}")
    import scenes
    cenv = vamp.Environment()
    cenv.add_pointcloud(scenes.cage_points(10000, seed=1), scenes.R_MIN, scenes.R_MAX, scenes.R_POINT)
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    q = torch.addcmul(torch.tensor(bench.S_A, device=dev), torch.rand((E, 7), generator=gen, device=dev),
                      torch.tensor(bench.S_M, device=dev)).contiguous()
    v = torch.empty(E, dtype=torch.uint8, device=dev)
    cenv.handle(ctx)
    fn(buf, 1)
    robot.fkcc_device(q.data_ptr(), E, cenv, v.data_ptr(), ctx)
    grab("capt_fkcc")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
