#!/usr/bin/env python3
"""Kernel A/B timing on one GPU (development tool, not the contract bench).

    VAMP_AMD_LIB=mr-vamp_amd/vamp_amd/libvampgpu_<v>.so python tools/kbench.py [--edges N] [--reps R]

Builds the bench.py workload (valid-endpoint cage edges capped at 1.0, plus raw pairs),
times validate_motions / fkcc / sphere_fk with HIP events on the launch stream and
prints one JSON line per kernel.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--edges", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("VAMP_AMD_LIB", "default")))
    ap.add_argument("--only-setb", action="store_true", help="validate set B only (PMC passes)")
    a = ap.parse_args()
    import torch

    import vamp_amd as vamp

    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.Stream(dev)
    ctx.set_stream(st.cuda_stream)
    env = vamp.Environment()
    for c in bench.CAGE:
        env.add_sphere(vamp.Sphere(c, 0.2))
    robot = vamp.panda_0_0
    with torch.cuda.stream(st):
        s, g = bench.make_edges(torch, vamp, env, robot, a.edges, 99, dev)
        ok = torch.empty(a.edges, dtype=torch.uint8, device=dev)
        nb = torch.empty(a.edges, dtype=torch.int32, device=dev)

        def timeit(fn):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                fn()
            e1.record(st)
            torch.cuda.synchronize(dev)
            return e0.elapsed_time(e1) / a.reps

        ms = timeit(lambda: robot.validate_device(s.data_ptr(), g.data_ptr(), a.edges, env, ok.data_ptr(),
                                                  nb.data_ptr(), ctx))
        units = 8 * nb.long().sum().item()
        print(json.dumps({"tag": a.tag, "kernel": "validate_setB", "ms": ms, "interp_per_s": units / ms * 1e3,
                          "ok": ok.float().mean().item()}))
        if a.only_setb:
            return
        # raw pairs (set A): mostly invalid, long edges
        gen = torch.Generator(device=dev)
        gen.manual_seed(5)
        sm = torch.tensor(bench.S_M, device=dev)
        sa = torch.tensor(bench.S_A, device=dev)
        ra = torch.addcmul(sa, torch.rand((a.edges, 7), generator=gen, device=dev), sm).contiguous()
        rb = torch.addcmul(sa, torch.rand((a.edges, 7), generator=gen, device=dev), sm).contiguous()
        ms = timeit(lambda: robot.validate_device(ra.data_ptr(), rb.data_ptr(), a.edges, env, ok.data_ptr(),
                                                  nb.data_ptr(), ctx))
        units = 8 * nb.long().sum().item()
        print(json.dumps({"tag": a.tag, "kernel": "validate_setA", "ms": ms, "interp_per_s": units / ms * 1e3,
                          "ok": ok.float().mean().item()}))
        nq = 1 << 22
        q = torch.addcmul(sa, torch.rand((nq, 7), generator=gen, device=dev), sm).contiguous()
        v = torch.empty(nq, dtype=torch.uint8, device=dev)
        ms = timeit(lambda: robot.fkcc_device(q.data_ptr(), nq, env, v.data_ptr(), ctx))
        print(json.dumps({"tag": a.tag, "kernel": "fkcc", "ms": ms, "configs_per_s": nq / ms * 1e3,
                          "valid": v.float().mean().item()}))
        out = torch.empty((3, 59, nq), device=dev)
        ms = timeit(lambda: robot.sphere_fk_device(q.data_ptr(), nq, out.data_ptr(), nq, ctx))
        print(json.dumps({"tag": a.tag, "kernel": "sphere_fk", "ms": ms, "GBps": 736 * nq / ms / 1e6}))


if __name__ == "__main__":
    main()
