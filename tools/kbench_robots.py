#!/usr/bin/env python3
"""Kernel A/B timing for the Fetch and two-Panda kernels (development tool, not the contract bench).

    VAMP_AMD_LIB=mr-vamp_amd/vamp_amd/libvampgpu_<v>.so python tools/kbench_robots.py [--n N]

Times, with HIP events on the launch stream: Fetch sample_fkcc over draws 1..4M on the MBM
table scene, Fetch validate_motions over valid-endpoint edges capped at 1.0, and the two-Panda
composite validate_motions (bench.py --workload pair edges).  One JSON line per kernel.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mr-vamp_amd"), os.path.join(ROOT, "tests")]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("VAMP_AMD_LIB", "default")))
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import torch

    import vamp_amd as vamp

    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)

    def timeit(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / a.reps

    env, _ = bench.fetch_scene(vamp)
    if a.only in ("", "fetch"):
        D = 4_000_000
        q = torch.empty((D, 8), device=dev)
        v = torch.empty(D, dtype=torch.uint8, device=dev)
        ms = timeit(lambda: vamp.fetch.sample_fkcc_device(1, D, env, q.data_ptr(), v.data_ptr(), ctx))
        print(json.dumps({"tag": a.tag, "kernel": "fetch_sample_fkcc", "ms": ms, "samples_per_s": D / ms * 1e3,
                          "valid": v.float().mean().item()}), flush=True)
        vq = q[v.bool()][: 2 * a.n]
        s, g = vq[0::2].contiguous(), vq[1::2].clone()
        d = torch.linalg.vector_norm((g - s).double(), dim=1)
        g = (s + (g - s) * torch.clamp(1.0 / torch.clamp(d, min=1e-9), max=1.0).float()[:, None]).contiguous()
        E = s.shape[0]
        ok = torch.empty(E, dtype=torch.uint8, device=dev)
        nb = torch.empty(E, dtype=torch.int32, device=dev)
        ms = timeit(lambda: vamp.fetch.validate_device(s.data_ptr(), g.data_ptr(), E, env, ok.data_ptr(), nb.data_ptr(),
                                                       ctx))
        print(json.dumps({"tag": a.tag, "kernel": "fetch_validate", "ms": ms,
                          "interp_per_s": 8 * nb.long().sum().item() / ms * 1e3, "ok": ok.float().mean().item()}),
              flush=True)
    if a.only in ("", "pair"):
        import oracle_py as op
        oenv = op.pair_scene()
        penv = vamp.Environment()
        for x, y, z, r, _ in oenv.spheres:
            penv.add_sphere(vamp.Sphere([x, y, z], r))
        for row in oenv.zcuboids:
            penv.add_cuboid(vamp.Cuboid.from_axes(row[0:3], row[3:6], row[6:9], row[9:12], row[12:15]))
        gen = torch.Generator(device=dev)
        gen.manual_seed(3)
        sm = torch.tensor(bench.S_M * 2, device=dev)
        sa = torch.tensor(bench.S_A * 2, device=dev)
        m = 4 * a.n
        q = torch.addcmul(sa, torch.rand((m, 14), generator=gen, device=dev), sm).contiguous()
        v = torch.empty(m, dtype=torch.uint8, device=dev)
        ms = timeit(lambda: vamp.panda_pair.fkcc_device(q.data_ptr(), m, penv, v.data_ptr(), ctx))
        print(json.dumps({"tag": a.tag, "kernel": "pair_fkcc", "ms": ms, "configs_per_s": m / ms * 1e3}), flush=True)
        vq = q[v.bool()][: 2 * a.n]
        s, g = vq[0::2].contiguous(), vq[1::2].clone()
        for sl in (slice(0, 7), slice(7, 14)):
            d = torch.linalg.vector_norm((g[:, sl] - s[:, sl]).double(), dim=1)
            g[:, sl] = s[:, sl] + (g[:, sl] - s[:, sl]) * torch.clamp(1.0 / torch.clamp(d, min=1e-9), max=1.0).float()[:, None]
        g = g.contiguous()
        E = s.shape[0]
        ok = torch.empty(E, dtype=torch.uint8, device=dev)
        nb = torch.empty(E, dtype=torch.int32, device=dev)
        ms = timeit(lambda: vamp.panda_pair.validate_device(s.data_ptr(), g.data_ptr(), E, penv, ok.data_ptr(),
                                                            nb.data_ptr(), ctx))
        print(json.dumps({"tag": a.tag, "kernel": "pair_validate", "ms": ms,
                          "interp_per_s": 8 * nb.long().sum().item() / ms * 1e3, "ok": ok.float().mean().item()}),
              flush=True)


if __name__ == "__main__":
    main()
