#!/usr/bin/env python3
"""Development probe (GPU box): does the ORDER of a configs[2] batch change the CAPT step's kernel time?

The point-cloud fkcc step (bench.py --workload capt: 2^20 uniform Panda configurations vs the 10k-point cage cloud)
is bound by the dependent cell-grid / tree gathers of each lane; in a random batch the 64 lanes of a wave read
unrelated cells.  This times vgpu_fkcc over the same configurations in several orders (HIP events, 20 calls each)
and checks the results are the same permutation of each other.  Orders: as drawn; sorted by a Morton key of
joints 0-3 (no FK); sorted by a Morton key of a world-frame sphere centre from sphere_fk (the forearm / the hand).
Prints one JSON line per order with the key + sort cost.  (torch only glues the probe; the kernels are the
library's.)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
import scenes  # noqa: E402
import vamp_amd as vamp  # noqa: E402


def spread(x, bits, dims):
    """bit i of x -> bit i * dims (int64 tensor)"""
    out = torch.zeros_like(x)
    for i in range(bits):
        out |= ((x >> i) & 1) << (i * dims)
    return out


def morton(cols, bits):
    key = torch.zeros(cols[0].shape[0], dtype=torch.int64, device=cols[0].device)
    for d, c in enumerate(cols):
        lo, hi = c.min(), c.max()
        u = ((c - lo) / (hi - lo + 1e-12) * ((1 << bits) - 1)).to(torch.int64)
        key |= spread(u, bits, len(cols)) << d
    return key


def main():
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    env = vamp.Environment()
    env.add_pointcloud(scenes.cage_points(10000, seed=1), scenes.R_MIN, scenes.R_MAX, scenes.R_POINT)
    robot = vamp.panda_0_0
    N = 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    q = torch.addcmul(torch.tensor(bench.S_A, device=dev), torch.rand((N, 7), generator=g, device=dev),
                      torch.tensor(bench.S_M, device=dev)).contiguous()
    env.handle(ctx)

    def time_fkcc(qq, reps=20):
        ok = torch.empty(N, dtype=torch.uint8, device=dev)
        for _ in range(3):
            robot.fkcc_device(qq.data_ptr(), N, env, ok.data_ptr(), ctx)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            robot.fkcc_device(qq.data_ptr(), N, env, ok.data_ptr(), ctx)
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / reps, ok.clone()

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            out = fn()
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / reps, out

    base_ms, base_ok = time_fkcc(q)
    print(json.dumps({"order": "as drawn", "fkcc_ms": base_ms}), flush=True)
    xyz = torch.empty((3, 59, N), dtype=torch.float32, device=dev)
    fk_ms, _ = timed(lambda: robot.sphere_fk_device(q.data_ptr(), N, xyz.data_ptr(), N, ctx))
    orders = {
        "morton q0-q3 (8 bits)": lambda: morton([q[:, j] for j in range(4)], 8),
        "morton q0-q2 (10 bits)": lambda: morton([q[:, j] for j in range(3)], 10),
        "morton sphere 30 xyz (10 bits)": lambda: morton([xyz[0, 30], xyz[1, 30], xyz[2, 30]], 10),
        "morton sphere 50 xyz (10 bits)": lambda: morton([xyz[0, 50], xyz[1, 50], xyz[2, 50]], 10),
        "morton sphere 20 xyz (10 bits)": lambda: morton([xyz[0, 20], xyz[1, 20], xyz[2, 20]], 10),
    }
    for name, keyf in orders.items():
        key_ms, key = timed(keyf)
        sort_ms, (_, perm) = timed(lambda: torch.sort(key))
        gather_ms, qs = timed(lambda: q[perm].contiguous())
        ms, ok = time_fkcc(qs)
        same = bool(torch.equal(ok, base_ok[perm]))
        print(json.dumps({"order": name, "fkcc_ms": ms, "key_ms": key_ms, "sort_ms": sort_ms, "gather_ms": gather_ms,
                          "sphere_fk_ms": fk_ms if "sphere" in name else 0.0, "results_equal": same}), flush=True)


if __name__ == "__main__":
    main()
