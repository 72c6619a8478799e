#!/usr/bin/env python3
"""Roadmap kNN timing on one GPU (development tool): the causal PRM* neighbour queries of the Fetch
Halton vertex sequence (BASELINE configs[3] sizes) through the brute-force scan and the spatial
index (vgpu_knn_index.hip), HIP events on the context stream; the two are compared where both run.

    python tools/knn_scale.py [n ...]     (default 100000 400000 2700000)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))


def main():
    import torch

    import vamp_amd as vamp
    from vamp_amd import roadmap
    from vamp_amd._lib import check, load

    sizes = [int(x) for x in sys.argv[1:]] or [100000, 400000, 2700000]
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.current_stream(dev)
    ctx.set_stream(st.cuda_stream)
    robot = vamp.fetch
    nmax = max(sizes)
    # the vertex sequence's geometry: scaled Halton<8> draws (validity does not matter to the kNN)
    q = torch.empty((nmax, 8), dtype=torch.float32, device=dev)
    ok = torch.empty(nmax, dtype=torch.uint8, device=dev)
    env = vamp.Environment()
    robot.sample_fkcc_device(1, nmax, env, q.data_ptr(), ok.data_ptr(), ctx)
    for n in sizes:
        V = q[:n].contiguous()
        k_np, r_np = roadmap.prm_neighbor_params(8, robot.space_measure(), n)
        kmax = int(max(1, k_np.max()))
        k = torch.from_numpy(k_np.view(np.int32)).to(dev)
        r = torch.from_numpy(r_np).to(dev)
        res = {}
        for mode in ([2, 1] if n <= int(os.environ.get("KNN_BRUTE_MAX", 400000)) else [2]):
            nbr = torch.zeros((n, kmax), dtype=torch.int32, device=dev)
            dd = torch.zeros((n, kmax), dtype=torch.float32, device=dev)
            cc = torch.zeros(n, dtype=torch.int32, device=dev)
            check(load().vgpu_set_knn_mode(ctx.h, mode), ctx.h)
            # wall clock around a synchronised call (the call may read sizes back mid-way, so
            # stream events alone can miss part of it); best of 3 after one warm-up call
            times = []
            for rep in range(4):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                check(load().vgpu_roadmap_knn(ctx.h, 8, V.data_ptr(), n, k.data_ptr(), r.data_ptr(), kmax,
                                              nbr.data_ptr(), dd.data_ptr(), cc.data_ptr()), ctx.h)
                check(load().vgpu_sync(ctx.h), ctx.h)
                torch.cuda.synchronize(dev)
                if rep:
                    times.append((time.perf_counter() - t0) * 1e3)
            res[mode] = (min(times), nbr, dd, cc)
            print(json.dumps({"n": n, "kmax": kmax, "mode": {1: "brute", 2: "index"}[mode],
                              "ms": res[mode][0], "candidates": int(cc.long().sum())}), flush=True)
        check(load().vgpu_set_knn_mode(ctx.h, 0), ctx.h)
        if 1 in res and 2 in res:
            (_, n1, d1, c1), (_, n2, d2, c2) = res[1], res[2]
            m = torch.arange(kmax, device=dev)[None, :] < c1[:, None]
            same = bool(torch.equal(c1, c2) and torch.equal(n1[m], n2[m]) and torch.equal(d1[m], d2[m]))
            print(json.dumps({"n": n, "index_equals_brute": same}), flush=True)
            if not same:
                sys.exit(1)


if __name__ == "__main__":
    main()
