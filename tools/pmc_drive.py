#!/usr/bin/env python3
"""Profiling driver: exactly the timed step of one bench.py workload, nothing else, so a rocprofv3
kernel trace or PMC pass over this process holds only that step's dispatches (development tool,
not the contract bench).

    python tools/pmc_drive.py prep --workload W          # inputs -> $TMPDIR/vamp_pmc_inputs/W.npz (unprofiled)
    rocprofv3 --pmc ... -- python3 tools/pmc_drive.py run --workload W [--calls C]

`run` loads the inputs, builds the environment (its upload kernels -- the CAPT cell grid -- are
excluded from the summaries by kernel name), runs one warm-up call and C measured calls of the
workload's step, and writes $TMPDIR/vamp_pmc_inputs/W.meta.json (units per call, calls) for
tools/pmc_report.py.  Workloads: validate (configs[1] set B, 2^20 edges), validate_setA, validate_table_pick (set B edges on the MBM
table_pick scene), rrtc / rrtc_pair (configs[0] / configs[4]'s planner: the solved paths' segments as one batch), capt
(configs[2], 2^20 configurations), fetch_prm (configs[3] vertex stage, 4M draws: the fused
sample+fkcc and the compaction), prm_edges (configs[3] edge stage: kNN + gather + validation +
pair selection + device assembly through vgpu_prm_edges_allgather at world size 1; prm_edges_full: at
the 2,681,709 valid vertices of 4M draws), pair
(configs[4], 2^20 composite edges).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402

OUT = os.path.join(os.environ.get("TMPDIR", "/tmp"), "vamp_pmc_inputs")  # large inputs: outside gpurun_out
WORKLOADS = ("validate", "validate_setA", "validate_table_pick", "capt", "fetch_prm", "prm_edges", "prm_edges_full",
             "pair", "rrtc", "rrtc_pair")


def setup(torch, vamp, w, dev, ctx, prep, inp, a):
    """(step(), units per call, unit name, extra meta) of workload w; prep=True builds and saves inputs"""
    path = os.path.join(OUT, f"{w}.npz")
    if w in ("rrtc", "rrtc_pair"):  # the bench line's GPU leg: every solved path's segments, one validate batch
        if prep:
            return None
        envs, S, G, robot, _ = bench.rrtc_problems(vamp, "panda_pair" if w == "rrtc_pair" else "panda")
        res = [robot.rrtc(S[k], G[k], envs[k], bench.RRTC_SETTINGS(vamp), robot.halton()) for k in range(len(S))]
        if w == "rrtc":  # one scene per problem: the problem with the most segments (the bench line's batch)
            k = int(np.argmax([len(r.path) for r in res]))
            envs, res = envs[k:k + 1], res[k:k + 1]
        a_ = torch.from_numpy(np.concatenate([r.path[:-1] for r in res])).to(dev)
        b_ = torch.from_numpy(np.concatenate([r.path[1:] for r in res])).to(dev)
        E = a_.shape[0]
        ok = torch.empty(E, dtype=torch.uint8, device=dev)
        nb = torch.empty(E, dtype=torch.int32, device=dev)
        env = envs[0]
        env.handle(ctx)
        return (lambda: robot.validate_device(a_.data_ptr(), b_.data_ptr(), E, env, ok.data_ptr(), nb.data_ptr(), ctx),
                E, "path segments", {})
    if w in ("validate", "validate_setA", "validate_table_pick"):
        if w == "validate_table_pick":
            env, _, _ = bench.scene_envs(vamp, "table_pick")
        else:
            env = vamp.Environment()
            for c in bench.CAGE:
                env.add_sphere(vamp.Sphere(c, 0.2))
        robot = vamp.panda_0_0
        E = a.edges
        if prep:
            s, g = bench.make_edges(torch, vamp, env, robot, E, bench.shard_seed(0), dev,
                                    edge_set="A" if w == "validate_setA" else "B")
            np.savez(path, starts=s.cpu().numpy(), goals=g.cpu().numpy())
            return None
        s, g = torch.from_numpy(inp["starts"]).to(dev), torch.from_numpy(inp["goals"]).to(dev)
        ok = torch.empty(E, dtype=torch.uint8, device=dev)
        nb = torch.empty(E, dtype=torch.int32, device=dev)
        return (lambda: robot.validate_device(s.data_ptr(), g.data_ptr(), E, env, ok.data_ptr(), nb.data_ptr(), ctx),
                E, "edges", {})
    if w == "pair":
        env, _ = bench.pair_scene_env(vamp)
        robot = vamp.panda_pair
        E = a.edges
        if prep:
            s, g = bench.make_pair_edges(torch, robot, env, E, bench.shard_seed(0), dev, ctx)
            np.savez(path, starts=s.cpu().numpy(), goals=g.cpu().numpy())
            return None
        s, g = torch.from_numpy(inp["starts"]).to(dev), torch.from_numpy(inp["goals"]).to(dev)
        ok = torch.empty(E, dtype=torch.uint8, device=dev)
        nb = torch.empty(E, dtype=torch.int32, device=dev)
        return (lambda: robot.validate_device(s.data_ptr(), g.data_ptr(), E, env, ok.data_ptr(), nb.data_ptr(), ctx),
                E, "edges", {})
    if w == "capt":
        import scenes
        if prep:
            return None
        env = vamp.Environment()
        env.add_pointcloud(scenes.cage_points(10000, seed=1), scenes.R_MIN, scenes.R_MAX, scenes.R_POINT)
        N = a.edges
        gen = torch.Generator(device=dev)
        gen.manual_seed(2)
        q = torch.addcmul(torch.tensor(bench.S_A, device=dev), torch.rand((N, 7), generator=gen, device=dev),
                          torch.tensor(bench.S_M, device=dev)).contiguous()
        ok = torch.empty(N, dtype=torch.uint8, device=dev)
        env.handle(ctx)
        return lambda: vamp.panda_0_0.fkcc_device(q.data_ptr(), N, env, ok.data_ptr(), ctx), N, "configurations", {}
    if w == "fetch_prm":
        from vamp_amd import roadmap
        if prep:
            return None
        env, _ = bench.fetch_scene(vamp)
        env.handle(ctx)
        D = a.draws
        return (lambda: roadmap.sample_valid_shard(torch, vamp.fetch, env, 1, D, ctx, dev), D, "draws", {})
    if w in ("prm_edges", "prm_edges_full"):
        from vamp_amd import roadmap
        if w == "prm_edges_full":
            a.vertices = 2681709  # the valid vertices of configs[3]'s 4M draws
        env, _ = bench.fetch_scene(vamp)
        if prep:
            draws = int(a.vertices / 0.6) + 4096
            rows, _, cnt = roadmap.sample_valid_shard(torch, vamp.fetch, env, 1, draws, ctx, dev)
            np.savez(path, V=rows[:min(a.vertices, cnt)].cpu().numpy())
            return None
        V = torch.from_numpy(inp["V"]).to(dev)
        comm = roadmap.Comm(ctx, 0, 1, roadmap.Comm.unique_id())
        n = V.shape[0]
        k, _ = roadmap.prm_neighbor_params(8, vamp.fetch.space_measure(), n)
        bound = int(np.minimum(k.astype(np.int64), np.arange(n, dtype=np.int64)).sum())
        bufs = roadmap.EdgeStageBuffers(torch, n, dev, 2 * bound)
        env.handle(ctx)
        return (lambda: roadmap.build_roadmap_edges_comm(torch, vamp.fetch, env, V, comm, bufs=bufs), n, "vertices",
                {"comm": comm})
    raise SystemExit(f"unknown workload {w}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("prep", "run"))
    ap.add_argument("--workload", choices=WORKLOADS, required=True)
    ap.add_argument("--calls", type=int, default=2)
    ap.add_argument("--edges", type=int, default=1 << 20)
    ap.add_argument("--draws", type=int, default=4_000_000)
    ap.add_argument("--vertices", type=int, default=100_000)
    a = ap.parse_args()
    import torch

    import vamp_amd as vamp
    os.makedirs(OUT, exist_ok=True)
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    w = a.workload
    if a.mode == "prep":
        setup(torch, vamp, w, dev, ctx, True, None, a)
        torch.cuda.synchronize(dev)
        print(f"prep {w} ok", flush=True)
        return
    p = os.path.join(OUT, f"{w}.npz")
    inp = np.load(p, allow_pickle=False) if os.path.exists(p) else None
    step, units, unit, keep = setup(torch, vamp, w, dev, ctx, False, inp, a)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # markers: torch.cuda._sleep dispatches a kernel named spin_kernel; tools/pmc_report.py keeps only the
    # dispatches between the first and the last one
    torch.cuda._sleep(1000)
    step()  # warm-up (counted by the profiler too: the report divides by calls + 1)
    e0.record(st)
    for _ in range(a.calls):
        step()
    e1.record(st)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / a.calls
    meta = {"workload": w, "units_per_call": units, "unit": unit, "calls_profiled": a.calls + 1, "ms_per_call": ms}
    with open(os.path.join(OUT, f"{w}.meta.json"), "w") as f:
        json.dump(meta, f)
    print(json.dumps(meta), flush=True)
    del keep


if __name__ == "__main__":
    main()
