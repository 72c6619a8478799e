#!/usr/bin/env python3
"""bench.py -- validated edge-interpolants/sec of the MI355X motion-validation rake.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--edges E] [--no-cpu]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1], SURVEY.md §8(d) config 2, set B): Panda 7-DOF
(PandaBase<0,0,0>), the 14-sphere cage of the reference's collision benchmark
(scripts/cpp/benchmark_collision_checks.cc:33-51), E = 2^20 edges per GPU between
collision-free endpoints with edge length capped at 1.0 rad (n_e = 4 -> 32 interpolants
per edge).  Endpoints are synthetic (seeded uniform draws, scaled by the Panda joint
limits), generated and filtered on the GPU before timing; inputs are resident in HBM.

One step = one vgpu_validate_motions launch over the rank's whole edge batch (reference
semantics: validate_motion per edge, 8-lane rake, early exit on the first colliding
block).  Units (rake/early-exit mode) = 8 x the rake blocks the reference
evaluates: every block of a valid edge, and an invalid edge's blocks through its first
invalid one (counted by the CPU rake on the same edges, whose results must equal the GPU's
edge for edge); the full count 8 * n_e of every edge is reported beside it.  Multi-GPU:
each rank owns an independent shard of edges (weak scaling, no collective on the data
path); the timed region is bracketed by barrier + synchronize and the max over ranks is
reported.  CPU baseline: the build's AVX2 rake (mr-vamp_amd/csrc/cpu) on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))

CAGE = [(0.55, 0, 0.25), (0.35, 0.35, 0.25), (0, 0.55, 0.25), (-0.55, 0, 0.25), (-0.35, -0.35, 0.25),
        (0, -0.55, 0.25), (0.35, -0.35, 0.25), (0.35, 0.35, 0.8), (0, 0.55, 0.8), (-0.35, 0.35, 0.8),
        (-0.55, 0, 0.8), (-0.35, -0.35, 0.8), (0, -0.55, 0.8), (0.35, -0.35, 0.8)]
S_M = [5.9342, 3.6652, 5.9342, 3.2289, 5.9342, 3.9095999999999997, 5.9342]
S_A = [-2.9671, -1.8326, -2.9671, -3.1416, -2.9671, -0.0873, -2.9671]
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 vector (= FP32 matrix) peak
EDGE_BYTES = 7 * 4 * 2 + 1 + 4  # start + goal in, ok + n_e out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--edges", type=int, default=1 << 20, help="edges per GPU")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample time")
    ap.add_argument("--oracle-edges", type=int, default=1 << 18,
                    help="edges checked against the scalar oracle (the CPU rake checks every edge)")
    ap.add_argument("--no-fk-leg", dest="fk_leg", action="store_false")
    ap.add_argument("--workload", default="validate",
                    choices=["validate", "capt", "fetch_prm", "prm_edges", "pair", "rrtc"],
                    help="validate: BASELINE configs[1] (the headline); capt: configs[2]; fetch_prm: configs[3] "
                         "vertex stage; prm_edges: configs[3] edge stage; pair: configs[4] two-Panda composite edges; "
                         "rrtc: configs[0] RRT-Connect on MBM table_pick (CPU rake)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="validate / pair: weak = --edges per GPU, each rank its own shard resident in HBM; strong = "
                         "one fixed batch of --edges split into contiguous ranges over the ranks, each step copying "
                         "its range in from pinned host memory and the results back (H2D + kernels + D2H timed)")
    ap.add_argument("--vertices", type=int, default=100_000,
                    help="prm_edges: roadmap vertices (RoadmapSettings::max_samples default, roadmap.hh:170)")
    ap.add_argument("--draws", type=int, default=4_000_000, help="fetch_prm: Halton draws per step (whole job)")
    ap.add_argument("--edge-set", default="B", choices=["A", "B"],
                    help="validate: SURVEY §8(d) config 2 set B (valid endpoints, length capped at 1.0: the headline) "
                         "or set A (raw uniform pairs, long edges, n_e ~ 20-40)")
    ap.add_argument("--base", default="000", choices=["000", "220"],
                    help="validate: PandaBase<0,0,0> (the headline) or the fork's default Panda (2,2,0) "
                         "(robots/panda_grid.hh:39)")
    ap.add_argument("--robot", default="panda", choices=["panda", "panda_pair"],
                    help="rrtc: the Panda on the MBM table_pick problems (configs[0]) or the two-Panda composite "
                         "(configs[4]'s planner half)")
    ap.add_argument("--scene", default="cage", choices=["cage", "table_pick"],
                    help="validate: the 14-sphere cage (the headline) or MotionBenchMaker table_pick_panda scene0001 "
                         "(tests/golden/panda_table_pick.npz)")
    return ap.parse_args()


def make_edges(torch, vamp, env, robot, n_edges, seed, dev, edge_set="B"):
    """set B = valid-endpoint edges, length capped at 1.0; set A = raw
    pairs of uniform configurations (no filter, no cap)."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    sm = torch.tensor(S_M, device=dev)
    sa = torch.tensor(S_A, device=dev)
    if edge_set == "A":
        u = torch.rand((2 * n_edges, 7), generator=g, device=dev, dtype=torch.float32)
        q = torch.addcmul(sa, u, sm)
        return q[0::2].contiguous(), q[1::2].contiguous()
    pool = []
    have = 0
    need = 2 * n_edges
    while have < need:
        m = max(1 << 20, int((need - have) / 0.17 * 1.1))
        u = torch.rand((m, 7), generator=g, device=dev, dtype=torch.float32)
        q = torch.addcmul(sa, u, sm).contiguous()
        ok = torch.empty(m, dtype=torch.uint8, device=dev)
        robot.fkcc_device(q.data_ptr(), m, env, ok.data_ptr())
        torch.cuda.synchronize(dev)
        v = q[ok.bool()]
        pool.append(v)
        have += v.shape[0]
    vq = torch.cat(pool)[:need]
    s = vq[0::2].contiguous()
    gl = vq[1::2].contiguous()
    d = torch.linalg.vector_norm((gl - s).double(), dim=1)
    scale = torch.clamp(1.0 / torch.clamp(d, min=1e-9), max=1.0).float()
    gl = (s + (gl - s) * scale[:, None]).contiguous()
    return s, gl


def host_threads():
    """CPU threads of the baseline legs: one per core of this rank's CPU share (16 on the GPU box,
    fewer when the affinity set is smaller)."""
    return max(1, min(16, len(os.sched_getaffinity(0))))


def cpu_rake_baseline(vamp, env, robot, starts, goals, seconds):
    """CPU reference timing: the build's own AVX2 rake (mr-vamp_amd/csrc/cpu/, one
    ConfigurationBlock<8> per register, bit-identical to the oracle and the GPU), one std::thread
    per core over static contiguous chunks, validate_motion with the reference's early exit.  The
    sample is the bench's whole edge batch, repeated until ~`seconds` of work.  Returns the line's
    cpu_baseline entry and the results of one pass (ok, n_e, blocks evaluated) for parity/units."""
    threads = host_threads()
    t = time.perf_counter()
    ok, nb, ne = robot.cpu_validate_batch(starts, goals, env, threads=threads)
    dt1 = max(time.perf_counter() - t, 1e-6)
    reps = max(1, int(seconds / dt1))
    t = time.perf_counter()
    for _ in range(reps):
        robot.cpu_validate_batch(starts, goals, env, threads=threads)
    dt = (time.perf_counter() - t) / reps
    ev = float(8 * ne.astype(np.int64).sum())
    full = float(8 * nb.astype(np.int64).sum())
    return {"value": ev / dt, "unit": "interpolants/s", "cores": threads, "kind": "port",
            "counting": "rake_early_exit (8 x rake blocks evaluated, the reference's early exit)",
            "value_full_mask_count": full / dt,
            "per_core": ev / dt / threads,
            "sample": f"the bench's {len(starts)} edges x {reps} passes ({dt:.3f} s per pass): mr-vamp_amd/csrc/cpu "
                      f"AVX2 rake (vgpu_cpu_validate_motions), {threads} threads, static contiguous chunks",
            "cpu_model": cpu_model(), "ok_fraction": float(ok.mean())}, ok, nb, ne


def scene_envs(vamp, scene):
    """(product Environment, oracle Env, description) of a validate scene: the 14-sphere cage, or
    MotionBenchMaker table_pick_panda scene0001 as resolved obstacle rows (tests/golden/panda_table_pick.npz)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as op

    op.build()
    env, oenv = vamp.Environment(), op.Env()
    if scene == "cage":
        for c in CAGE:
            env.add_sphere(vamp.Sphere(c, 0.2))
            oenv.add_sphere(c, np.float32(0.2))
        return env, oenv, "14-sphere cage"
    fx = np.load(os.path.join(ROOT, "tests", "golden", "panda_table_pick.npz"), allow_pickle=False)
    for k in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
        setattr(oenv, k, [list(r) for r in fx["env_" + k]])
    for row in fx["env_spheres"]:
        env.add_sphere(vamp.Sphere(row[0:3], float(row[3])))
    for row in np.concatenate([fx["env_cuboids"], fx["env_zcuboids"]]):
        env.add_cuboid(vamp.Cuboid.from_axes(row[0:3], row[3:6], row[6:9], row[9:12], row[12:15]))
    for row in np.concatenate([fx["env_capsules"], fx["env_zcapsules"]]):
        p1 = np.array(row[0:3], np.float32)
        env.add_capsule(vamp.Cylinder(p1, (p1 + np.array(row[3:6], np.float32)).astype(np.float32), float(row[6])))
    return env, oenv, "MBM table_pick_panda scene0001 (12 cuboids/capsules)"


def oracle_sample(oenv, starts, goals, n, base):
    """The independent checker (oracle/vamp_oracle.c, scalar restatement) on the first n edges."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as op

    return op.validate_motions(oenv, starts[:n], goals[:n], base, host_threads())


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parity_record(got_ok, got_n, ref_ok, ref_n, checker):
    """GPU results vs the checker on the same edges: bitwise on ok[] and n_e."""
    m = len(ref_ok)
    g_ok = np.asarray(got_ok[:m]).astype(bool)
    g_n = np.asarray(got_n[:m])
    return {"edges_compared": int(m), "mismatches": int((g_ok != np.asarray(ref_ok).astype(bool)).sum()),
            "n_mismatches": int((g_n != np.asarray(ref_n)).sum()), "checker": checker}


def algorithmic_flops(oenv, starts, goals, base, n=65536):
    """Executed float ops per edge under reference semantics (validate_motion with early
    exit), counted by the instrumented restatement (oracle/vamp_oracle.c vo_stats.flops) on the
    first n = 65536 of the bench's own edges; split into the first rake block (head kernel) and the
    back-steps (tail kernel).  Returns (head_per_edge, tail_per_edge, edges counted)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as op

    h, t = op.validate_flops(oenv, starts[:n], goals[:n], base, host_threads())
    return float(h.mean()), float(t.mean()), int(len(h))


def prof_record(workload):
    """The newest committed step profile of a workload (tools/prof_step.sh -> profiles/rNN_prof_<workload>.json,
    the highest round NN): kernel trace + PMC of exactly one timed step of this build's code.  (path, record) or
    (None, None)."""
    import glob
    import re
    best = None
    for path in glob.glob(os.path.join(ROOT, "profiles", f"r*_prof_{workload}.json")):
        m = re.match(r"r(\d+)_prof_", os.path.basename(path))
        if m and (best is None or int(m.group(1)) > best[0]):
            best = (int(m.group(1)), path)
    if best is None:
        return None, None
    with open(best[1]) as f:
        return os.path.relpath(best[1], ROOT), json.load(f)


def traffic_fields(workload, units):
    """`traffic` of a roofline from the workload's committed profile: its HBM bytes per call ((2 x FETCH_SIZE +
    WRITE_SIZE) x 1 KiB over the step's kernels, MI355X_MICROARCH.md's gfx950 correction) scaled to this run's
    units, plus the per-kernel L2 hit rates when the profile has them"""
    path, rec = prof_record(workload)
    if not rec or not rec.get("hbm_bytes_per_call"):
        return {"traffic": None, "traffic_source": None}
    out = {"traffic": rec["hbm_bytes_per_call"] * units / rec["units_per_call"],
           "traffic_source": f"{path}: PMC of one timed step of this workload (not measured in this run), "
                             f"{rec['hbm_bytes_per_call'] / rec['units_per_call']:.1f} B per {rec.get('unit', 'unit')}"}
    l2 = {k: v["L2_hit_rate"] for k, v in (rec.get("kernels") or {}).items()
          if v.get("L2_hit_rate") is not None and v.get("ms_per_call", 0) > 0.01}
    if l2:
        out["l2_hit_rate"] = l2
    return out


def c_ok_head_items(n_blocks, n_evaluated):
    """The largest back-step index the tail enumerates per edge: n_e - 1 for an edge that survives its
    first block (the CPU rake evaluated more than one block), 0 otherwise."""
    nb = np.asarray(n_blocks, np.int64)
    ne = np.asarray(n_evaluated, np.int64)
    return np.where(ne > 1, nb - 1, 0)


def strong_slice(n, rank, world):
    """contiguous range of a fixed batch of n units owned by `rank` (strong scaling)"""
    lo = n * rank // world
    return lo, n * (rank + 1) // world - lo


class PinnedShard:
    """Strong-scaling step of one rank: its edge range lives in pinned host memory; a step copies
    it to the device, validates it and copies the results back (the serving path)."""

    def __init__(self, torch, starts, goals, dev):
        self.h_s = starts.cpu().pin_memory()
        self.h_g = goals.cpu().pin_memory()
        self.d_s = torch.empty_like(starts)
        self.d_g = torch.empty_like(goals)
        self.h_ok = torch.empty(starts.shape[0], dtype=torch.uint8).pin_memory()

    def step(self, robot, env, ok, nb, ctx):
        self.d_s.copy_(self.h_s, non_blocking=True)
        self.d_g.copy_(self.h_g, non_blocking=True)
        robot.validate_device(self.d_s.data_ptr(), self.d_g.data_ptr(), self.d_s.shape[0], env, ok.data_ptr(),
                              nb.data_ptr(), ctx)
        self.h_ok.copy_(ok, non_blocking=True)


def shard_seed(rank):
    """Each rank draws its own independent edge shard (weak scaling: E edges per GPU)."""
    return 1234 + 7919 * rank


def reduce_over_ranks(dist, torch, wall, units, dev, world):
    """(max wall time over ranks, sum of units over ranks): the job finishes when the
    slowest rank does, and value = every rank's interpolants / that time.  The reduction
    tensor lives on `dev` (RCCL) or on the CPU (gloo)."""
    if world <= 1:
        return float(wall), float(units)
    on = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    mx = torch.tensor([wall], dtype=torch.float64, device=on)
    sm = torch.tensor([units], dtype=torch.float64, device=on)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx[0]), float(sm[0])


def fetch_scene(vamp):
    """MotionBenchMaker table_pick_fetch scene0001 as resolved obstacle rows (the committed
    fixture tests/golden/fetch_table_pick.npz; tests/oracle_py.py:mbm_env builds it)."""
    fx = np.load(os.path.join(ROOT, "tests", "golden", "fetch_table_pick.npz"), allow_pickle=False)
    env = vamp.Environment()
    for row in fx["env_spheres"]:
        env.add_sphere(vamp.Sphere(row[0:3], float(row[3])))
    for row in np.concatenate([fx["env_cuboids"], fx["env_zcuboids"]]):
        env.add_cuboid(vamp.Cuboid.from_axes(row[0:3], row[3:6], row[6:9], row[9:12], row[12:15]))
    for row in np.concatenate([fx["env_capsules"], fx["env_zcapsules"]]):
        p1 = np.array(row[0:3], np.float32)
        env.add_capsule(vamp.Cylinder(p1, (p1 + np.array(row[3:6], np.float32)).astype(np.float32), float(row[6])))
    return env, fx


def run_fetch_prm(a, torch, dist, rank, world, dev, stream, ctx, vamp):
    """BASELINE configs[3], vertex stage: draws 1..D of Halton<8> ->
    scale -> Fetch fkcc on the MBM table_pick scene, sharded by contiguous draw ranges over the
    ranks, valid vertices compacted on the device and all-gathered over RCCL.  Total draws fixed
    as N grows (strong scaling); one step = the whole stage including the exchange."""
    from vamp_amd import roadmap

    env, fx = fetch_scene(vamp)
    robot = vamp.fetch
    lo, n = roadmap.shard_range(a.draws, rank, world, 1)

    def step():
        rows, draws, cnt = roadmap.sample_valid_shard(torch, robot, env, lo, n, ctx, dev)
        if world > 1:
            rows, draws = roadmap.allgather_vertices(torch, dist, rows, draws, cnt)
            return rows.shape[0]
        return cnt

    for _ in range(a.warmup):
        n_vertices = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s0.record(stream)
    for _ in range(a.steps):
        n_vertices = step()
    s1.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    step_ev_ms = s0.elapsed_time(s1) / a.steps
    if world > 1:
        dist.barrier()
    wall_max, units_all = reduce_over_ranks(dist, torch, t1 - t0, float(n), dev, world)

    # the dominant kernel alone (fused sample + fkcc), HIP events on the launch stream
    q = torch.empty((max(n, 1), 8), dtype=torch.float32, device=dev)
    valid = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(a.steps):
        robot.sample_fkcc_device(lo, n, env, q.data_ptr(), valid.data_ptr(), ctx)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = e0.elapsed_time(e1) / a.steps
    if rank != 0:
        return
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as op
    from test_oracle_fetch import fetch_env

    oenv = fetch_env(op, fx)
    ks = np.arange(1, 1 + 4096) * max(1, a.draws // 4096)
    qs = op.robot_scale("fetch", op.halton(8, ks))
    _, _, _, fl = op.robot_fkcc("fetch", oenv, qs, stats=True)
    f_sample = float(fl.mean())
    cpu = None
    parity = None
    if not a.no_cpu and world == 1:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        m0 = 65536
        t = time.perf_counter()
        robot.cpu_fkcc_batch(op.robot_scale("fetch", op.halton(8, np.arange(1, m0 + 1))), env, threads=threads)
        dt0 = max(time.perf_counter() - t, 1e-3)
        m = int(min(n, m0 * a.cpu_seconds / dt0))
        qc = op.robot_scale("fetch", op.halton(8, np.arange(1, m + 1)))
        t = time.perf_counter()
        okc = robot.cpu_fkcc_batch(qc, env, threads=threads)
        dt = time.perf_counter() - t
        g_ok = valid[:m].cpu().numpy().astype(bool)
        g_q = q[:m].cpu().numpy()
        oo = op.robot_fkcc_threads("fetch", oenv, qc[:65536], threads=threads).astype(bool)
        parity = {"draws_compared": int(m), "mismatches": int((g_ok != okc).sum()),
                  "sample_mismatches": int((g_q.view(np.uint32) != qc.view(np.uint32)).any(1).sum()),
                  "checker": "mr-vamp_amd/csrc/cpu AVX2 rake Fetch fkcc on the oracle's Halton<8> + scale draws",
                  "oracle_mismatches": int((g_ok[:65536] != oo).sum()),
                  "oracle_checker": "oracle/vamp_oracle.c Fetch fkcc, first 65536 draws"}
        cpu = {"value": m / dt, "unit": "samples/s", "cores": threads, "kind": "port",
               "sample": f"draws 1..{m} of the same stage (Halton<8> scaling on the host untimed), "
                         f"mr-vamp_amd/csrc/cpu AVX2 rake Fetch fkcc, {threads} threads, {dt:.1f} s",
               "cpu_model": cpu_model()}
    line = {
        "metric": "PRM vertex-stage samples/sec (Fetch 8-DOF Halton<8> + FK+CC, RCCL all-gather of valid vertices)",
        "value": units_all * a.steps / wall_max,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall_max / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Halton<8> draws 1..D, the reference sampler; MBM table_pick_fetch scene0001)",
        "config": {"workload": f"BASELINE configs[3]: Fetch 8-DOF PRM vertex stage, {a.draws} draws sharded over "
                               f"{world} GPU(s), all-gather of valid vertices",
                   "robot": "Fetch", "draws_total": a.draws, "vertices": int(n_vertices),
                   "parallelism": f"dp{world} (contiguous draw ranges, one all-gather)"},
        "roofline": {"kernel": "vgpu_sample_fkcc: staged Halton + scale + fkcc (bound / queue / children kernels)",
                     "bound": "valu", "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     **utilisation("fetch_prm" if world == 1 else None, n, step_ev_ms, f_sample * n),
                     **traffic_fields("fetch_prm", n), "kernel_ms": step_ev_ms, "sample_fkcc_kernel_ms": kern_ms,
                     "algorithmic_flops_per_sample": f_sample,
                     "algorithmic_bytes_per_sample": 8 * 4 + 1, "step_ms_events": step_ev_ms,
                     "utilisation_note": "over the whole step (fused sample + fkcc, compaction, index conversion), the "
                                         "span the step profile covers"},
        "cpu_baseline": cpu,
        "parity": parity,
    }
    emit(line)


def run_prm_edges(a, torch, dist, rank, world, dev, stream, ctx, vamp):
    """BASELINE configs[3] edge stage: Roadmap::build_roadmap's graph over the
    first V vertices of the Fetch vertex sequence (two valid draws as start and goal, then the
    valid Halton<8> draws in order; MBM table_pick scene).  One step = the C ABI's sharded stage
    vgpu_prm_edges_allgather (each rank's queries by equal prefix work: neighbour queries, candidate
    gather, validate_motion of every candidate, device pair selection; one RCCL all-gather of the
    valid pairs; the roadmap assembled on every rank's device).  The Roadmap (offsets, adjacency,
    components) stays in HBM: the boundary's host copy -- the host Roadmap the reference returns -- is
    timed separately as `pcie_inclusive` (the same step plus the device-to-host copy into pinned
    memory), never as `value`.  Total vertices fixed (strong scaling)."""
    from vamp_amd import roadmap
    from vamp_amd._lib import check, load

    env, fx = fetch_scene(vamp)
    robot = vamp.fetch
    dim = 8
    draws = int(a.vertices / 0.6) + 4096
    rows, _, cnt = roadmap.sample_valid_shard(torch, robot, env, 1, draws, ctx, dev)
    n = min(a.vertices, cnt)
    V = rows[:n].contiguous()
    del rows
    k_np, r_np = roadmap.prm_neighbor_params(dim, robot.space_measure(), n)
    kmax = int(max(1, min(int(k_np.max()), n)))
    bound = int(np.minimum(k_np.astype(np.int64), np.arange(n, dtype=np.int64)).sum())
    comm = roadmap.Comm.from_torch(torch, dist, ctx)
    bufs = roadmap.EdgeStageBuffers(torch, n, dev, 2 * bound)
    off_h = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
    adj_h = torch.empty(max(2 * bound, 1), dtype=torch.int32, pin_memory=True)
    comp_h = torch.empty(max(n, 1), dtype=torch.int32, pin_memory=True)
    info = {}

    def step():
        roadmap.build_roadmap_edges_comm(torch, robot, env, V, comm, ctx=ctx, bufs=bufs)

    def step_d2h():  # the step plus the Roadmap's copy into pinned host memory
        off, adj, comp = roadmap.build_roadmap_edges_comm(torch, robot, env, V, comm, ctx=ctx, bufs=bufs)
        m = adj.numel()
        off_h.copy_(off, non_blocking=True)
        adj_h[:m].copy_(adj, non_blocking=True)
        comp_h[:n].copy_(comp, non_blocking=True)
        info["n_adj"] = m

    ev = []
    wall = timed_steps(a, torch, dist, dev, world, step, ev)
    step_ev_ms = ev[0]
    wall_max, units_all = reduce_over_ranks(dist, torch, wall, float(n) / world, dev, world)
    # PCIe-inclusive rate (reported beside value): the same warm-up and step count as value, each step ending in the
    # host copy; the parity checks below read the host Roadmap of the last of them
    pa = argparse.Namespace(**{**vars(a)})
    wall_pcie = timed_steps(pa, torch, dist, dev, world, step_d2h)
    wall_pcie_max, _ = reduce_over_ranks(dist, torch, wall_pcie, float(n) / world, dev, world)
    pcie_ms = wall_pcie_max / pa.steps * 1e3
    # parity of the step's graph: the torch-path pieces (edges_shard = kNN + gather + validate on this rank's
    # queries, all-gather over torch.distributed) assembled on the host by vgpu_roadmap_assemble
    k = torch.from_numpy(k_np.view(np.int32)).to(dev)
    r = torch.from_numpy(r_np).to(dev)
    qf, qc = roadmap.query_split(n, rank, world)
    assert (qf, qc) == roadmap.query_split_c(n, rank, world)
    # where one step's time goes (extra synchronised pieces outside the timed region): kNN, candidate gather
    # + validation, the pair exchange, device assembly, the device-to-host copy of the Roadmap
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pairs = roadmap.edges_shard(torch, robot, env, V, k, r, kmax, qf, qc, ctx)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        pairs = roadmap.allgather_pairs(torch, dist, pairs)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    off_d, adj_d, comp_d = roadmap.assemble_device(torch, n, pairs, ctx)
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    ph = pairs.cpu().numpy()
    off_r, adj_r, comp_r = roadmap.assemble(n, ph)  # the host assembly: the checker
    m = info["n_adj"]
    step_equal = bool(np.array_equal(off_h.numpy(), off_r) and np.array_equal(adj_h[:m].numpy().view(np.uint32), adj_r)
                      and np.array_equal(comp_h[:n].numpy().view(np.uint32), comp_r))
    info["components"] = int(len(np.unique(comp_r)))
    info["pairs"] = int(len(ph))
    del pairs, ph, off_d, adj_d, comp_d, off_r, adj_r, comp_r
    # the pieces alone with HIP events on the launch stream: the kNN kernel (both methods of vgpu_set_knn_mode:
    # brute force -- the roofline, its flops are the ones executed -- and the spatial index, auto's choice from
    # 65536 vertices), then gather + validate_motion of the candidates
    nbr = torch.empty((max(qc, 1), kmax), dtype=torch.int32, device=dev)
    dd = torch.empty((max(qc, 1), kmax), dtype=torch.float32, device=dev)
    cc = torch.empty(max(qc, 1), dtype=torch.int32, device=dev)
    knn = {}
    lists = {}
    for mode, name in ((2, "index"), (1, "brute")):
        check(load().vgpu_set_knn_mode(ctx.h, mode), ctx.h)
        reps = 1 if n >= 1_000_000 else a.steps
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            check(load().vgpu_roadmap_knn_range(ctx.h, dim, V.data_ptr(), n, qf, qc, k.data_ptr(), r.data_ptr(), kmax,
                                                nbr.data_ptr(), dd.data_ptr(), cc.data_ptr()), ctx.h)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        knn[name] = e0.elapsed_time(e1) / reps
        lists[name] = (nbr[:qc].clone(), cc[:qc].clone())
    check(load().vgpu_set_knn_mode(ctx.h, 0), ctx.h)
    if "brute" in lists:
        (nb_b, cc_b), (nb_i, cc_i) = lists["brute"], lists["index"]
        width = torch.arange(kmax, device=dev)[None, :] < cc_b[:, None].long()
        index_equals_brute = bool(torch.equal(cc_b, cc_i)) and bool(torch.equal(nb_b[width], nb_i[width]))
        del nb_b, cc_b
    else:
        index_equals_brute = None
    nb_i, cc_i = lists["index"]
    del lists
    candidates = int(cc_i.long().sum())
    offs = torch.zeros(qc + 1, dtype=torch.int32, device=dev)
    offs[1:] = torch.cumsum(cc_i, 0)
    starts = torch.empty((max(candidates, 1), dim), dtype=torch.float32, device=dev)
    goals = torch.empty_like(starts)
    okc = torch.empty(max(candidates, 1), dtype=torch.uint8, device=dev)
    nbc = torch.empty(max(candidates, 1), dtype=torch.int32, device=dev)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(stream)
    check(load().vgpu_roadmap_edge_gather(ctx.h, dim, V.data_ptr(), qf, qc, nb_i.data_ptr(), kmax, cc_i.data_ptr(),
                                          offs.data_ptr(), starts.data_ptr(), goals.data_ptr()), ctx.h)
    e1.record(stream)
    robot.validate_device(starts.data_ptr(), goals.data_ptr(), candidates, env, okc.data_ptr(), nbc.data_ptr(), ctx=ctx)
    e2.record(stream)
    torch.cuda.synchronize(dev)
    gather_ms, validate_ms = e0.elapsed_time(e1), e1.elapsed_time(e2)
    cand_interp = float(8 * nbc[:candidates].long().sum().item())
    # a strided sample of the candidate edges for the algorithmic flop count (rank 0, below)
    stride = max(1, candidates // 8192)
    cand_sample = (starts[:candidates:stride][:8192].cpu().numpy(), goals[:candidates:stride][:8192].cpu().numpy())
    del starts, goals, okc, nbc, nb_i, cc_i, offs
    phases = {"knn_index_ms": knn["index"], "gather_ms": gather_ms, "validate_ms": validate_ms,
              "validate_candidates": candidates, "validate_interpolants_full_mask_count": cand_interp,
              "validate_interpolants_per_s_full_mask_count": cand_interp / (validate_ms * 1e-3),
              "rest_of_step_ms (selection, exchange, assembly)":
                  step_ev_ms - knn["index" if n >= 65536 else "brute"] - gather_ms - validate_ms,
              "torch_path_gpu_knn_gather_validate_ms": (t1 - t0) * 1e3, "torch_path_exchange_ms": (t2 - t1) * 1e3,
              "torch_path_device_assembly_ms": (t3 - t2) * 1e3,
              "step_roadmap_equals_host_assembly_of_torch_path_pairs": step_equal,
              "roadmap_d2h_bytes": int((n + 1) * 8 + m * 4 + n * 4),
              "pcie_inclusive_ms_per_step": pcie_ms,
              "pcie_inclusive_vertices_per_s": units_all / (pcie_ms * 1e-3)}
    comm.close()
    if rank != 0:
        return
    # algorithmic work of the brute-force query kernel: one Space<8>::distance per (vertex, earlier
    # vertex) pair = 8 sub + 8 mul + 7 add + 1 sqrt (nn.hh:53-57)
    pairs_scanned = sum(range(qf, qf + qc))
    knn_ms = knn.get("brute")
    knn_brute_tflops = 24.0 * pairs_scanned / (knn_ms * 1e-3) / 1e12 if knn_ms else None
    # the step's dominant work: validate_motion of every candidate edge (the Fetch's staged bound / queue /
    # children kernels), priced in the float ops the reference executes for those edges (early exit
    # included), counted by the instrumented restatement on a strided sample of this run's candidates
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as op
    from test_oracle_fetch import fetch_env

    oenv = fetch_env(op, fx)
    f_cand = float(op.robot_validate_flops("fetch", oenv, *cand_sample, threads=host_threads()).mean())
    val_tflops = f_cand * candidates / (validate_ms * 1e-3) / 1e12
    # the spatial-index kNN: its bytes past L2 (PMC of the committed step profile at this size) over its time
    prof_w = "prm_edges" if n <= 200_000 else "prm_edges_full"
    ppath, prec = prof_record(prof_w)
    knn_bytes = None
    if prec and int(prec.get("units_per_call", 0)) == n:
        for kname, kv in (prec.get("kernels") or {}).items():
            if kname.startswith("knnidx::group_kernel") and kv.get("FETCH_SIZE") is not None:
                knn_bytes = (2 * kv["FETCH_SIZE"] + kv.get("WRITE_SIZE", 0.0)) * 1024.0
    knn_roof = {"kernel": "knnidx::group_kernel<8, 4> (causal neighbour queries through the spatial index)",
                "bound": "hbm", "ms": knn["index"], "unit": "GB/s", "peak": HBM_PEAK_GBS,
                "traffic": knn_bytes,
                "achieved_traffic_rate": knn_bytes / (knn["index"] * 1e-3) / 1e9 if knn_bytes else None,
                "frac_traffic_rate": knn_bytes / (knn["index"] * 1e-3) / 1e9 / HBM_PEAK_GBS if knn_bytes else None,
                "algorithmic_bytes": int(n * dim * 4 + qc * (4 + 8 * kmax)),
                "traffic_source": f"{ppath}: (2 x FETCH_SIZE + WRITE_SIZE) of the kernel in one timed step"
                if knn_bytes else None,
                "note": "algorithmic bytes = the vertex set once + the lists; the kernel re-reads candidate tiles "
                        "(traffic past L2, served mostly by the 256 MB Infinity Cache): its rate against the HBM peak "
                        "is the measure of how close it runs to the memory system's limit"}
    parity = None
    cpu = None
    if not a.no_cpu and world == 1:
        # the reference's host path for the stage: an exact k-d tree neighbour query (nigh's role,
        # planning/nn.hh:89-95; csrc/cpu/vcpu_roadmap.cpp) and validate_motion on the AVX2 rake
        # (csrc/cpu), over a prefix of the same vertex sequence, all host threads of this rank; at full
        # size (>= 1M vertices) the prefix is at least 1M vertices
        threads = host_threads()
        Vh = V.cpu().numpy()
        m_min = min(n, 1_000_000) if n >= 1_000_000 else 0
        m = min(n, max(4000, m_min))
        while True:  # grow the prefix until the stage takes ~cpu_seconds / 3
            t = time.perf_counter()
            nb_, _, cn_ = roadmap.cpu_knn(Vh[:m], np.arange(m), robot.space_measure(), threads=threads)
            qi = np.repeat(np.arange(m), cn_.astype(np.int64))
            qm = (np.arange(len(qi)) - np.repeat(np.cumsum(cn_.astype(np.int64)) - cn_, cn_.astype(np.int64)))
            qj = nb_[qi, qm].astype(np.int64)
            t_nn = time.perf_counter() - t
            ok_c = robot.cpu_validate_batch(Vh[qj], Vh[qi], env, threads=threads)[0]
            dt = time.perf_counter() - t
            if dt >= a.cpu_seconds / 3 or m >= n:
                break
            m = min(n, int(m * min(4.0, max(1.3, (a.cpu_seconds / max(dt, 1e-3)) ** 0.5))))
        parity = graph_parity(n, m, qi[ok_c], qj[ok_c], off_h.numpy(), adj_h[:info["n_adj"]].numpy(),
                              comp_h[:n].numpy(), roadmap)
        cpu = {"value": m / dt, "unit": "vertices/s", "cores": threads, "kind": "port",
               "measurement_boundary": "the CPU path returns a host Roadmap; compare it with "
                                       "phases.pcie_inclusive_vertices_per_s (the GPU step ending in the Roadmap's copy "
                                       "to pinned host memory, same warm-up and steps as value) -- `value` leaves the "
                                       "Roadmap in HBM (inputs and outputs resident, the bench contract)",
               "sample": f"the first {m} vertices of the same sequence: exact k-d tree neighbour queries "
                         f"(vgpu_cpu_roadmap_knn, {t_nn:.2f} s) + validate_motion of the {len(qi)} candidates on the "
                         f"AVX2 rake (mr-vamp_amd/csrc/cpu), {threads} threads, {dt:.1f} s in all; the host graph "
                         f"assembly is not included (the stage is superlinear in the vertex count: the rate at {n} is lower)",
               "cpu_model": cpu_model()}
    line = {
        "metric": "PRM edge-stage roadmap vertices/sec (Fetch 8-DOF build_roadmap: neighbour queries + edge validation)",
        "value": units_all * a.steps / wall_max,
        "unit": "vertices/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall_max / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (the Halton<8> vertex sequence of configs[3] on MBM table_pick_fetch scene0001)",
        "config": {"workload": f"BASELINE configs[3] edge stage: build_roadmap graph over {n} Fetch vertices, queries "
                               f"split over {world} GPU(s) (vgpu_prm_edges_allgather, C ABI over RCCL), one exchange "
                               f"of valid pairs, Roadmap left in HBM (its host copy: phases.pcie_inclusive_*)",
                   "robot": "Fetch", "vertices": n, "kmax": kmax, "candidate_edges_rank0": candidates,
                   "valid_edges": info.get("pairs"), "components": info.get("components"),
                   "parallelism": f"dp{world} (query ranges of equal prefix work, one all-gather)"},
        "roofline": {"kernel": "validate_motion of the step's candidate edges: the Fetch staged bound / queue / "
                               "children kernels (rank 0's candidates)", "bound": "valu",
                     "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", **utilisation(prof_w, n, step_ev_ms),
                     "reference_work_achieved": val_tflops, "reference_work_frac": val_tflops / FP32_PEAK_TFLOPS,
                     "reference_work_note": "the candidate validation's reference float ops over its own kernel time "
                                            "(validate_ms); `frac` is the executed FP32 of the whole step",
                     "kernel_ms": step_ev_ms, "validate_kernel_ms": validate_ms,
                     "algorithmic_flops_per_candidate_edge": f_cand, "candidate_edges": candidates,
                     "algorithmic_bytes_per_candidate_edge": 2 * dim * 4 + 1, **traffic_fields(prof_w, n),
                     "traffic_note": "traffic = HBM bytes of the whole step (all its kernels) from the committed profile",
                     "step_kernel_ms_events": step_ev_ms,
                     "knn_index": knn_roof,
                     "knn_brute": {"ms": knn_ms, "achieved_tflops": knn_brute_tflops,
                                   "algorithmic_flops_per_vertex_pair": 24, "vertex_pairs_rank0": pairs_scanned,
                                   "note": "the brute-force kernel (not run by the step: auto mode uses the index "
                                           "from 65536 vertices), timed for the index == brute force check"},
                     "knn_ms": knn, "knn_mode_in_step": "index" if n >= 65536 else "brute",
                     "index_equals_brute": index_equals_brute,
                     "utilisation_note": "frac / executed over the whole step (every kernel the step profile holds)"},
        "cpu_baseline": cpu,
        "parity": parity,
        "phases": phases,
    }
    emit(line)
    graph_ok = parity is None or (parity["query_lists_mismatched"] == 0 and parity.get("graph_equal") is not False)
    if not (index_equals_brute is not False and step_equal and graph_ok):
        print("PARITY FAILURE (kNN index vs brute force, the C edge stage vs the host assembly, or the roadmap vs the "
              f"CPU path): {parity}", file=sys.stderr)
        sys.exit(3)


def graph_parity(n, m, qi, qj, off, adj, comp, roadmap):
    """The step's roadmap (GPU) against the CPU path's graph (exact k-d tree neighbour queries + the AVX2 rake,
    build_roadmap's append order) on the queries 0 .. m-1 the CPU leg ran: vertex i's own list -- the leading
    entries < i of its adjacency list, appended when i was inserted (prm.hh:267-276) -- must equal i's valid
    CPU neighbours in order; with m = n also the whole Roadmap (offsets, adjacency, components) of the host
    assembly of the CPU pairs."""
    off = np.asarray(off, np.int64)
    adj = np.asarray(adj).view(np.uint32).astype(np.int64)
    owner = np.repeat(np.arange(n, dtype=np.int64), np.diff(off))
    own = adj < owner
    g_i, g_j = owner[own], adj[own]
    keep = g_i < m
    g_i, g_j = g_i[keep], g_j[keep]
    c_i, c_j = np.asarray(qi, np.int64), np.asarray(qj, np.int64)
    if len(g_i) == len(c_i) and np.array_equal(g_i, c_i) and np.array_equal(g_j, c_j):
        bad = 0
    else:  # per query: which lists differ
        gs = np.searchsorted(g_i, np.arange(m + 1))
        cs = np.searchsorted(c_i, np.arange(m + 1))
        bad = sum(1 for i in range(m) if not np.array_equal(g_j[gs[i]:gs[i + 1]], c_j[cs[i]:cs[i + 1]]))
    rec = {"queries_compared": int(m), "query_lists_mismatched": int(bad), "valid_pairs_gpu": int(len(g_i)),
           "valid_pairs_cpu": int(len(c_i)),
           "checker": "CPU path on the same vertices: vgpu_cpu_roadmap_knn (exact k-d tree) + the AVX2 rake "
                      "(mr-vamp_amd/csrc/cpu), valid pairs in query order"}
    if m == n:
        o2, a2, c2 = roadmap.assemble(n, np.stack([c_i, c_j], 1).astype(np.uint32))
        rec["graph_equal"] = bool(np.array_equal(off, o2) and np.array_equal(adj, a2.astype(np.int64)) and
                                  np.array_equal(np.asarray(comp).view(np.uint32), c2))
        rec["graph_checker"] = "vgpu_roadmap_assemble (host) of the CPU pairs: offsets, adjacency, components"
    return rec


def timed_steps(a, torch, dist, dev, world, step, events=None):
    """warmup, then exactly `steps` steps between barrier + synchronize; returns wall seconds.  events: a
    list that receives the per-step milliseconds between HIP events recorded on the current (launch)
    stream around the steps"""
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.steps):
        step()
    e1.record()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    if events is not None:
        events.append(e0.elapsed_time(e1) / a.steps)
    return t1 - t0


VALU_ISSUE_PER_S = 256 * 4 * 2.4e9 / 2  # 1024 SIMDs x one wave64 VALU instruction per 2 cycles at 2.4 GHz


def executed_record(workload, units, kernel_ms):
    """Hardware utilisation beside the reference-work `frac`: the executed VALU instructions and FP32
    operations per unit from the newest committed PMC record of the same workload (profiles/rNN_prof_<w>.json:
    tools/pmc_drive.py under rocprofv3, tools/pmc_report.py), times this run's units, over this run's
    kernel time.  valu_issue_frac = SQ_INSTS_VALU / (time x 1.2288e12 wave-instructions/s);
    fp32_exec_frac = 64 x (ADD + MUL + 2 FMA) / time / peak."""
    path, rec = prof_record(workload)
    if not rec or not kernel_ms:
        return None
    pu = rec.get("per_unit") or {}
    if not pu.get("valu_insts"):
        return None
    t = kernel_ms * 1e-3
    hbm = rec.get("hbm_bytes_per_call")
    return {"valu_issue_frac": pu["valu_insts"] * units / t / VALU_ISSUE_PER_S,
            "fp32_exec_frac": pu["fp32_ops"] * units / t / 1e12 / FP32_PEAK_TFLOPS,
            "fp_share_of_valu_insts": pu.get("fp_insts_share_of_valu"),
            "wait_frac": rec.get("wait_frac"),
            "valu_insts_per_unit": pu["valu_insts"], "fp32_ops_per_unit": pu["fp32_ops"],
            "hbm_bytes_per_call_pmc": hbm * units / rec["units_per_call"] if hbm else None,
            "pmc_kernel_ms_per_call": rec.get("kernel_ms_per_call"), "pmc_units_per_call": rec.get("units_per_call"),
            "source": path + " (committed PMC of the same workload's step; per-unit counts x this run's units / "
                             "this run's kernel time)"}


FRAC_MEANING = ("executed FP32 utilisation: 64 x (ADD + MUL + 2 FMA) FP32 VALU instructions per unit from the committed PMC "
                "record of this workload's step (profiles/rNN_prof_<workload>.json, same build) x this run's units / this "
                "run's kernel time / the FP32 peak -- what the hardware executed, bounded by 1.  The reference's own work "
                "(its float ops for these inputs, early exits included, counted by the instrumented oracle) over the same "
                "time is `reference_work_frac`: it counts work the GPU legitimately skips (mid spheres, the wrist gate, "
                "never-firing self checks, the obstacle prefilter), so it measures algorithmic savings plus speed and may "
                "exceed 1")


def utilisation(workload, units, kernel_ms, ref_flops=None):
    """The roofline's rate fields: `achieved` / `frac` = EXECUTED FP32 (bounded by 1) from the
    committed PMC record of the same workload's step over this run's kernel time; `frac_at_profile_time` = the same
    count over the record's own kernel time (what the record alone recomputes to); `reference_work_achieved` /
    `reference_work_frac` = the reference's float ops (ref_flops per launch) over this run's kernel time."""
    ex = executed_record(workload, units, kernel_ms) if workload else None
    _, rec = prof_record(workload) if workload else (None, None)
    out = {"achieved": None, "frac": None, "frac_at_profile_time": None}
    if ex:
        out["frac"] = ex["fp32_exec_frac"]
        out["achieved"] = ex["fp32_exec_frac"] * FP32_PEAK_TFLOPS
        if rec and rec.get("kernel_ms_per_call"):
            out["frac_at_profile_time"] = rec["fp32_ops_per_call"] / (rec["kernel_ms_per_call"] * 1e-3) / 1e12 / \
                FP32_PEAK_TFLOPS
    if ref_flops is not None and kernel_ms:
        ra = ref_flops / (kernel_ms * 1e-3) / 1e12
        out["reference_work_achieved"] = ra
        out["reference_work_frac"] = ra / FP32_PEAK_TFLOPS
    out["frac_meaning"] = FRAC_MEANING
    out["executed"] = ex
    return out


def phase_utilisation(workload, units, phase_ms):
    """executed FP32 fraction per validate phase: the record's per-kernel FP32 counts split by source kind (head:
    the lead, bound, children, count and queue kernels of SrcHeadT; tail: those of SrcTailT), scaled to this run's
    units, over this run's phase times (HIP events inside the library).  Bounded by 1 like `frac`."""
    _, rec = prof_record(workload)
    if not rec or not rec.get("kernels"):
        return None
    fp = {"head": 0.0, "tail": 0.0}
    for name, k in rec["kernels"].items():
        ops = 64.0 * (k.get("SQ_INSTS_VALU_ADD_F32", 0) + k.get("SQ_INSTS_VALU_MUL_F32", 0) +
                      2 * k.get("SQ_INSTS_VALU_FMA_F32", 0))
        if "SrcHeadT" in name:
            fp["head"] += ops
        elif "SrcTailT" in name:
            fp["tail"] += ops
    scale = units / rec["units_per_call"]
    return {p: (fp[p] * scale / (phase_ms[p] * 1e-3) / 1e12 / FP32_PEAK_TFLOPS if phase_ms.get(p) else None)
            for p in fp}


def contract_line(a, world, wall_max, units_all, metric, unit, scaling, data, config, roofline, cpu):
    return {"metric": metric, "value": units_all * a.steps / wall_max, "unit": unit, "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": wall_max / a.steps * 1e3, "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32", "data": data, "config": config,
            "roofline": roofline, "cpu_baseline": cpu}


def pair_scene_env(vamp):
    """configs[4]'s scene (tests/oracle_py.py pair_scene: a table and 3 spheres) as an Environment"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as op

    oenv = op.pair_scene()
    env = vamp.Environment()
    for x, y, z, r, _ in oenv.spheres:
        env.add_sphere(vamp.Sphere([x, y, z], r))
    for row in oenv.cuboids + oenv.zcuboids:
        env.add_cuboid(vamp.Cuboid.from_axes(row[0:3], row[3:6], row[6:9], row[9:12], row[12:15]))
    return env, oenv


def make_pair_edges(torch, robot, env, E, seed, dev, ctx):
    """configs[4] edges: pairs of collision-free composite configurations (drawn on the device, checked
    with the composite fkcc), each arm's sub-edge capped at length 1.0"""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    sm = torch.tensor(S_M * 2, device=dev)
    sa = torch.tensor(S_A * 2, device=dev)
    pool, have = [], 0
    while have < 2 * E:
        m = 1 << 21
        q = torch.addcmul(sa, torch.rand((m, 14), generator=g, device=dev), sm).contiguous()
        ok = torch.empty(m, dtype=torch.uint8, device=dev)
        robot.fkcc_device(q.data_ptr(), m, env, ok.data_ptr(), ctx)
        torch.cuda.synchronize(dev)
        v = q[ok.bool()]
        pool.append(v)
        have += v.shape[0]
    vq = torch.cat(pool)[: 2 * E]
    starts, goals = vq[0::2].contiguous(), vq[1::2].clone()
    for sl in (slice(0, 7), slice(7, 14)):
        d = torch.linalg.vector_norm((goals[:, sl] - starts[:, sl]).double(), dim=1)
        sc = torch.clamp(1.0 / torch.clamp(d, min=1e-9), max=1.0).float()
        goals[:, sl] = starts[:, sl] + (goals[:, sl] - starts[:, sl]) * sc[:, None]
    return starts, goals.contiguous()


def run_pair(a, torch, dist, rank, world, dev, stream, ctx, vamp):
    """BASELINE configs[4]: two Pandas (bases (0,0,0) and (1,0,0)), 14-dof
    edges between collision-free composite configurations, each arm's sub-edge capped at 1.0;
    validate_motion over the composite (fkcc of both arms + inter-arm spheres).  Independent edge
    shards per rank (weak scaling, no collective)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as op

    env, oenv = pair_scene_env(vamp)
    robot = vamp.panda_pair
    strong = a.scaling == "strong"
    E = a.edges
    starts, goals = make_pair_edges(torch, robot, env, E, shard_seed(0 if strong else rank), dev, ctx)
    if strong:  # one fixed batch, this rank's contiguous range, through pinned host memory
        lo, E = strong_slice(a.edges, rank, world)
        starts, goals = starts[lo:lo + E].contiguous(), goals[lo:lo + E].contiguous()
        pinned = PinnedShard(torch, starts, goals, dev)
    okd = torch.empty(E, dtype=torch.uint8, device=dev)
    nb = torch.empty(E, dtype=torch.int32, device=dev)

    def step():
        if strong:
            pinned.step(robot, env, okd, nb, ctx)
        else:
            robot.validate_device(starts.data_ptr(), goals.data_ptr(), E, env, okd.data_ptr(), nb.data_ptr(), ctx)

    ev = []
    wall = timed_steps(a, torch, dist, dev, world, step, ev)
    kern_ms = ev[0]
    # rake/early-exit units from the CPU rake on the same edges (bit-identical results), as configs[1]
    _, c_nb, c_ne = robot.cpu_validate_batch(starts.cpu().numpy(), goals.cpu().numpy(), env, threads=host_threads())
    units = float(8 * c_ne.astype(np.int64).sum())
    wall_max, units_all = reduce_over_ranks(dist, torch, wall, units, dev, world)
    _, units_full_all = reduce_over_ranks(dist, torch, wall, float(8 * c_nb.astype(np.int64).sum()), dev, world)
    if rank != 0:
        return
    s_np, g_np = starts[:256].cpu().numpy(), goals[:256].cpu().numpy()
    fl = op.pair_validate_flops(oenv, s_np, g_np)  # executed float ops per edge, reference semantics
    f_edge = float(np.mean(fl))
    cpu = None
    parity = None
    if not a.no_cpu and world == 1:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        sc_, gc_ = starts.cpu().numpy(), goals.cpu().numpy()
        n0 = 2048 * threads
        t = time.perf_counter()
        robot.cpu_validate_batch(sc_[:n0], gc_[:n0], env, threads=threads)
        dt0 = max(time.perf_counter() - t, 1e-3)
        m = int(min(len(sc_), n0 * a.cpu_seconds / dt0))
        t = time.perf_counter()
        okc, nbc, nec = robot.cpu_validate_batch(sc_[:m], gc_[:m], env, threads=threads)
        dt = time.perf_counter() - t
        g_ok, g_nb = okd.cpu().numpy(), nb.cpu().numpy()
        oo, on = op.pair_validate_motions(oenv, sc_[:8192], gc_[:8192], threads=threads)
        parity = {"cpu_rake": parity_record(g_ok, g_nb, okc, nbc, f"mr-vamp_amd/csrc/cpu AVX2 rake, first {m} edges"),
                  "oracle": parity_record(g_ok, g_nb, oo, on, "oracle/vamp_oracle.c vo_pair_validate_motions, "
                                                              "first 8192 edges")}
        cpu = {"value": float(8 * nec.astype(np.int64).sum()) / dt, "unit": "interpolants/s", "cores": threads,
               "kind": "port", "counting": "rake_early_exit",
               "value_full_mask_count": float(8 * nbc.astype(np.int64).sum()) / dt,
               "sample": f"{m} edges of the same workload, mr-vamp_amd/csrc/cpu AVX2 rake (composite), "
                         f"{threads} threads, {dt:.1f} s", "cpu_model": cpu_model()}
    line = contract_line(
        a, world, wall_max, units_all,
        "validated edge-interpolants/sec (2x Panda 14-DOF composite FK+CC with inter-robot collision)",
        "interpolants/s", a.scaling,
        "synthetic (seeded uniform composite configurations; collision-free endpoints, each arm's sub-edge capped at 1.0)",
        {"workload": f"BASELINE configs[4]: PandaBase<0,0,0> + PandaBase<100,0,0>, {E} edges per GPU, table + 3 spheres"
                     if not strong else f"BASELINE configs[4] strong scaling: {a.edges} composite edges split over "
                                        f"{world} GPU(s), H2D from pinned host memory + validate + D2H per step",
         "robot": "panda_pair", "edges_per_gpu": E, "interpolants_per_gpu": units,
         "edge_valid_fraction": float(okd.float().mean().item()),
         "parallelism": f"dp{world} (independent edge shards, no collective)"},
        {"kernel": "pair_validate_head/tail kernels (one validate_motions call)", "bound": "valu",
         "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", **utilisation("pair" if not strong else None, E, kern_ms,
                                                                     f_edge * E),
         **traffic_fields("pair", E), "algorithmic_flops_per_edge": f_edge, "kernel_ms": kern_ms,
         "step_ms_wall": wall / a.steps * 1e3},
        cpu)
    line["counting"] = "rake_early_exit (8 x rake blocks the reference evaluates)"
    line["value_full_mask_count"] = units_full_all * a.steps / wall_max
    line["parity"] = parity
    emit(line)


def RRTC_SETTINGS(vamp):
    """RRTCSettings of the MBM runs: range 1.0, 1e6 iterations / samples (src/vamp/constants.py:1,49-55)"""
    return vamp.RRTCSettings(range=1.0, max_iterations=1000000, max_samples=1000000)


def rrtc_problems(vamp, robot_name):
    """(environments, starts, goals, robot, description) of the rrtc workload.
    panda: the 16 MotionBenchMaker table_pick problems (scene + request 1..16, resolved into
    tests/golden/panda_table_pick_problems.npz), one environment each, PandaBase<0,0,0>.
    panda_pair: configs[4]'s planner half -- 16 composite problems on configs[4]'s scene (a table and three spheres,
    pair_scene_env), start and goal collision-free composite configurations whose straight edge is invalid, drawn
    from a seeded uniform stream and filtered by the CPU rake (the same draws as tests/test_rrtc.py pair_problems)."""
    if robot_name == "panda_pair":
        env, _ = pair_scene_env(vamp)
        robot = vamp.panda_pair
        rng = np.random.default_rng(41)
        q = robot.scale_configuration(rng.random((40 * 16, 14), dtype=np.float32))
        q = q[robot.cpu_fkcc_batch(q, env)]
        s, g = q[0::2][:8 * 16], q[1::2][:8 * 16]
        m = min(len(s), len(g))
        ok, _, _ = robot.cpu_validate_batch(s[:m], g[:m], env)
        hard = np.nonzero(~ok)[0][:16]
        return [env] * 16, list(s[hard]), list(g[hard]), robot, \
            "configs[4] composite: 16 problems on the table + 3 spheres scene (straight edge invalid)"
    fx = np.load(os.path.join(ROOT, "tests", "golden", "panda_table_pick_problems.npz"), allow_pickle=False)
    P = int(fx["n_problems"])
    envs, starts, goals = [], [], []
    for k in range(1, P + 1):
        env = vamp.Environment()
        for row in fx[f"p{k}_env_spheres"]:
            env.add_sphere(vamp.Sphere(row[0:3], float(row[3])))
        for row in np.concatenate([fx[f"p{k}_env_cuboids"], fx[f"p{k}_env_zcuboids"]]):
            env.add_cuboid(vamp.Cuboid.from_axes(row[0:3], row[3:6], row[6:9], row[9:12], row[12:15]))
        for row in np.concatenate([fx[f"p{k}_env_capsules"], fx[f"p{k}_env_zcapsules"]]):
            p1 = np.array(row[0:3], np.float32)
            env.add_capsule(vamp.Cylinder(p1, (p1 + np.array(row[3:6], np.float32)).astype(np.float32), float(row[6])))
        envs.append(env)
        starts.append(fx[f"p{k}_start"])
        goals.append(fx[f"p{k}_goal"])
    return envs, starts, goals, vamp.panda_0_0, "MBM table_pick_panda scene/request 0001-0016"


def run_rrtc(a, torch, dist, rank, world, dev, stream, ctx, vamp):
    """BASELINE configs[0]: Panda RRT-Connect (planning/rrtc.hh) on the
    MotionBenchMaker table_pick problems (scene + request 1..16, resolved into
    tests/golden/panda_table_pick_problems.npz), CPU only -- the planner and its validate_vector
    checks on the CPU rake, one core, RRTCSettings range 1.0 / 1e6 iterations, Halton<7> reset per
    problem (scripts/evaluate_mbm.py:95-96), PandaBase<0,0,0> (the scenes are origin-centred) and
    the fork's default Panda (2,2,0) on problem 1.  One step = one solve of every problem; the
    value is the median planning time (PlanningResult.nanoseconds).  Every solved path's segments
    are re-checked on the GPU (vgpu_validate_motions) against the CPU rake -- that batch is the line's
    roofline (HIP events, its step profile profiles/rNN_prof_rrtc.json).  N ranks = replicas.
    --robot panda_pair: configs[4]'s planner half, RRT-Connect on the two-Panda composite (rrtc_problems)."""
    pair = a.robot == "panda_pair"
    envs, starts, goals, robot0, desc = rrtc_problems(vamp, a.robot)
    P = len(starts)
    settings = RRTC_SETTINGS(vamp)
    runs = [(robot0, k) for k in range(P)] + ([] if pair else [(vamp.panda, 0)])
    results = []

    def step():
        results.clear()
        for robot, k in runs:
            results.append(robot.rrtc(starts[k], goals[k], envs[k], settings, robot.halton()))

    wall = timed_steps(a, torch, dist, dev, world, step)
    wall_max, _ = reduce_over_ranks(dist, torch, wall, 0.0, dev, world)
    if rank != 0:
        return
    ns = np.array([r.nanoseconds for r in results[:P]], np.float64)
    its = np.array([r.iterations for r in results[:P]])
    # the solved paths' segments through the GPU batch path vs the CPU rake (same edges)
    seg_s = np.concatenate([r.path[:-1] for r in results[:P] if r.solved])
    seg_g = np.concatenate([r.path[1:] for r in results[:P] if r.solved])
    owner = np.concatenate([np.full(len(r.path) - 1, i) for i, r in enumerate(results[:P]) if r.solved])
    gpu_ok = np.zeros(len(seg_s), bool)
    cpu_ok = np.zeros(len(seg_s), bool)
    groups = [np.ones(len(seg_s), bool)] if pair else [owner == i for i in range(P)]
    for i, m in enumerate(groups):
        if m.any():
            gpu_ok[m] = robot0.validate_batch(seg_s[m], seg_g[m], envs[i], ctx)[0]
            cpu_ok[m] = robot0.cpu_validate_batch(seg_s[m], seg_g[m], envs[i], threads=1)[0]
    # the roofline: the GPU leg's batch (all segments of the composite; for the Panda, one scene per problem, the
    # problem with the most segments) resident in HBM, HIP events on the launch stream
    k0 = 0 if pair else int(np.argmax([m.sum() for m in groups]))
    m0 = groups[k0]
    ds, dg = torch.from_numpy(seg_s[m0]).to(dev), torch.from_numpy(seg_g[m0]).to(dev)
    E = int(m0.sum())
    okd = torch.empty(E, dtype=torch.uint8, device=dev)
    nbd = torch.empty(E, dtype=torch.int32, device=dev)
    for _ in range(3):
        robot0.validate_device(ds.data_ptr(), dg.data_ptr(), E, envs[k0], okd.data_ptr(), nbd.data_ptr(), ctx)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(20):
        robot0.validate_device(ds.data_ptr(), dg.data_ptr(), E, envs[k0], okd.data_ptr(), nbd.data_ptr(), ctx)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    seg_ms = e0.elapsed_time(e1) / 20
    prof_w = "rrtc_pair" if pair else "rrtc"
    roof = {"kernel": "vgpu_validate_motions of the solved paths' segments (the line's GPU leg), "
                      + ("all 16 problems' segments, one batch" if pair else
                         f"problem {k0 + 1}'s segments (the most of the 16; one scene per problem)"),
            "bound": "latency (a few hundred edges: far below one wave per CU)", "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s", **utilisation(prof_w, E, seg_ms), **traffic_fields(prof_w, E), "kernel_ms": seg_ms,
            "segments": E, "algorithmic_bytes_per_segment": 2 * robot0.dimension() * 4 + 1 + 4}
    med_us = float(np.median(ns)) / 1e3
    line = {
        "metric": ("2x Panda composite RRT-Connect planning time, median (CPU rake)" if pair else
                   "Panda MBM RRT-Connect planning time, median (CPU rake)"), "value": med_us, "unit": "us",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": wall_max / a.steps * 1e3,
        "higher_is_better": False, "scaling": "replicas", "vs_baseline": None if pair else med_us / 35.0,
        "dtype": "f32",
        "data": ("synthetic (seeded uniform composite configurations on configs[4]'s scene)" if pair else
                 "MotionBenchMaker table_pick_panda scene/request 0001-0016 (resources/panda/problems.tar.bz2, resolved "
                 "into tests/golden/panda_table_pick_problems.npz)"),
        "config": ({"workload": f"BASELINE configs[4] planner: 2x Panda composite (14-DOF) RRT-Connect, {desc}",
                    "robot": "panda_pair (PandaBase<0,0,0> + PandaBase<100,0,0>)", "planner": "RRTC<PandaPair, 8, 32>",
                    "settings": "range 1.0, dynamic domain, balanced, 1e6 iterations/samples, Halton<14> reset per problem",
                    "parallelism": "one core per problem (replicas over ranks)"} if pair else
                   {"workload": f"BASELINE configs[0]: Panda 7-DOF RRT-Connect, {P} MBM table_pick problems, CPU only",
                    "robot": "PandaBase<0,0,0> (+ Panda (2,2,0) on problem 1)", "planner": "RRTC<Panda, 8, 32>",
                    "settings": "range 1.0, dynamic domain, balanced, 1e6 iterations/samples, Halton<7> reset per problem",
                    "parallelism": "one core per problem (replicas over ranks)"}),
        "problems": [{"problem": k + 1, "solved": bool(r.solved), "ns": int(r.nanoseconds), "iterations": int(r.iterations),
                      "path_len": int(len(r.path)), "cost": float(r.cost), "trees": list(r.size)}
                     for k, r in enumerate(results[:P])],
        "solved": int(sum(r.solved for r in results[:P])), "iterations_median": float(np.median(its)),
        "path_segments": {"count": int(len(seg_s)), "gpu_valid": int(gpu_ok.sum()),
                          "gpu_vs_cpu_rake_mismatches": int((gpu_ok != cpu_ok).sum())},
        "roofline": roof,
        "cpu_baseline": None, "cpu_model": cpu_model(),
    }
    if pair:
        line["baseline_note"] = "no reference counterpart (the reference has no composite robot, SURVEY §0 finding 10)"
    else:
        line["baseline_note"] = ("vs_baseline = median / 35 us, the reference README's median over all MBM problems on one "
                                 "desktop core (BASELINE.md); this run: table_pick only, GPU box host core")
        b220 = results[P]
        line["panda_2_2_0_problem1"] = {"solved": bool(b220.solved), "ns": int(b220.nanoseconds),
                                        "iterations": int(b220.iterations)}
    emit(line)


def run_capt(a, torch, dist, rank, world, dev, stream, ctx, vamp):
    """BASELINE configs[2]: Panda vs a 10k-point CAPT (points on the 14
    cage spheres, r_min 0.012, r_max 0.06, r_point 0.0025), per-configuration fkcc of 2^20 uniform
    configurations against the point-cloud-only environment.  Independent shards per rank."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import scenes

    pts = scenes.cage_points(10000, seed=1)
    env = vamp.Environment()
    env.add_pointcloud(pts, scenes.R_MIN, scenes.R_MAX, scenes.R_POINT)
    robot = vamp.panda_0_0
    N = a.edges
    g = torch.Generator(device=dev)
    g.manual_seed(2 + 7919 * rank)
    q = torch.addcmul(torch.tensor(S_A, device=dev), torch.rand((N, 7), generator=g, device=dev),
                      torch.tensor(S_M, device=dev)).contiguous()
    ok = torch.empty(N, dtype=torch.uint8, device=dev)

    def step():
        robot.fkcc_device(q.data_ptr(), N, env, ok.data_ptr(), ctx)

    ev = []
    wall = timed_steps(a, torch, dist, dev, world, step, ev)
    kern_ms = ev[0]
    wall_max, units_all = reduce_over_ranks(dist, torch, wall, float(N), dev, world)
    # configs[2]'s "1M collision queries" as raw CAPT::collides_simd sphere queries (scenes.raw_queries:
    # x, y ~ U[-1, 1], z ~ U[0, 1.2], r ~ U[r_min, r_max]), outside the contract's timed region
    rq_c, rq_r = scenes.raw_queries(1 << 20)
    cd, rd = torch.from_numpy(rq_c).to(dev), torch.from_numpy(rq_r).to(dev)
    rq_out = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    hp = env.handle(ctx)

    def raw():
        env.pointcloud_collides_device(cd.data_ptr(), rd.data_ptr(), 1 << 20, rq_out.data_ptr(), simd=True, ctx=ctx)

    for _ in range(3):
        raw()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(20):
        raw()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    raw_ms = e0.elapsed_time(e1) / 20
    # the cell grid's build (vgpu_capt_grid.hip) is part of each device upload: time one re-upload
    t = time.perf_counter()
    env._changed()
    env.handle(ctx)
    torch.cuda.synchronize(dev)
    upload_ms = (time.perf_counter() - t) * 1e3
    # an incremental change (Environment.attach / detach, environment.cc:161-163): only the blob's tail is
    # re-sent, the cloud and its cell grid stay (vgpu_env_upload_stats counts the grid builds)
    from vamp_amd._lib import check as _check, load as _load
    att = vamp.Attachment([0.0, 0.0, 0.1], [0.0, 0.0, 0.0, 1.0])
    att.add_sphere(vamp.Sphere([0.0, 0.0, 0.05], 0.03))
    st0 = env.upload_stats(ctx)
    t = time.perf_counter()
    for _ in range(10):
        env.attach(att)
        _check(_load().vgpu_env_upload(env.handle(ctx)), ctx.h)
        env.detach()
        _check(_load().vgpu_env_upload(env.handle(ctx)), ctx.h)
    incr_ms = (time.perf_counter() - t) * 1e3 / 20
    st1 = env.upload_stats(ctx)
    del hp
    if rank != 0:
        return
    import oracle_py as op
    oenv = op.Env().add_pointcloud(pts, scenes.R_MIN, scenes.R_MAX, scenes.R_POINT)
    raw_want = op.Capt(pts, scenes.R_MIN, scenes.R_MAX, scenes.R_POINT).collides(rq_c[:1 << 17], rq_r[:1 << 17],
                                                                                 simd=True)
    raw_got = rq_out[:1 << 17].cpu().numpy().astype(bool)
    qs = q[:2048].cpu().numpy()
    _, _, _, fl = op.fkcc(oenv, qs, (0, 0, 0), stats=True)
    f_cfg = float(fl.mean())
    cpu = None
    parity = None
    if not a.no_cpu and world == 1:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        qc = q.cpu().numpy()
        n0 = 4096 * threads
        t = time.perf_counter()
        robot.cpu_fkcc_batch(qc[:n0], env, threads=threads)
        dt0 = max(time.perf_counter() - t, 1e-3)
        m = int(min(len(qc), n0 * a.cpu_seconds / dt0))
        t = time.perf_counter()
        okc = robot.cpu_fkcc_batch(qc[:m], env, threads=threads)
        dt = time.perf_counter() - t
        g_ok = ok.cpu().numpy().astype(bool)
        oo = op.fkcc_threads(oenv, qc[:65536], (0, 0, 0), threads).astype(bool)
        parity = {"cpu_rake": {"configs_compared": int(m), "mismatches": int((g_ok[:m] != okc).sum()),
                               "checker": "mr-vamp_amd/csrc/cpu AVX2 rake fkcc + CAPT"},
                  "oracle": {"configs_compared": 65536, "mismatches": int((g_ok[:65536] != oo).sum()),
                             "checker": "oracle/vamp_oracle.c fkcc + CAPT"}}
        cpu = {"value": m / dt, "unit": "configs/s", "cores": threads, "kind": "port",
               "sample": f"{m} configurations of the same workload, mr-vamp_amd/csrc/cpu AVX2 rake fkcc (broadcast "
                         f"block per configuration, CAPT collides_simd), {threads} threads, {dt:.1f} s",
               "cpu_model": cpu_model()}
    tf = traffic_fields("capt", N)
    line = contract_line(
        a, world, wall_max, units_all, "CAPT point-cloud collision queries/sec (Panda 7-DOF fkcc vs 10k-point cloud)",
        "configs/s", "weak", "synthetic (10k points on the cage spheres, seed 1; uniform Panda configurations)",
        {"workload": f"BASELINE configs[2]: Panda 7-DOF vs 10k-point CAPT, {N} configurations per GPU",
         "robot": "PandaBase<0,0,0>", "configs_per_gpu": N, "valid_fraction": float(ok.float().mean().item()),
         "parallelism": f"dp{world} (independent shards, no collective)"},
        {"kernel": "fkcc (staged, point-cloud ext path)", "bound": "valu",
         "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", **utilisation("capt", N, kern_ms, f_cfg * N), **tf,
         "algorithmic_bytes_per_config": 7 * 4 + 1, "algorithmic_flops_per_config": f_cfg, "kernel_ms": kern_ms,
         "step_ms_wall": wall / a.steps * 1e3,
         "note": "latency-bound gathers, not FLOPs: the cell grid (vgpu_capt_grid.hip) decides most sphere queries "
                 "with one dependent 8-B load after the sphere's FK; undecided ones are queued per wave in LDS and "
                 "resolved a full wave at a time (descent from the cell's node, leaf box, affordance scan: "
                 "~3-8 dependent L2 loads); CAPT arrays + grid (~21 MB) L2/MALL resident"},
        cpu)
    line["parity"] = parity
    line["raw_queries"] = {
        "queries": 1 << 20, "ms": raw_ms, "queries_per_s": (1 << 20) / raw_ms * 1e3,
        "hit_fraction": float(rq_out.float().mean().item()),
        "oracle_mismatches": int((raw_got != raw_want).sum()), "oracle_compared": 1 << 17,
        "note": "one lane per sphere, CAPT::collides_simd semantics (capt.hh:457-541) through the cell grid; HIP events"}
    line["environment_upload_ms"] = {"ms": upload_ms, "note": "one re-realisation of the environment on the device: "
                                                              "handle create, CAPT arrays from the host twin, blob upload, "
                                                              "cell-grid build (host wall clock)",
                                     "incremental_ms": incr_ms,
                                     "incremental_grid_builds": st1["grids"] - st0["grids"],
                                     "incremental_note": "Environment.attach or detach + vgpu_env_upload (tail only, "
                                                         "in place), mean of 20, host wall clock"}
    emit(line)


_OUT = None  # the process's real stdout (fd 1 is pointed at stderr while the bench runs)


def emit(line):
    """The contract's one JSON line, on the real stdout.  Everything else -- including banners that native
    libraries printf to fd 1 (RCCL prints its version at communicator creation) -- goes to stderr."""
    out = _OUT or sys.stdout
    out.write(json.dumps(line) + "\n")
    out.flush()


def main():
    global _OUT
    a = parse()
    sys.stdout.flush()
    _OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world > 1:
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import vamp_amd as vamp

    ctx = vamp.context(local)
    # one explicit stream for torch plumbing AND the vgpu launches, so the HIP events below
    # bracket exactly the kernels (the legacy default stream would be handle 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    if a.workload != "validate":
        {"fetch_prm": run_fetch_prm, "prm_edges": run_prm_edges, "pair": run_pair, "capt": run_capt,
         "rrtc": run_rrtc}[a.workload](
            a, torch, dist, rank, world, dev, stream, ctx, vamp)
        if world > 1:
            dist.destroy_process_group()
        return
    env, oenv, scene_desc = scene_envs(vamp, a.scene)
    base = (0, 0, 0) if a.base == "000" else (200, 200, 0)
    robot = vamp.PandaBase(*base)

    strong = a.scaling == "strong"
    if strong:  # one fixed batch (the same seed on every rank), this rank's contiguous range
        s_full, g_full = make_edges(torch, vamp, env, robot, a.edges, seed=shard_seed(0), dev=dev, edge_set=a.edge_set)
        lo, E = strong_slice(a.edges, rank, world)
        starts, goals = s_full[lo:lo + E].contiguous(), g_full[lo:lo + E].contiguous()
        del s_full, g_full
        pinned = PinnedShard(torch, starts, goals, dev)
    else:
        E = a.edges
        starts, goals = make_edges(torch, vamp, env, robot, E, seed=shard_seed(rank), dev=dev, edge_set=a.edge_set)
    ok = torch.empty(E, dtype=torch.uint8, device=dev)
    nb = torch.empty(E, dtype=torch.int32, device=dev)

    def step():
        if strong:
            pinned.step(robot, env, ok, nb, ctx)
        else:
            robot.validate_device(starts.data_ptr(), goals.data_ptr(), E, env, ok.data_ptr(), nb.data_ptr(), ctx)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    ok_frac = float(ok.float().mean().item())
    # Units: the reference's early exit counts the interpolants of the rake blocks
    # it evaluates -- up to and including an edge's first invalid block.  Those counts come from the
    # CPU rake on the same edges (bit-identical results, and it reports the first failing block);
    # the GPU's own results are compared with it edge by edge below.
    s_all, g_all = starts.cpu().numpy(), goals.cpu().numpy()
    if not a.no_cpu and world == 1:
        cpu_leg, c_ok, c_nb, c_ne = cpu_rake_baseline(vamp, env, robot, s_all, g_all, a.cpu_seconds)
    else:
        c_ok, c_nb, c_ne = robot.cpu_validate_batch(s_all, g_all, env, threads=host_threads())
    units_local = float(8 * c_ne.astype(np.int64).sum())       # rake_early_exit
    units_full_local = float(8 * c_nb.astype(np.int64).sum())  # every interpolant of every edge

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    wall = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / a.steps  # HIP events on the launch stream

    wall_max, units_all = reduce_over_ranks(dist, torch, wall, units_local, dev, world)
    _, units_full_all = reduce_over_ranks(dist, torch, wall, units_full_local, dev, world)

    # secondary leg (untimed for the headline): the HBM-bound sphere_fk stream, 4M configs
    fk_leg = None
    if a.fk_leg and rank == 0:
        nq = 1 << 22
        q = torch.rand((nq, 7), device=dev, dtype=torch.float32) * 6.0 - 3.0
        out = torch.empty((3, 59, nq), device=dev, dtype=torch.float32)
        for _ in range(2):
            robot.sphere_fk_device(q.data_ptr(), nq, out.data_ptr(), nq, ctx)
        f0 = torch.cuda.Event(enable_timing=True)
        f1 = torch.cuda.Event(enable_timing=True)
        f0.record(stream)
        reps = 10
        for _ in range(reps):
            robot.sphere_fk_device(q.data_ptr(), nq, out.data_ptr(), nq, ctx)
        f1.record(stream)
        torch.cuda.synchronize(dev)
        fk_ms = f0.elapsed_time(f1) / reps
        gbs = 736.0 * nq / (fk_ms * 1e-3) / 1e9
        fk_leg = {"kernel": "panda_sphere_fk_kernel", "bound": "hbm", "configs": nq, "ms": fk_ms,
                  "configs_per_s": nq / (fk_ms * 1e-3), "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": gbs / HBM_PEAK_GBS, "bytes_per_config": 736}
        del q, out

    # full-mask mode: every rake block of every edge evaluated and kept -- its own
    # timed pass over the same (device-resident) edges, HIP events on the launch stream
    full_mask = None
    if not strong:
        cap = int(units_full_local // 8) + 64
        blk = torch.empty(cap, dtype=torch.uint8, device=dev)
        okm = torch.empty(E, dtype=torch.uint8, device=dev)

        def mask_step():
            return robot.validate_mask_device(starts.data_ptr(), goals.data_ptr(), E, env, okm.data_ptr(), 0,
                                              blk.data_ptr(), cap, ctx)

        for _ in range(max(1, a.warmup)):
            total_blocks = mask_step()
        m0, m1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        m0.record(stream)
        for _ in range(a.steps):
            mask_step()
        m1.record(stream)
        torch.cuda.synchronize(dev)
        mask_ms = m0.elapsed_time(m1) / a.steps
        full_mask = {"ms_per_step": mask_ms, "blocks": total_blocks, "interpolants": 8 * total_blocks,
                     "value": 8 * total_blocks / (mask_ms * 1e-3), "unit": "interpolants/s",
                     "edge_results_equal_early_exit": bool(torch.equal(okm, ok)),
                     "note": "vgpu_validate_motions_mask: every block of every edge evaluated (no early exit), each "
                             "block's result kept; includes its one block-count read-back"}
        del blk, okm

    # per-phase kernel time (HIP events inside the library, separate untimed pass)
    ctx.set_profiling(True)
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    phases = ctx.phase_times()
    ctx.set_profiling(False)
    calls = max(1, phases["calls"])
    head_ms = phases["head_ms"] / calls
    tail_ms = phases["tail_ms"] / calls
    scan_ms = phases["scan_ms"] / calls

    if rank == 0:
        f_head, f_tail, f_edges = algorithmic_flops(oenv, s_all, g_all, base)
        # O(n_e^2) back-step enumeration (vgpu_panda.hh rake_block: block k = k sequential subtractions):
        # its float ops per edge on the tail's items (edges valid after block 0), against the tail's
        # algorithmic work -- the cost a per-edge prefix kernel would remove
        tail_items = c_ok_head_items(c_nb, c_ne)
        backstep_ops = 56.0 * float((tail_items * (tail_items + 1) // 2).sum()) / max(1, len(c_nb))  # 7 rows x 8 lanes
        achieved = f_head * E / (head_ms * 1e-3) / 1e12
        prof_w = {("B", "000", "cage"): "validate", ("A", "000", "cage"): "validate_setA",
                  ("B", "000", "table_pick"): "validate_table_pick"}.get((a.edge_set, a.base, a.scene))
        tf = traffic_fields(prof_w, E) if prof_w and not strong else {"traffic": None, "traffic_source": None}
        cpu = None
        parity = None
        parity_failed = []
        if not a.no_cpu and world == 1:
            cpu = cpu_leg
            g_ok, g_nb = ok.cpu().numpy(), nb.cpu().numpy()
            parity = {"cpu_rake": parity_record(g_ok, g_nb, c_ok, c_nb, "mr-vamp_amd/csrc/cpu AVX2 rake, every edge"),
                      "oracle": parity_record(g_ok, g_nb, *oracle_sample(oenv, s_all, g_all, a.oracle_edges, base),
                                              "oracle/vamp_oracle.c validate_motion (scalar restatement), first "
                                              f"{a.oracle_edges} edges")}
            parity_failed = [k for k, v in parity.items() if v["mismatches"] or v["n_mismatches"]]
        ms_step = wall_max / a.steps * 1e3
        line = {
            "metric": "validated edge-interpolants/sec (Panda 7-DOF FK+CC)",
            "value": units_all * a.steps / wall_max,
            "unit": "interpolants/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded uniform Panda configurations; collision-free endpoints, edges capped at 1.0)",
            "config": {
                "workload": (f"BASELINE configs[1]: Panda 7-DOF, {E} edges per GPU (set {a.edge_set}), {scene_desc}, "
                             "validate_motion (rake 8, resolution 32, early exit)") if not strong else
                            (f"BASELINE configs[1] strong scaling: one batch of {a.edges} Panda edges split over "
                             f"{world} GPU(s); each step H2D from pinned host memory + validate + D2H of the results"),
                "robot": f"PandaBase<{base[0]},{base[1]},{base[2]}>",
                "edge_set": a.edge_set + (" (valid endpoints, length capped at 1.0)" if a.edge_set == "B" else
                                          " (raw uniform pairs)"),
                "scene": a.scene,
                "mean_n_e": float(c_nb.mean()),
                "edges_per_gpu": E,
                "interpolants_per_gpu": units_local,
                "edge_valid_fraction": ok_frac,
                "parallelism": f"dp{world} (independent edge shards, no collective)" if not strong else
                               f"dp{world} (contiguous ranges of one batch, no collective)",
            },
            "counting": "rake_early_exit: 8 x rake blocks the reference evaluates (through an edge's first invalid "
                        "block); value_full_mask_count counts 8 * n_e of every edge, evaluated or not",
            "value_full_mask_count": units_full_all * a.steps / wall_max,
            "roofline": {
                "kernel": "validate_motions step: staged bound/queue/children kernels of head and tail "
                          "(vgpu_staged.hip), one call",
                "bound": "valu",
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                **utilisation(prof_w if not strong else None, E, kern_ms, (f_head + f_tail) * E),
                **tf,
                "traffic_measured_in_run": False,
                "algorithmic_flops_per_launch": (f_head + f_tail) * E,
                "algorithmic_flops_per_edge": f_head + f_tail,
                "kernel_ms": kern_ms,
                "algorithmic_bytes_per_launch": EDGE_BYTES * E,
                "hbm_frac": EDGE_BYTES * E / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "algorithmic_flops_sample_edges": f_edges,
                "backstep_subtract_flops_per_edge": backstep_ops,
                "backstep_frac_of_tail": backstep_ops / max(f_tail, 1e-9),
                "phase_ms": {"head": head_ms, "scan_and_count": scan_ms, "tail": tail_ms},
                "phase_frac": phase_utilisation(prof_w, E, {"head": head_ms, "tail": tail_ms})
                if prof_w and not strong else None,
                "phase_reference_work_frac": {"head": achieved / FP32_PEAK_TFLOPS,
                                              "tail": f_tail * E / (max(tail_ms, 1e-9) * 1e-3) / 1e12 / FP32_PEAK_TFLOPS},
            },
            "roofline_hbm_fk": fk_leg,
            "full_mask": full_mask,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        emit(line)
        if parity_failed:
            print(f"PARITY FAILURE ({', '.join(parity_failed)}): {parity}", file=sys.stderr)
            sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
