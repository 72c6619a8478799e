"""Generate the committed golden fixtures under tests/golden/.

    python tools/make_golden.py            (build container only: needs /root/reference)

Two independent sources, neither of them this project's product code:

1. ``ref_pins.npz`` -- outputs of ``oracle/_ref/ref_probe``, compiled by oracle/Makefile
   from the reference's own vector layer and halton.hh with the reference release flags
   (sin/cos, max_extent sqrt, the validate_motion rake arithmetic, Halton<7|8>).
2. ``fk_panda.npz``, ``fkcc_panda_cage.npz``, ``edges_panda_cage.npz``,
   ``mbm_table_pick.npz`` -- the reference's generated ``robots/panda/fk.hh`` (sphere_fk and
   interleaved_sphere_fk) evaluated by ``tools/fkhh_interp.py`` (ref32 mode), with the
   collision predicates of collision/validity.hh restated in numpy.  Each mask carries the
   margins (min |test value|, min |cull difference|) used for margin-filtered parity.

Inputs are seeded numpy draws (not the reference's mt19937 stream -- the reference has no
runnable driver here); the scenes are the reference's sphere cage
(scripts/cpp/benchmark_collision_checks.cc:33-51) and MotionBenchMaker table_pick problems
(resources/panda/problems.tar.bz2).
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fkhh_interp as fi  # noqa: E402
import oracle_py as op  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
# --lut FILE (an rsqrt table saved by tools/dump_host_rsqrt.py on another host, e.g. the GPU box's
# EPYC): the same inputs, every collision output evaluated under THAT host's _mm256_rsqrt_ps cull,
# written to tests/golden/alt_rsqrt/.  A test on that host then compares against it without the
# cross-host cull-margin filter (tests/conftest.py:host_fixture).
ALT_LUT = None
ALT_DIR = os.path.join(GOLD, "alt_rsqrt")


def host_lut():
    """the rsqrt table the interpreted reference culls with: this host's, or --lut's"""
    if ALT_LUT is not None:
        return ALT_LUT
    return op.rsqrt_probe()


def out_path(name):
    if ALT_LUT is not None:
        os.makedirs(ALT_DIR, exist_ok=True)
        return os.path.join(ALT_DIR, name)
    return os.path.join(GOLD, name)
PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
F = np.float32

LO = np.array([-2.9671, -1.8326, -2.9671, -3.1416, -2.9671, -0.0873, -2.9671], F)
HI = np.array([2.9671, 1.8326, 2.9671, 0.0873, 2.9671, 3.8223, 2.9671], F)


def probe(mode, arr, *args):
    with tempfile.TemporaryDirectory() as d:
        i, o = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        np.asarray(arr, F).tofile(i)
        subprocess.check_call([PROBE, mode, i, o, *map(str, args)])
        return np.fromfile(o, F)


def make_ref_pins(rng):
    q = np.concatenate([rng.uniform(-3.3, 4.0, 65536 - 4096), np.linspace(-3.2, 3.9, 4096)]).astype(F)
    sc = probe("sincos", q)
    n = len(q)
    ext_in = np.zeros((8192, 4), F)
    ext_in[:, :3] = rng.uniform(-1.6, 1.6, (8192, 3)).astype(F)
    ext_in[:8, :3] = 0.0  # zero vector: rsqrt(0) = inf -> NaN extent
    ext_in[:, 3] = np.repeat(rng.choice(np.array([0.012, 0.06, 0.104, 0.154, 0.2], F), 1024), 8)
    ex = probe("extent", ext_in)
    # rake: random edges of all lengths + short ones
    E = 1024
    s = (LO + rng.random((E, 7), dtype=F) * (HI - LO)).astype(F)
    g = (LO + rng.random((E, 7), dtype=F) * (HI - LO)).astype(F)
    g[: E // 2] = (s[: E // 2] + (g[: E // 2] - s[: E // 2]) * F(0.15)).astype(F)
    g[:4] = s[:4]  # zero-length edges (validate(q) path)
    NB = 4
    rk = probe("rake", np.concatenate([s, g], 1), NB).reshape(E, 2 + NB * 56)
    h7 = np.concatenate([probe("halton", [0], 7, 2048, 0).reshape(-1, 7),
                         probe("halton", [0], 7, 40, 999_980).reshape(-1, 7)])
    h8 = np.concatenate([probe("halton", [0], 8, 2048, 0).reshape(-1, 8),
                         probe("halton", [0], 8, 40, 999_980).reshape(-1, 8),
                         probe("halton", [0], 8, 24, 2_000_990).reshape(-1, 8)])
    k7 = np.concatenate([np.arange(1, 2049), np.arange(999_981, 1_000_021)])
    k8 = np.concatenate([k7, np.arange(2_000_991, 2_001_015)])
    lut, kb = host_lut()
    np.savez_compressed(out_path("ref_pins.npz"), sincos_q=q, sin=sc[:n], cos=sc[n:],
                        extent_in=ext_in, extent=ex[:8192], extent_root=ex[8192:], rsqrt_lut=lut, rsqrt_kbits=kb,
                        rake_starts=s, rake_goals=g, rake_out=rk, rake_blocks=NB, halton7=h7, halton7_k=k7,
                        halton8=h8, halton8_k=k8)


def make_sql2s_pins(rng):
    """ref_probe "sql2s": the scalar float sphere_sphere_sql2 of filter_robot_from_pointcloud
    (bindings/common.hh:71-72), half the inputs within 1e-6 (relative) of contact."""
    n = 65536
    a = rng.uniform(-1, 1, (n, 8)).astype(F)
    a[:, 3] = rng.uniform(0.01, 0.3, n)
    a[:, 7] = rng.choice(np.array([0.0025, 0.01, 0.05], F), n)
    d = rng.normal(size=(n // 2, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    h = n // 2
    a[:h, 4:7] = (a[:h, 0:3] + d * (a[:h, 3:4] + a[:h, 7:8]) * (1 + rng.uniform(-1e-6, 1e-6, (h, 1)))).astype(F)
    np.savez_compressed(os.path.join(GOLD, "ref_pins_sql2s.npz"), sql2s_in=a, sql2s=probe("sql2s", a))


def make_ext_pins(rng):
    """Expression pins for the point-cloud and heightfield paths (ref_probe modes sql2,
    capt_box, hf): collision::sql2_3 compiled from the reference's math.hh, and restated
    capt.hh / sphere_heightfield.hh expressions compiled with the reference's types and flags."""
    N = 8 * 1024
    a = rng.normal(size=(N, 3)).astype(F)
    b = np.repeat(rng.normal(size=(N // 8, 3)).astype(F), 8, axis=0)
    sql2_in = np.concatenate([a, b], 1).astype(F)
    sql2 = probe("sql2", sql2_in)
    c = rng.normal(size=(N, 3)).astype(F)
    lo = (rng.normal(size=(N, 3)) * 0.5 - 0.3).astype(F)
    up = (lo + rng.random((N, 3)).astype(F)).astype(F)
    lo[:64] = -np.inf  # unbounded cells (the root volume)
    up[64:128] = np.inf
    r = (rng.random(N) * 0.06).astype(F)
    rp = np.repeat((rng.random(N // 8) * 0.01).astype(F), 8)
    box_in = np.concatenate([c, lo, up, r[:, None], rp[:, None]], 1).astype(F)
    box = probe("capt_box", box_in).reshape(4, N)
    xd, yd = 37, 29
    hdr = np.array([0.3, -0.2, 0.1, 1 / 0.05, 1 / 0.04, 1 / 0.5, xd, yd], F)
    data = rng.random(xd * yd).astype(F)
    q = np.zeros((N, 4), F)
    q[:, 0] = rng.uniform(-0.9, 0.9, N)
    q[:, 1] = rng.uniform(-0.9, 0.9, N)
    q[:, 2] = rng.uniform(0, 1, N)
    q[:, 3] = np.repeat(rng.uniform(0.01, 0.1, N // 8), 8)
    hf = probe("hf", np.concatenate([hdr, data, q.ravel()]))
    u = rng.random((4096, 7), dtype=F)
    u[:2] = [[0] * 7, [1] * 7]
    scaled = probe("scale", u).reshape(-1, 7)
    np.savez_compressed(os.path.join(GOLD, "ref_pins_ext.npz"), scale_u=u, scale_q=scaled,
                        sql2_in=sql2_in, sql2=sql2, box_in=box_in,
                        box_vec=box[0], box_rc=box[1], vol_distsq=box[2], vol_ball=box[3], hf_hdr=hdr,
                        hf_data=data, hf_q=q, hf=hf)


def sphere_cage():
    e = op.sphere_cage_env()
    return e, fi.EnvNP(spheres=e.arrays()["spheres"])


def interp_validate(cc, starts, goals, base, envnp, rs, res=32, cc_first=None, att=None):
    """validate_motion (planning/validate.hh:23-75) over E edges, 8-lane groups; with cc_first /
    att the first block goes through interleaved_sphere_fk_attachment (validate.hh:43)."""
    E, D = starts.shape
    v = (goals - starts).astype(F)
    if D <= 8:
        sq = np.zeros((E, 8), F)
        sq[:, :D] = (v * v).astype(F)
    else:  # two registers: fma(lo, lo, hi * hi) (ref_probe "l2norm")
        lo, hi = np.zeros((E, 8), F), np.zeros((E, 8), F)
        lo[:, :] = v[:, :8]
        hi[:, :D - 8] = v[:, 8:]
        sq = fi.fma32(lo, lo, (hi * hi).astype(F))
    dist = np.sqrt((((sq[:, 0] + sq[:, 4]) + (sq[:, 2] + sq[:, 6])) + ((sq[:, 1] + sq[:, 5]) + (sq[:, 3] + sq[:, 7])))
                   .astype(F)).astype(F)
    n = np.maximum(np.ceil((dist / F(8) * F(res)).astype(F)), F(1)).astype(np.int64)
    pct = (np.arange(1, 9, dtype=F) / F(8)).astype(F)
    block = fi.fma32(v[:, None, :], pct[None, :, None], starts[:, None, :])  # (E, 8, D)
    back = (v / (F(8) * n[:, None].astype(F))).astype(F)
    ok = np.ones(E, bool)
    tmarg = np.full(E, np.inf)
    cmarg = np.full(E, np.inf)
    alive = np.ones(E, bool)
    for k in range(int(n.max())):
        if k > 0:
            block = (block - back[:, None, :]).astype(F)
        idx = np.where(alive & (n > k))[0]
        if len(idx) == 0:
            break
        q = block[idx].reshape(-1, D)
        if k == 0 and cc_first is not None:
            valid, st = fi.run_fkcc(cc_first, q, base, envnp, rs, G=8, att=att)
        else:
            valid, st = fi.run_fkcc(cc, q, base, envnp, rs, G=8)
        valid = valid.reshape(-1, 8)[:, 0]
        tmarg[idx] = np.minimum(tmarg[idx], st.test_margin.reshape(-1, 8).min(1))
        cmarg[idx] = np.minimum(cmarg[idx], st.cull_margin.reshape(-1, 8).min(1))
        ok[idx] &= valid
        alive[idx] &= valid
    return ok, n, tmarg, cmarg


def mbm_scene(robot, name):
    import tarfile

    import yaml
    with tarfile.open(f"/root/reference/resources/{robot}/problems.tar.bz2") as t:
        return yaml.safe_load(t.extractfile(f"problems/{name}").read().decode())


def envnp_of(env):
    a = env.arrays()
    return fi.EnvNP(spheres=a["spheres"], capsules=a["capsules"], zcapsules=a["zcapsules"], cuboids=a["cuboids"],
                    zcuboids=a["zcuboids"])


def make_robot(rng, robot, scene, out_name, n_cfg=16384, n_empty=4096, n_edges=1024, fk_fixture=True):
    """A generated robot (fetch, ur5, baxter): FK centres, per-configuration masks and edges on
    the empty scene and one MotionBenchMaker scene, from the reference's generated
    robots/<robot>/fk.hh evaluated by tools/fkhh_interp.py."""
    src = open(f"/root/reference/src/impl/vamp/robots/{robot}/fk.hh").read()
    fk = fi.parse_function(src, r"inline void sphere_fk\(")
    cc = fi.parse_function(src, r"inline bool interleaved_sphere_fk\(")
    dim = op.ROBOTS[robot][1]
    lut, kb = host_lut()
    rs = fi.RsqrtHost(lut, kb)
    q = op.robot_scale(robot, rng.random((1024, dim), dtype=F))
    xyz, r = fi.run_sphere_fk(fk, q, (0, 0, 0))
    if fk_fixture:
        np.savez_compressed(out_path(f"fk_{robot}.npz"), q=q, radii=r.astype(F),
                            xyz=np.ascontiguousarray(np.transpose(xyz, (2, 1, 0))))
        print(f"fk_{robot}.npz")
    env = op.mbm_env(mbm_scene(robot, scene))
    arr = env.arrays()
    envnp = envnp_of(env)
    empty = fi.EnvNP(spheres=np.zeros((0, 5), F))
    q = op.robot_scale(robot, rng.random((n_cfg, dim), dtype=F))
    valid, st = fi.run_fkcc(cc, q, (0, 0, 0), envnp, rs, G=1)
    qe = op.robot_scale(robot, rng.random((n_empty, dim), dtype=F))
    valid_e, st_e = fi.run_fkcc(cc, qe, (0, 0, 0), empty, rs, G=1)
    # edges: raw pairs (short) and valid-endpoint pairs capped at length 1.0
    E = n_edges
    s = op.robot_scale(robot, rng.random((E, dim), dtype=F))
    g = op.robot_scale(robot, rng.random((E, dim), dtype=F))
    g = (s + (g - s) * F(0.25)).astype(F)
    vq = q[valid]
    sb, gb = vq[0:2 * E:2][:E], vq[1:2 * E:2][:E]
    d = np.linalg.norm((gb - sb).astype(np.float64), axis=1)
    sc = np.minimum(1.0, 1.0 / np.maximum(d, 1e-9)).astype(F)
    gb = (sb + (gb - sb) * sc[:, None]).astype(F)
    starts = np.concatenate([s, sb])
    goals = np.concatenate([g, gb])
    starts[:4] = goals[:4]
    ok, n, tm, cm = interp_validate(cc, starts, goals, (0, 0, 0), envnp, rs, op.RESOLUTION[robot])
    np.savez_compressed(out_path(out_name), rsqrt_lut=lut, rsqrt_kbits=kb,
                        **{"env_" + k: v for k, v in arr.items()},
                        q=q, valid=valid, test_margin=st.test_margin.astype(F), cull_margin=st.cull_margin.astype(F),
                        q_empty=qe, valid_empty=valid_e, test_margin_empty=st_e.test_margin.astype(F),
                        starts=starts, goals=goals, ok=ok, n=n.astype(np.int32), edge_test_margin=tm.astype(F),
                        edge_cull_margin=cm.astype(F))
    print(out_name, valid.mean(), valid_e.mean(), ok[:E].mean(), ok[E:].mean(), n.max())


def mbm_request(robot, name, dim):
    """start / goal joint positions of a MotionBenchMaker request (request*.yaml): the first `dim`
    joints of start_state, the goal_constraints' joint positions in joint order"""
    import tarfile

    import yaml
    with tarfile.open(f"/root/reference/resources/{robot}/problems.tar.bz2") as t:
        rq = yaml.safe_load(t.extractfile(f"problems/{name}").read().decode())
    start = np.array(rq["start_state"]["joint_state"]["position"][:dim], F)
    goal = np.array([c["position"] for c in rq["goal_constraints"][0]["joint_constraints"]][:dim], F)
    return start, goal


def make_panda_mbm(rng, n_problems=16):
    """Panda on MotionBenchMaker table_pick (the configs[0] planning problem and the configs[1] MBM
    run): masks / edges on scene0001 from the reference DAG (make_robot), plus the
    first `n_problems` problems' resolved scenes, start / goal and the reference-DAG result of the
    straight start -> goal validate_motion (base (0,0,0): the scenes are origin-centred)."""
    make_robot(rng, "panda", "table_pick_panda/scene0001.yaml", "panda_table_pick.npz", fk_fixture=False)
    fk, cc = fi.load_panda()
    lut, kb = host_lut()
    rs = fi.RsqrtHost(lut, kb)
    out = {"rsqrt_lut": lut, "rsqrt_kbits": kb}
    for k in range(1, n_problems + 1):
        env = op.mbm_env(mbm_scene("panda", f"table_pick_panda/scene{k:04d}.yaml"))
        start, goal = mbm_request("panda", f"table_pick_panda/request{k:04d}.yaml", 7)
        ok, n, tm, cm = interp_validate(cc, start[None], goal[None], (0, 0, 0), envnp_of(env), rs)
        for key, v in env.arrays().items():
            out[f"p{k}_env_{key}"] = v
        out.update({f"p{k}_start": start, f"p{k}_goal": goal, f"p{k}_ok": ok, f"p{k}_n": n.astype(np.int32),
                    f"p{k}_test_margin": tm.astype(F), f"p{k}_cull_margin": cm.astype(F)})
    np.savez_compressed(out_path("panda_table_pick_problems.npz"), n_problems=np.int32(n_problems), **out)
    print("panda_table_pick_problems.npz", [bool(out[f"p{k}_ok"][0]) for k in range(1, n_problems + 1)])


def make_eefk(rng, n=1024):
    """Robot::eefk fixtures: the reference's generated eefk (robots/<robot>/fk.hh) evaluated in
    double by tools/eefk_ref.py at uniform configurations, Panda / Fetch / UR5."""
    import eefk_ref
    out = {}
    for robot in ("panda", "fetch", "ur5"):
        dim, run = eefk_ref.make_eval(robot)
        q = op.robot_scale(robot, rng.random((n, dim), dtype=F))
        out[f"{robot}_q"] = q
        out[f"{robot}_pose"] = run(q)
    np.savez_compressed(out_path("eefk.npz"), **out)
    print("eefk.npz")


def make_fetch(rng):
    make_robot(rng, "fetch", "table_pick_fetch/scene0001.yaml", "fetch_table_pick.npz")


def make_attach(rng):
    """Panda with a held object (tests/oracle_py.py:held_object) on the sphere cage, bases (0,0,0)
    and (200,200,0): per-configuration fkcc_attach masks (interleaved_sphere_fk_attachment) and
    edges whose first block goes through it (validate.hh:43)."""
    src = open("/root/reference/src/impl/vamp/robots/panda/fk.hh").read()
    cc = fi.parse_function(src, r"inline bool interleaved_sphere_fk\(")
    ca = fi.parse_function(src, r"inline bool interleaved_sphere_fk_attachment\(")
    lut, kb = host_lut()
    rs = fi.RsqrtHost(lut, kb)
    env, envnp = sphere_cage()
    att = op.held_object()
    ad = att.as_dict()
    out = {}
    for tag, base in (("b000", (0, 0, 0)), ("b220", (200, 200, 0))):
        q = op.scale(rng.random((8192, 7), dtype=F))
        valid, st = fi.run_fkcc(ca, q, base, envnp, rs, G=1, att=ad)
        plain, _ = fi.run_fkcc(cc, q, base, envnp, rs, G=1)
        out.update({f"q_{tag}": q, f"valid_{tag}": valid, f"plain_{tag}": plain,
                    f"test_margin_{tag}": st.test_margin.astype(F), f"cull_margin_{tag}": st.cull_margin.astype(F)})
    E = 1024
    pool = op.scale(rng.random((20000, 7), dtype=F))
    pv = op.fkcc_threads(env, pool, (0, 0, 0))
    vq = pool[pv]
    s, g = vq[0:2 * E:2][:E], vq[1:2 * E:2][:E]
    d = np.linalg.norm((g - s).astype(np.float64), axis=1)
    g = (s + (g - s) * np.minimum(1.0, 1.0 / np.maximum(d, 1e-9)).astype(F)[:, None]).astype(F)
    ok, n, tm, cm = interp_validate(cc, s, g, (0, 0, 0), envnp, rs, 32, cc_first=ca, att=ad)
    np.savez_compressed(out_path("attach_panda_cage.npz"), rsqrt_lut=lut, rsqrt_kbits=kb,
                        att_tf=ad["tf"], att_spheres=ad["spheres"], starts=s, goals=g, ok=ok, n=n.astype(np.int32),
                        edge_test_margin=tm.astype(F), edge_cull_margin=cm.astype(F), **out)
    print("attach_panda_cage.npz", out["valid_b000"].mean(), out["plain_b000"].mean(), out["valid_b220"].mean(),
          ok.mean())


def make_attach_robot(rng, robot, scene, n_cfg=8192, n_edges=1024):
    """Fetch / UR5 with the held object on one MotionBenchMaker scene: per-configuration
    fkcc_attach masks (the robot's interleaved_sphere_fk_attachment) next to plain fkcc, and
    valid-endpoint edges capped at 1.0 whose first block goes through it (validate.hh:43)."""
    src = open(f"/root/reference/src/impl/vamp/robots/{robot}/fk.hh").read()
    cc = fi.parse_function(src, r"inline bool interleaved_sphere_fk\(")
    ca = fi.parse_function(src, r"inline bool interleaved_sphere_fk_attachment\(")
    dim = op.ROBOTS[robot][1]
    lut, kb = host_lut()
    rs = fi.RsqrtHost(lut, kb)
    env = op.mbm_env(mbm_scene(robot, scene))
    envnp = envnp_of(env)
    ad = op.held_object().as_dict()
    q = op.robot_scale(robot, rng.random((n_cfg, dim), dtype=F))
    valid, st = fi.run_fkcc(ca, q, (0, 0, 0), envnp, rs, G=1, att=ad)
    plain, _ = fi.run_fkcc(cc, q, (0, 0, 0), envnp, rs, G=1)
    pool = op.robot_scale(robot, rng.random((8 * n_edges, dim), dtype=F))
    pv = op.robot_fkcc_threads(robot, env, pool)
    vq = pool[pv]
    E = min(n_edges, len(vq) // 2)
    s, g = vq[0:2 * E:2], vq[1:2 * E:2]
    d = np.linalg.norm((g - s).astype(np.float64), axis=1)
    g = (s + (g - s) * np.minimum(1.0, 1.0 / np.maximum(d, 1e-9)).astype(F)[:, None]).astype(F)
    ok, n, tm, cm = interp_validate(cc, s, g, (0, 0, 0), envnp, rs, op.RESOLUTION[robot], cc_first=ca, att=ad)
    arr = env.arrays()
    np.savez_compressed(out_path(f"attach_{robot}.npz"), rsqrt_lut=lut, rsqrt_kbits=kb,
                        att_tf=ad["tf"], att_spheres=ad["spheres"], q=q, valid=valid, plain=plain,
                        test_margin=st.test_margin.astype(F), cull_margin=st.cull_margin.astype(F), starts=s, goals=g,
                        ok=ok, n=n.astype(np.int32), edge_test_margin=tm.astype(F), edge_cull_margin=cm.astype(F),
                        **{"env_" + k: v for k, v in arr.items()})
    print(f"attach_{robot}.npz", valid.mean(), plain.mean(), ok.mean())


def make_l2_pins(rng):
    """FloatVector<dim>::l2_norm for dim 7, 8 and 14 (ref_probe "l2norm"): the 14-lane form is
    two registers contracted as fma(lo, lo, hi * hi) before the hsum."""
    out = {}
    for dim in (7, 8, 14):
        v = (rng.normal(size=(4096, dim)) * rng.choice([1e-3, 1.0, 30.0], size=(4096, 1))).astype(F)
        out[f"v{dim}"] = v
        out[f"d{dim}"] = probe("l2norm", v, dim)
    np.savez_compressed(out_path("ref_pins_l2.npz"), **out)


def pair_inter_flat(xa, xb):
    """min over the 59 x 59 sphere pairs of arm A vs arm B of sphere_sphere_sql2 (dot_3
    contracted as fma(x, x, fma(z, z, y*y)), sphere_sphere.hh:10-22), per configuration."""
    _, rad = None, None
    r = np.asarray(RADII_PANDA, F)
    dx = (xa[0][:, :, None] - xb[0][:, None, :]).astype(F)
    dy = (xa[1][:, :, None] - xb[1][:, None, :]).astype(F)
    dz = (xa[2][:, :, None] - xb[2][:, None, :]).astype(F)
    rs = (r[:, None] + r[None, :]).astype(F)
    d2 = fi.fma32(dx, dx, fi.fma32(dz, dz, (dy * dy).astype(F)))
    val = fi.fma32(-rs, rs, d2)
    return val.reshape(val.shape[0], -1)


RADII_PANDA = None


def make_pair(rng):
    """Two-Panda composite (BASELINE configs[4]): per-arm masks from the reference DAG
    (fk.hh interleaved_sphere_fk at bases (0,0,0) and (100,0,0)) and the flat 59 x 59 inter-arm
    sphere test on the DAG's sphere_fk centres, for configurations and for 14-dof edges (rake
    over the pinned two-register l2_norm).  There is no reference composite: this fixes the
    composition (AND of the three) independently of the C restatement's bounding-first order."""
    global RADII_PANDA
    fk, cc = fi.load_panda()
    lut, kb = host_lut()
    rs = fi.RsqrtHost(lut, kb)
    env = op.pair_scene()
    envnp = envnp_of(env)
    N = 8192
    u = rng.random((N, 14), dtype=F)
    q = np.concatenate([op.scale(u[:, :7]), op.scale(u[:, 7:])], 1)
    va, sta = fi.run_fkcc(cc, q[:, :7], (0, 0, 0), envnp, rs, G=1)
    vb, stb = fi.run_fkcc(cc, q[:, 7:], (100, 0, 0), envnp, rs, G=1)
    xa, RADII_PANDA = fi.run_sphere_fk(fk, q[:, :7], (0, 0, 0))
    xb, _ = fi.run_sphere_fk(fk, q[:, 7:], (100, 0, 0))
    inter = pair_inter_flat([xa[i].T for i in range(3)], [xb[i].T for i in range(3)])
    hit = (inter.view(np.uint32) >> 31).astype(bool).any(1)
    imarg = np.abs(inter).min(1)
    valid = va & vb & ~hit
    tm = np.minimum(sta.test_margin, stb.test_margin)
    cm = np.minimum(sta.cull_margin, stb.cull_margin)
    # edges between valid composite configurations, each arm's sub-edge capped at 1.0
    E = 1024
    vq = q[valid]
    s, g = vq[0:2 * E:2][:E].copy(), vq[1:2 * E:2][:E].copy()
    for a in (slice(0, 7), slice(7, 14)):
        d = np.linalg.norm((g[:, a] - s[:, a]).astype(np.float64), axis=1)
        sc = np.minimum(1.0, 1.0 / np.maximum(d, 1e-9)).astype(F)
        g[:, a] = (s[:, a] + (g[:, a] - s[:, a]) * sc[:, None]).astype(F)
    ok, n, etm = pair_interp_validate(fk, cc, s, g, envnp, rs)
    np.savez_compressed(out_path("pair_scene.npz"), rsqrt_lut=lut, rsqrt_kbits=kb,
                        **{"env_" + k: v for k, v in env.arrays().items()}, q=q, valid=valid,
                        valid_a=va, valid_b=vb, inter_hit=hit, inter_margin=imarg.astype(F), test_margin=tm.astype(F), cull_margin=cm.astype(F),
                        starts=s, goals=g, ok=ok, n=n.astype(np.int32), edge_test_margin=etm[0].astype(F),
                        edge_inter_margin=etm[1].astype(F))
    print("pair_scene.npz", valid.mean(), hit.mean(), ok.mean(), n.max())


def pair_interp_validate(fk, cc, starts, goals, envnp, rs):
    E, D = starts.shape
    v = (goals - starts).astype(F)
    lo, hi = np.zeros((E, 8), F), np.zeros((E, 8), F)
    lo[:, :8] = v[:, :8]
    hi[:, :D - 8] = v[:, 8:]
    sq = fi.fma32(lo, lo, (hi * hi).astype(F))
    dist = np.sqrt((((sq[:, 0] + sq[:, 4]) + (sq[:, 2] + sq[:, 6])) + ((sq[:, 1] + sq[:, 5]) + (sq[:, 3] + sq[:, 7])))
                   .astype(F)).astype(F)
    n = np.maximum(np.ceil((dist / F(8) * F(32)).astype(F)), F(1)).astype(np.int64)
    pct = (np.arange(1, 9, dtype=F) / F(8)).astype(F)
    block = fi.fma32(v[:, None, :], pct[None, :, None], starts[:, None, :])
    back = (v / (F(8) * n[:, None].astype(F))).astype(F)
    ok = np.ones(E, bool)
    alive = np.ones(E, bool)
    tmarg = np.full(E, np.inf)
    imarg = np.full(E, np.inf)
    for k in range(int(n.max())):
        if k > 0:
            block = (block - back[:, None, :]).astype(F)
        idx = np.where(alive & (n > k))[0]
        if len(idx) == 0:
            break
        q = block[idx].reshape(-1, 14)
        va, sa = fi.run_fkcc(cc, q[:, :7], (0, 0, 0), envnp, rs, G=8)
        vb, sb = fi.run_fkcc(cc, q[:, 7:], (100, 0, 0), envnp, rs, G=8)
        xa, _ = fi.run_sphere_fk(fk, q[:, :7], (0, 0, 0))
        xb, _ = fi.run_sphere_fk(fk, q[:, 7:], (100, 0, 0))
        inter = pair_inter_flat([xa[i].T for i in range(3)], [xb[i].T for i in range(3)])
        hit = (inter.view(np.uint32) >> 31).astype(bool).any(1).reshape(-1, 8).any(1)
        valid = va.reshape(-1, 8)[:, 0] & vb.reshape(-1, 8)[:, 0] & ~hit
        m = np.minimum(sa.test_margin, sb.test_margin).reshape(-1, 8).min(1)
        tmarg[idx] = np.minimum(tmarg[idx], m)
        imarg[idx] = np.minimum(imarg[idx], np.abs(inter).min(1).reshape(-1, 8).min(1))
        ok[idx] &= valid
        alive[idx] &= valid
    return ok, n, (tmarg, imarg)


def main():
    global ALT_LUT
    os.makedirs(GOLD, exist_ok=True)
    if "--lut" in sys.argv:
        z = np.load(sys.argv[sys.argv.index("--lut") + 1], allow_pickle=False)
        ALT_LUT = (z["rsqrt_lut"].astype(np.uint32), int(z["rsqrt_kbits"]))
    if "--pair" in sys.argv:
        make_l2_pins(np.random.default_rng(20261017))
        make_pair(np.random.default_rng(20261018))
        return
    if "--fetch" in sys.argv:
        make_fetch(np.random.default_rng(20261016))
        return
    if "--eefk" in sys.argv:
        make_eefk(np.random.default_rng(20261025))
        return
    if "--panda-mbm" in sys.argv:
        make_panda_mbm(np.random.default_rng(20261024))
        return
    if "--attach-fetch" in sys.argv:
        make_attach_robot(np.random.default_rng(20261022), "fetch", "table_pick_fetch/scene0001.yaml")
        return
    if "--sql2s" in sys.argv:
        make_sql2s_pins(np.random.default_rng(20261101))
        print("ref_pins_sql2s.npz")
        return
    if "--attach-ur5" in sys.argv:
        make_attach_robot(np.random.default_rng(20261023), "ur5", "table_pick_ur5/scene0001.yaml")
        return
    if "--attach" in sys.argv:
        make_attach(np.random.default_rng(20261021))
        return
    if "--ur5" in sys.argv:
        make_robot(np.random.default_rng(20261019), "ur5", "table_pick_ur5/scene0001.yaml", "ur5_table_pick.npz")
        return
    if "--baxter" in sys.argv:
        make_robot(np.random.default_rng(20261020), "baxter", "bookshelf_tall_both_arms_easy_baxter/scene0001.yaml",
                   "baxter_bookshelf.npz", n_cfg=8192, n_empty=2048, n_edges=512)
        return
    if not os.path.exists(PROBE):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    rng = np.random.default_rng(20251015)
    make_ref_pins(rng)  # (under --lut only for its rng draws: the pins are this host's probe)
    if ALT_LUT is not None:
        os.remove(out_path("ref_pins.npz"))
    else:
        print("ref_pins.npz")
        make_ext_pins(np.random.default_rng(20261015))
        print("ref_pins_ext.npz")

    fk, cc = fi.load_panda()
    lut, kb = host_lut()
    rs = fi.RsqrtHost(lut, kb)

    # ---- FK sphere centres at both bases
    q = op.scale(rng.random((1024, 7), dtype=F))
    out = {}
    for tag, base in (("b000", (0, 0, 0)), ("b220", (200, 200, 0)), ("b105", (100, -50, 5))):
        xyz, r = fi.run_sphere_fk(fk, q, base)
        out[tag] = np.ascontiguousarray(np.transpose(xyz, (2, 1, 0)))
    if ALT_LUT is None:  # FK does not cull: nothing host-dependent
        np.savez_compressed(out_path("fk_panda.npz"), q=q, radii=r.astype(F), **out)
        print("fk_panda.npz")

    # ---- per-configuration masks (G = 1) on the sphere cage
    env, envnp = sphere_cage()
    q = op.scale(rng.random((32768, 7), dtype=F))
    valid, st = fi.run_fkcc(cc, q, (0, 0, 0), envnp, rs, G=1)
    q2 = op.scale(rng.random((8192, 7), dtype=F))
    valid2, st2 = fi.run_fkcc(cc, q2, (200, 200, 0), envnp, rs, G=1)
    np.savez_compressed(out_path("fkcc_panda_cage.npz"), env_spheres=env.arrays()["spheres"], q=q,
                        valid=valid, test_margin=st.test_margin.astype(F), cull_margin=st.cull_margin.astype(F),
                        q_b220=q2, valid_b220=valid2, test_margin_b220=st2.test_margin.astype(F),
                        cull_margin_b220=st2.cull_margin.astype(F), rsqrt_lut=lut, rsqrt_kbits=kb)
    print("fkcc_panda_cage.npz", valid.mean(), valid2.mean())

    # ---- edges: raw pairs and valid-endpoint pairs capped at length 1.0
    E = 4096
    s = op.scale(rng.random((E, 7), dtype=F))
    g = op.scale(rng.random((E, 7), dtype=F))
    pool = op.scale(rng.random((40000, 7), dtype=F))
    pv = op.fkcc_threads(env, pool, (0, 0, 0))
    vq = pool[pv]
    sb, gb = vq[0:2 * E:2][:E], vq[1:2 * E:2][:E]
    d = np.linalg.norm((gb - sb).astype(np.float64), axis=1)
    scale = np.minimum(1.0, 1.0 / np.maximum(d, 1e-9)).astype(F)
    gb = (sb + (gb - sb) * scale[:, None]).astype(F)
    starts = np.concatenate([s, sb])
    goals = np.concatenate([g, gb])
    starts[:8] = goals[:8]  # zero-length edges
    ok, n, tm, cm = interp_validate(cc, starts, goals, (0, 0, 0), envnp, rs)
    np.savez_compressed(out_path("edges_panda_cage.npz"), starts=starts, goals=goals, ok=ok,
                        n=n.astype(np.int32), test_margin=tm.astype(F), cull_margin=cm.astype(F),
                        **({"rsqrt_lut": lut, "rsqrt_kbits": kb} if ALT_LUT is not None else {}))
    print("edges_panda_cage.npz", ok[:E].mean(), ok[E:].mean(), n.max())


if __name__ == "__main__":
    main()
