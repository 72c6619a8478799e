"""GPU parity on grazing contacts: capsules, z-capsules, cuboids and z-cuboids placed so that one robot sphere
touches them to within a few parts per million of its radius -- face contacts and the tight corners of the
obstacles' bounding spheres (a cuboid corner on the box diagonal, a capsule end on its axis) -- then configs
jittered around that pose.  Every obstacle record the device scans carries a bounding sphere, and a wave skips
a record none of its lanes' spheres reach (vgpu_device.hh scan_type, vgpu_api.cpp obstacle_bound); the skip
must never drop a record whose test (sphere_capsule.hh:9-43, sphere_cuboid.hh:9-52) would fire, so the
per-config masks and motion results equal the oracle's bit for bit -- right at the threshold too.
"""
import json
import os

import numpy as np
import pytest

from test_gpu_parity import gpu_env_from_oracle

pytestmark = pytest.mark.gpu
F = np.float32
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def robot_of(vamp, robot):
    return vamp.panda_0_0 if robot == "panda" else getattr(vamp, robot)


def radii(robot):
    m = json.load(open(os.path.join(ROOT, "model", f"{robot}.json")))
    return np.array([s["radius"] for s in m["spheres"]], np.float64)


def rotation(rng):
    q = rng.normal(size=4)
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def unit(v):
    return v / np.linalg.norm(v)


def obstacle(rng, p, r):
    """a random obstacle touching the sphere (p, r): add(env, gap) places it at distance `gap` from p"""
    kind = rng.integers(6)
    if kind in (0, 1):  # cuboid (0: face contact, 1: corner on the diagonal); z-cuboid with prob. 1/2
        if rng.random() < 0.5:
            a = rng.uniform(0, 2 * np.pi)
            R = np.array([[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]])
        else:
            R = rotation(rng)
        h = rng.uniform(0.02, 0.3, 3)
        if kind == 0:
            k, sgn = rng.integers(3), rng.choice([-1.0, 1.0])
            return lambda env, gap: env.add_cuboid_axes(p + R[:, k] * (h[k] + gap) * sgn, R[:, 0], R[:, 1], R[:, 2], h)
        d = R @ (h * rng.choice([-1.0, 1.0], 3))
        return lambda env, gap: env.add_cuboid_axes(p - unit(d) * (np.linalg.norm(d) + gap), R[:, 0], R[:, 1],
                                                    R[:, 2], h)
    if kind in (2, 3):  # capsule (2: side contact, 3: end cap on the axis); vertical with prob. 1/2
        rc, L = rng.uniform(0.01, 0.1), rng.uniform(0.05, 0.5)
        t = np.array([0.0, 0.0, 1.0]) if rng.random() < 0.5 else unit(rng.normal(size=3))
        if kind == 2:
            n, f = unit(np.cross(t, rng.normal(size=3))), rng.uniform(0.1, 0.9)
            return lambda env, gap: env.add_capsule_endpoints(p + n * (gap + rc) - t * L * f,
                                                              p + n * (gap + rc) + t * L * (1 - f), rc)
        sgn = rng.choice([-1.0, 1.0])
        return lambda env, gap: env.add_capsule_endpoints(p + sgn * t * (gap + rc), p + sgn * t * (gap + rc + L), rc)
    if kind == 4:  # a sheared box (non-orthonormal axes: never skipped) in face contact
        a1 = unit(rng.normal(size=3))
        a2 = unit(a1 + rng.normal(size=3))
        a3 = unit(np.cross(a1, a2))
        h = rng.uniform(0.02, 0.2, 3)
        return lambda env, gap: env.add_cuboid_axes(p + a3 * (h[2] + gap), a1, a2, a3, h)
    n = unit(rng.normal(size=3))  # a sphere in contact
    return lambda env, gap: env.add_sphere(p + n * (gap + 0.05), 0.05)


def grazing_env(oracle, robot, rng, q0, rads, n_obs=3, tries=200):
    """up to n_obs obstacles, each touching one robot sphere of q0 at distance r * (1 + d), |d| <= 4e-6, and
    clear of every other sphere (checked on the oracle with the obstacle 1e-3 r further out)"""
    centres = oracle.robot_sphere_fk(robot, q0[None])[0].astype(np.float64)
    env, safe, n = oracle.Env(), oracle.Env(), 0
    for _ in range(tries):
        i = rng.integers(len(rads))
        add = obstacle(rng, centres[i], rads[i])
        trial = oracle.Env()
        for kind in ("spheres", "capsules", "zcapsules", "cuboids", "zcuboids"):
            getattr(trial, kind).extend(getattr(safe, kind))
        add(trial, rads[i] * 1.001)
        if not oracle.robot_fkcc_threads(robot, trial, q0[None])[0]:
            continue
        add(safe, rads[i] * 1.001)
        add(env, rads[i] * (1.0 + rng.uniform(-4e-6, 4e-6)))
        n += 1
        if n == n_obs:
            break
    return env, n


@pytest.mark.parametrize("robot", ["panda", "fetch"])
def test_grazing_obstacles_fkcc_and_motions(vamp, oracle, robot):
    rng = np.random.default_rng(2024)
    rob = robot_of(vamp, robot)
    rads = radii(robot)
    dim = oracle.ROBOTS[robot][1]
    u = rng.random((4000, dim), dtype=F)
    q_all = oracle.robot_scale(robot, u)
    free = oracle.robot_fkcc_threads(robot, oracle.Env(), q_all)
    q_free = q_all[free]
    mixed = 0
    for trial in range(20):
        q0 = q_free[trial]
        oenv, n_obs = grazing_env(oracle, robot, rng, q0, rads)
        assert n_obs == 3
        env = gpu_env_from_oracle(vamp, oenv)
        # jitter of ~1e-6 rad moves the spheres by ~1e-6 m: on both sides of the contacts
        q = (q0[None] + rng.normal(scale=2e-6, size=(1024, dim))).astype(F)
        q[0] = q0
        got = rob.fkcc_batch(q, env)
        want = oracle.robot_fkcc_threads(robot, oenv, q)
        assert np.array_equal(got, want), f"{robot} trial {trial}: {np.flatnonzero(got != want)[:10]}"
        mixed += 0 < want.sum() < len(want)
        s = q[:256]
        g = (q[256:512] + rng.normal(scale=1e-3, size=(256, dim))).astype(F)
        ok, n = rob.validate_batch(s, g, env)
        rok, rn = oracle.robot_validate_motions(robot, oenv, s, g)
        assert np.array_equal(n, rn) and np.array_equal(ok, rok), f"{robot} trial {trial} motions"
    assert mixed >= 10  # the jitter straddles the contacts in several scenes
