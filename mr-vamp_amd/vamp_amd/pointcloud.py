"""MotionBenchMaker point-cloud harness: the mirror of the reference's ``vamp.pointcloud``
(src/vamp/pointcloud.py:1-167) over this package.

A problem's boxes and cylinders are sampled on their surfaces (numpy, ``np.random.seed(0)``, the
same draws in the same order as the reference's samplers, which it takes from geometrout), the
cloud is filtered on the GPU (``filter_pointcloud``, collision/filter.hh:175-268) with the robot's
first-joint origin and reach (constants.py:57-77), and a CAPT is built from the kept points
(``Environment.add_pointcloud``, environment.cc:148-158).  ``problem_dict_to_pointcloud`` returns
what the reference's returns: (env, original_pc, filtered_pc, filter_time, build_time).

MotionBenchMaker scenes come as ``scene*.yaml`` (resources/<robot>/problems.tar.bz2); the
reference's evaluation script reads them from a pickled dict whose objects carry ``position``,
``orientation_quat_xyzw`` and ``half_extents`` (boxes) or ``radius`` / ``length`` (cylinders);
``scene_to_problem_dict`` builds that dict from a parsed scene (no pickle involved).

Parity: the sampled points follow pointcloud.py's float64 arithmetic op for op (quaternion matrix,
homogeneous transform); no reference outputs exist here to pin them against (the reference package
needs its compiled extension to import), so the sampler is parity-unpinned and tested by its
properties (tests/test_pointcloud.py); the filter and the CAPT build downstream are pinned.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional

import numpy as np

# constants.py:57-77
ROBOT_RADII_RANGES = {"baxter": (0.012, 0.08), "fetch": (0.012, 0.055), "panda": (0.012, 0.06),
                      "sphere": (0.2, 0.2), "ur5": (0.015, 0.08)}
ROBOT_FIRST_JOINT_LOCATIONS = {"fetch": [0.0, 0.0, 0.4], "ur5": [0.0, 0.0, 0.91], "panda": [0.0, 0.0, 0.0]}
ROBOT_MAX_RADII = {"ur5": 1.2, "fetch": 1.5, "panda": 1.19}
POINT_RADIUS = 0.0025


# ---- poses (transformations.py:194-205, 1173-1194, 1671-1687) -----------------------------------
def pose_matrix(position, quat_xyzw) -> np.ndarray:
    """4x4 homogeneous pose: translation(position) . rotation(quaternion x y z w), float64."""
    q = np.array(quat_xyzw[:4], dtype=np.float64, copy=True)
    nq = float(np.dot(q, q))
    R = np.identity(4)
    if nq >= np.finfo(float).eps * 4.0:
        q *= math.sqrt(2.0 / nq)
        o = np.outer(q, q)
        R = np.array(((1.0 - o[1, 1] - o[2, 2], o[0, 1] - o[2, 3], o[0, 2] + o[1, 3], 0.0),
                      (o[0, 1] + o[2, 3], 1.0 - o[0, 0] - o[2, 2], o[1, 2] - o[0, 3], 0.0),
                      (o[0, 2] - o[1, 3], o[1, 2] + o[0, 3], 1.0 - o[0, 0] - o[1, 1], 0.0),
                      (0.0, 0.0, 0.0, 1.0)), dtype=np.float64)
    T = np.identity(4)
    T[:3, 3] = np.asarray(position, np.float64)[:3]
    return np.dot(T, R)


def _apply_pose(points: np.ndarray, M: np.ndarray) -> np.ndarray:
    """points (n x 3, float64) mapped by M through homogeneous coordinates, in place."""
    h = np.concatenate((points.T, np.ones((1, points.shape[0]))), axis=0)
    points[:, :3] = np.dot(M, h)[:3, :].T
    return points


def _jitter(points: np.ndarray, noise: float) -> np.ndarray:
    # the reference draws the noise array even when noise == 0 (it then adds zeros)
    return points + (2 * noise * np.random.random_sample(points.shape) - noise)


# ---- surface samplers (pointcloud.py:29-108) ------------------------------------------------------
def sphere_sample_surface(center, radius: float, num_points: int, noise: float) -> np.ndarray:
    p = np.random.uniform(-1.0, 1.0, (num_points, 3))
    p /= np.linalg.norm(p, axis=1)[:, None]
    p = radius * p + center
    if noise > 0.0:
        return p + np.random.uniform(-noise, noise, p.shape)
    return p


def cylinder_sample_surface(pose: np.ndarray, radius: float, height: float, num_points: int,
                            noise: float) -> np.ndarray:
    """Bottom cap / side / top cap chosen with probability proportional to their areas."""
    ang = np.random.uniform(-np.pi, np.pi, num_points)
    xy = np.stack((np.cos(ang), np.sin(ang)), axis=1)
    cap = np.pi * radius ** 2
    side = height * 2 * np.pi * radius
    area = side + 2 * np.pi * radius ** 2
    surf = np.searchsorted(np.cumsum(np.array([cap / area, side / area, cap / area])),
                           np.random.random(num_points), side="right")
    bottom, lateral, top = surf == 0, surf == 1, surf == 2
    xy[bottom] *= np.random.uniform(0, radius, size=(np.count_nonzero(bottom), 1))
    xy[lateral] *= radius
    xy[top] *= np.random.uniform(0, radius, size=(np.count_nonzero(top), 1))
    z = np.ones((num_points, 1))
    z[bottom] = -height / 2
    z[lateral] = np.random.uniform(-height / 2, height / 2, size=(np.count_nonzero(lateral), 1))
    z[top] = height / 2
    pts = _apply_pose(np.concatenate((xy, z), axis=1), pose)
    return _jitter(pts, noise)


def cuboid_sample_surface(pose: np.ndarray, dims, num_points: int, noise: float) -> np.ndarray:
    """A face chosen with probability proportional to its area (+x, -x, +y, -y, +z, -z), the point
    projected onto it."""
    dims = np.asarray(dims, np.float64)
    pts = np.random.uniform(-1.0, 1.0, (num_points, 3)) * dims / 2
    face_area = np.array([dims[1] * dims[2]] * 2 + [dims[0] * dims[2]] * 2 + [dims[0] * dims[1]] * 2)
    face_area /= np.sum(face_area)
    face = np.searchsorted(np.cumsum(face_area), np.random.random(num_points), side="right")
    for f in range(6):
        axis, sign = f // 2, (1.0 if f % 2 == 0 else -1.0)
        pts[face == f, axis] = sign * dims[axis] / 2
    pts = _apply_pose(pts, pose)
    return _jitter(pts, noise)


def box_to_pc(box: dict, n: int) -> np.ndarray:
    return cuboid_sample_surface(pose_matrix(box["position"], box["orientation_quat_xyzw"]),
                                 np.array(box["half_extents"]) * 2, n, 0)


def cylinder_to_pc(cyl: dict, n: int) -> np.ndarray:
    return cylinder_sample_surface(pose_matrix(cyl["position"], cyl["orientation_quat_xyzw"]), cyl["radius"],
                                   cyl["length"], n, 0)


def problem_to_pointcloud(problem: dict, n: int) -> np.ndarray:
    """n surface samples per object, cylinders first, then boxes (pointcloud.py:122-126)."""
    np.random.seed(0)
    return np.vstack([cylinder_to_pc(c, n) for c in problem.get("cylinder", [])] +
                     [box_to_pc(b, n) for b in problem.get("box", [])])


# ---- MotionBenchMaker scene -> problem dict ------------------------------------------------------
def scene_to_problem_dict(scene: dict, name: str = "") -> Dict[str, List[dict]]:
    """A parsed MotionBenchMaker ``scene*.yaml`` as the reference's problem dict: every box and
    cylinder primitive with its pose (MBM stores orientations as x y z w)."""
    out = {"problem": name, "box": [], "cylinder": [], "sphere": []}
    for obj in scene["world"]["collision_objects"]:
        for k, (prim, pose) in enumerate(zip(obj["primitives"], obj["primitive_poses"])):
            d = {"name": f"{obj.get('id', 'object')}_{k}", "position": list(map(float, pose["position"])),
                 "orientation_quat_xyzw": list(map(float, pose["orientation"]))}
            if prim["type"] == "box":
                d["half_extents"] = [float(v) / 2 for v in prim["dimensions"]]
                out["box"].append(d)
            elif prim["type"] == "cylinder":
                d["length"], d["radius"] = float(prim["dimensions"][0]), float(prim["dimensions"][1])
                out["cylinder"].append(d)
            elif prim["type"] == "sphere":
                d["radius"] = float(prim["dimensions"][0])
                out["sphere"].append(d)
    return out


def problem_dict_to_pointcloud(robot: str, problem: dict, samples_per_object: int, filter_radius: float,
                               filter_cull: bool, ctx=None):
    """pointcloud.py:129-167: sample, filter on the GPU around the robot's first joint, build the
    CAPT.  Returns (env, original_pc, filtered_pc, filter_time, build_time); filter_time in
    nanoseconds of wall clock around the GPU filter call, build_time the CAPT build's nanoseconds."""
    from . import Environment, filter_pointcloud

    original = problem_to_pointcloud(problem, samples_per_object)
    origin = ROBOT_FIRST_JOINT_LOCATIONS.get(robot, [0.0, 0.0, 0.0])
    reach = ROBOT_MAX_RADII.get(robot, 1.4)
    lo = np.asarray(origin) - reach
    hi = np.asarray(origin) + reach
    t0 = time.perf_counter_ns()
    filtered = filter_pointcloud(original.astype(np.float32), filter_radius, reach, origin, lo, hi, filter_cull,
                                 ctx)
    filter_time = time.perf_counter_ns() - t0
    r_min, r_max = ROBOT_RADII_RANGES[robot]
    env = Environment()
    build_time = env.add_pointcloud(filtered, r_min, r_max, POINT_RADIUS)
    return env, original.tolist(), filtered.tolist(), filter_time, build_time
