"""MotionBenchMaker point-cloud harness (vamp_amd.pointcloud, the mirror of the reference's
src/vamp/pointcloud.py:1-167): surface samplers, the MBM scene -> problem dict, and the
sample -> filter -> CAPT pipeline.

Parity: the samplers restate pointcloud.py's float64 numpy arithmetic draw for draw; the reference
package cannot be imported here (it needs its compiled extension), so the sampled points are
parity-unpinned and checked by their properties (on the surfaces, per-object counts, seed
determinism).  Downstream, the GPU filter and the CAPT build are checked bit-exact against the
oracle on the harness's own cloud (GPU test), and fkcc against the filtered cloud == oracle.
Fixture: tests/golden/mbm_table_pick_panda_0001.json (tools/make_pc_fixture.py).
"""
import json
import os

import numpy as np
import pytest

from vamp_amd import pointcloud as vpc

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def problem():
    with open(os.path.join(HERE, "golden", "mbm_table_pick_panda_0001.json")) as f:
        return json.load(f)


def _local(points, obj):
    M = vpc.pose_matrix(obj["position"], obj["orientation_quat_xyzw"])
    return (points - M[:3, 3]) @ M[:3, :3]  # rotate back (orthonormal)


def test_fixture_objects(problem):
    assert len(problem["box"]) == 10 and len(problem["cylinder"]) == 2
    for b in problem["box"]:
        assert len(b["half_extents"]) == 3 and min(b["half_extents"]) > 0
    for c in problem["cylinder"]:
        assert c["radius"] > 0 and c["length"] > 0


def test_pose_matrix_is_rigid():
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.normal(size=4)
        M = vpc.pose_matrix(rng.normal(size=3), q)
        R = M[:3, :3]
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
        assert abs(np.linalg.det(R) - 1) < 1e-12
    # x y z w order: a quarter turn about z maps x to y
    M = vpc.pose_matrix([0, 0, 0], [0, 0, np.sin(np.pi / 4), np.cos(np.pi / 4)])
    np.testing.assert_allclose(M[:3, :3] @ [1, 0, 0], [0, 1, 0], atol=1e-12)
    np.testing.assert_array_equal(vpc.pose_matrix([1, 2, 3], [0, 0, 0, 0]), np.array(
        [[1, 0, 0, 1], [0, 1, 0, 2], [0, 0, 1, 3], [0, 0, 0, 1]], float))


def test_samples_lie_on_the_surfaces(problem):
    n = 500
    pc = vpc.problem_to_pointcloud(problem, n)
    objs = problem["cylinder"] + problem["box"]  # cylinders first (pointcloud.py:122-126)
    assert pc.shape == (n * len(objs), 3) and pc.dtype == np.float64
    for k, o in enumerate(objs):
        loc = _local(pc[k * n:(k + 1) * n], o)
        if "half_extents" in o:
            h = np.asarray(o["half_extents"])
            assert (np.abs(loc) <= h + 1e-9).all()
            on_face = np.isclose(np.abs(loc), h, atol=1e-9).any(axis=1)
            assert on_face.all()
        else:
            r = np.hypot(loc[:, 0], loc[:, 1])
            on_cap = np.isclose(np.abs(loc[:, 2]), o["length"] / 2, atol=1e-9) & (r <= o["radius"] + 1e-9)
            on_side = np.isclose(r, o["radius"], atol=1e-9) & (np.abs(loc[:, 2]) <= o["length"] / 2 + 1e-9)
            assert (on_cap | on_side).all()
            assert on_side.any() and on_cap.any()


def test_sampler_is_seeded(problem):
    a = vpc.problem_to_pointcloud(problem, 64)
    b = vpc.problem_to_pointcloud(problem, 64)
    np.testing.assert_array_equal(a, b)
    c = vpc.problem_to_pointcloud({"box": problem["box"][:1]}, 64)
    np.random.seed(0)
    d = vpc.box_to_pc(problem["box"][0], 64)
    np.testing.assert_array_equal(c, d)


def test_face_choice_follows_area():
    # a flat box: the two large faces take almost every sample
    np.random.seed(1)
    pts = vpc.cuboid_sample_surface(np.identity(4), [1.0, 1.0, 0.01], 20000, 0)
    frac = np.isclose(np.abs(pts[:, 2]), 0.005).mean()
    assert 0.97 < frac < 0.995


def test_sphere_sampler():
    np.random.seed(2)
    p = vpc.sphere_sample_surface(np.array([1.0, 2.0, 3.0]), 0.5, 1000, 0.0)
    np.testing.assert_allclose(np.linalg.norm(p - [1, 2, 3], axis=1), 0.5, atol=1e-12)


def test_scene_conversion_roundtrip(problem):
    scene = {"world": {"collision_objects": [
        {"id": "a", "primitives": [{"type": "box", "dimensions": [0.2, 0.4, 0.6]},
                                   {"type": "cylinder", "dimensions": [0.5, 0.05]}],
         "primitive_poses": [{"position": [1, 2, 3], "orientation": [0, 0, 0, 1]},
                             {"position": [0, 0, 1], "orientation": [0, 0, 0, 1]}]}]}}
    d = vpc.scene_to_problem_dict(scene, "x")
    assert d["box"][0]["half_extents"] == [0.1, 0.2, 0.3]
    assert d["cylinder"][0]["length"] == 0.5 and d["cylinder"][0]["radius"] == 0.05
    assert d["box"][0]["orientation_quat_xyzw"] == [0.0, 0.0, 0.0, 1.0]


@pytest.mark.gpu
def test_mbm_pipeline_matches_oracle(problem):
    """problem_dict_to_pointcloud on the GPU: the filter keeps exactly the oracle's points, the
    CAPT equals the oracle's build bit for bit, and Panda fkcc against it == oracle."""
    import oracle_py as O

    import vamp_amd as vamp
    env, orig, filt, ft, bt = vpc.problem_dict_to_pointcloud("panda", problem, 2000, 0.01, True)
    orig = np.asarray(orig, np.float32)
    filt = np.asarray(filt, np.float32)
    assert orig.shape == (12 * 2000, 3) and 0 < filt.shape[0] < orig.shape[0] and ft > 0 and bt > 0
    o, reach = vpc.ROBOT_FIRST_JOINT_LOCATIONS["panda"], vpc.ROBOT_MAX_RADII["panda"]
    want = O.filter_pointcloud(orig, 0.01, reach, o, np.asarray(o) - reach, np.asarray(o) + reach, True)
    np.testing.assert_array_equal(filt.view(np.uint32), orig[want].view(np.uint32))
    r_min, r_max = vpc.ROBOT_RADII_RANGES["panda"]
    got = env.pointcloud_arrays()
    ref = O.Capt(filt, r_min, r_max, vpc.POINT_RADIUS).arrays()
    for k in ("nlog2", "tests", "aabbs", "aff_starts", "aff"):
        a, b = np.atleast_1d(np.asarray(got[k])), np.atleast_1d(np.asarray(ref[k]))
        assert a.shape == b.shape and a.dtype == b.dtype, k
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), k
    rng = np.random.default_rng(5)
    q = vamp.panda_0_0.scale_configuration(rng.uniform(0, 1, (4096, 7)).astype(np.float32))
    oe = O.Env().add_pointcloud(filt, r_min, r_max, vpc.POINT_RADIUS)
    valid = vamp.panda_0_0.fkcc_batch(q, env)
    np.testing.assert_array_equal(np.asarray(valid, bool), O.fkcc(oe, q))
    print(f"MBM table_pick_panda #1: {orig.shape[0]} sampled, {filt.shape[0]} kept, "
          f"{int(np.count_nonzero(valid))}/{q.shape[0]} configurations valid")
