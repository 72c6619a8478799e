"""CAPT built on the device (vgpu_capt_build.hip, SURVEY §8f rank 4 second half) against the host
build (vgpu_capt.cpp, itself == the oracle's restatement bit for bit, tests/test_capt.py): every
array identical -- median tests, leaf boxes, affordance starts and the +inf-padded affordance
vectors -- on clouds of several sizes (powers of two and not, 1 and 2 points), with exact ties
(duplicated points, shared coordinates: both builds order equal keys by point index), and on the
MotionBenchMaker harness's filtered cloud fed straight from device memory."""
import json
import os

import numpy as np
import pytest

from scenes import R_MAX, R_MIN, R_POINT, cage_points

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def _same(a, b):
    a, b = np.atleast_1d(np.asarray(a)), np.atleast_1d(np.asarray(b))
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def _device_vs_host(torch, pts, r_min=R_MIN, r_max=R_MAX, r_point=R_POINT):
    import vamp_amd as vamp
    pts = np.ascontiguousarray(pts, np.float32)
    host = vamp.Environment()
    host.add_pointcloud(pts, r_min, r_max, r_point)
    want = host.pointcloud_arrays()
    d = torch.from_numpy(pts).to("cuda:0")
    env = vamp.Environment()
    ns = env.add_pointcloud_device(d.data_ptr(), pts.shape[0], r_min, r_max, r_point)
    assert ns > 0
    got = env.pointcloud_arrays()
    for k in ("nlog2", "tests", "aabbs", "aff_starts", "aff", "aabb_top"):
        assert _same(got[k], want[k]), k
    return env, d


def _ties(n, seed):
    rng = np.random.default_rng(seed)
    base = rng.uniform(-0.6, 0.6, (n // 4, 3)).astype(np.float32)
    pts = np.concatenate([base, base, np.round(rng.uniform(-0.6, 0.6, (n - 2 * (n // 4), 3)), 1)]).astype(np.float32)
    pts[::7, 0] = 0.25  # a shared coordinate plane
    pts[::11, 2] = -0.0  # signed zeros compare equal to +0
    return pts


@pytest.mark.parametrize("n,seed", [(10000, 1), (1000, 7), (777, 8), (2, 9), (1, 10), (4096, 11), (33333, 12)])
def test_device_build_equals_host(torch, n, seed):
    _device_vs_host(torch, cage_points(n, seed))


@pytest.mark.parametrize("n,seed", [(3000, 21), (512, 22)])
def test_device_build_with_ties(torch, n, seed):
    _device_vs_host(torch, _ties(n, seed))


def test_device_built_env_queries(torch):
    """fkcc against the device-built tree == against the host-built one (same arrays, same query)."""
    import vamp_amd as vamp
    pts = cage_points(5000, 3)
    env_d, keep = _device_vs_host(torch, pts)
    env_h = vamp.Environment()
    env_h.add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
    q = vamp.panda_0_0.scale_configuration(np.random.default_rng(4).uniform(0, 1, (8192, 7)).astype(np.float32))
    a = np.asarray(vamp.panda_0_0.fkcc_batch(q, env_d), bool)
    b = np.asarray(vamp.panda_0_0.fkcc_batch(q, env_h), bool)
    np.testing.assert_array_equal(a, b)
    assert 0 < a.mean() < 1


def test_mbm_cloud_device_build(torch):
    from vamp_amd import pointcloud as vpc
    with open(os.path.join(HERE, "golden", "mbm_table_pick_panda_0001.json")) as f:
        problem = json.load(f)
    _, _, filt, _, _ = vpc.problem_dict_to_pointcloud("panda", problem, 2000, 0.01, True)
    r_min, r_max = vpc.ROBOT_RADII_RANGES["panda"]
    _device_vs_host(torch, np.asarray(filt, np.float32), r_min, r_max, vpc.POINT_RADIUS)


def test_device_built_cloud_outlives_points_and_edits(torch):
    """The device-built arrays live in the environment's host twin: after the points are freed and an
    obstacle is added, realising the environment again (handle()) copies the arrays -- no rebuild, no
    read of the freed buffer -- and fkcc equals an environment built on the host with the same edits."""
    import vamp_amd as vamp
    pts = cage_points(4000, 5)
    d = torch.from_numpy(pts).to("cuda:0")
    env_d = vamp.Environment()
    env_d.add_pointcloud_device(d.data_ptr(), pts.shape[0], R_MIN, R_MAX, R_POINT)
    q = vamp.panda_0_0.scale_configuration(np.random.default_rng(6).uniform(0, 1, (4096, 7)).astype(np.float32))
    first = vamp.panda_0_0.fkcc_batch(q, env_d)
    del d
    torch.cuda.empty_cache()
    env_d.add_sphere(vamp.Sphere([0.4, 0.0, 0.5], 0.1))  # invalidates the device copy: realised again
    env_h = vamp.Environment()
    env_h.add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
    env_h.add_sphere(vamp.Sphere([0.4, 0.0, 0.5], 0.1))
    a = vamp.panda_0_0.fkcc_batch(q, env_d)
    np.testing.assert_array_equal(a, vamp.panda_0_0.fkcc_batch(q, env_h))
    assert (a <= first).all() and a.sum() < first.sum()
    if torch.cuda.device_count() > 1:  # a second context realises it from the same arrays
        ctx1 = vamp.context(1)
        np.testing.assert_array_equal(vamp.panda_0_0.fkcc_batch(q, env_d, ctx1), a)
