"""vamp.<robot>.filter_from_pointcloud (bindings/common.hh:36-87, bound at :713) on the GPU against
the oracle restatement (oracle/vamp_oracle.c vo_robot_filter_pointcloud): the kept points, in input
order, bit for bit -- Panda at both bases, Fetch, UR5 and Baxter, with an environment of every
primitive type, with a point-cloud (CAPT) environment, and with an empty one.  The robot-sphere test
is the reference's scalar float sphere_sphere_sql2 as its release build contracts it (pinned by
ref_probe "sql2s", tests/test_ref_pin.py)."""
import numpy as np
import pytest

from scenes import R_MAX, R_MIN, R_POINT, cage_points
from test_gpu_parity import gpu_env_from_oracle, random_scene

pytestmark = pytest.mark.gpu
F = np.float32
DIMS = {"panda": 7, "fetch": 8, "ur5": 6, "baxter": 14}


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def cloud_near_robot(oracle, robot, q, base, n, rng):
    """points on and around the robot's spheres at q (many overlap, many graze), plus clutter"""
    c = oracle.robot_sphere_fk(robot, q[None], base)[0]
    pick = c[rng.integers(0, len(c), n // 2)]
    d = rng.normal(size=(n // 2, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    near = pick + d * rng.uniform(0.0, 0.2, (n // 2, 1))
    far = rng.uniform([-1.2, -1.2, -0.2], [1.2, 1.2, 1.6], (n - n // 2, 3))
    if base != (0, 0, 0):
        far += np.array(base, np.float64) / 100.0
    return np.concatenate([near, far]).astype(F)


@pytest.mark.parametrize("robot,base", [("panda", (0, 0, 0)), ("panda", (200, 200, 0)), ("fetch", (0, 0, 0)),
                                        ("ur5", (0, 0, 0)), ("baxter", (0, 0, 0))])
def test_filter_from_pointcloud_equals_oracle(vamp, oracle, robot, base):
    rng = np.random.default_rng(hash(robot) % 1000 + base[0])
    oenv = random_scene(oracle, rng, 3, 3, 2)
    env = gpu_env_from_oracle(vamp, oenv)
    rob = vamp.PandaBase(*base) if robot == "panda" else getattr(vamp, robot)
    dim = DIMS[robot]
    for trial in range(3):
        q = oracle.robot_scale(robot, rng.random((1, dim), dtype=F))[0]
        pc = cloud_near_robot(oracle, robot, q, base, 20000, rng)
        for pr in (0.0025, 0.02):
            keep = oracle.robot_filter_pointcloud(robot, oenv, q, pc, pr, base)
            got = rob.filter_from_pointcloud(pc, q, env, pr)
            assert np.array_equal(got, pc[keep]), (robot, trial, pr, len(got), int(keep.sum()))
            assert 0.05 < keep.mean() < 0.95
    # empty environment: only the robot's own spheres remove points
    empty = vamp.Environment()
    q = oracle.robot_scale(robot, rng.random((1, dim), dtype=F))[0]
    pc = cloud_near_robot(oracle, robot, q, base, 5000, rng)
    keep = oracle.robot_filter_pointcloud(robot, oracle.Env(), q, pc, 0.01, base)
    assert np.array_equal(rob.filter_from_pointcloud(pc, q, empty, 0.01), pc[keep])
    assert rob.filter_from_pointcloud(np.zeros((0, 3), F), q, empty, 0.01).shape == (0, 3)


def test_filter_from_pointcloud_capt_env_and_device(vamp, oracle):
    """A point-cloud environment (the CAPT path of sphere_environment_in_collision) and the device
    form (keep flags straight into HBM)."""
    import torch
    pts = cage_points(4000, 9)
    oenv = oracle.Env().add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
    env = vamp.Environment()
    env.add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
    rng = np.random.default_rng(5)
    q = oracle.scale(rng.random((1, 7), dtype=F))[0]
    pc = np.concatenate([cloud_near_robot(oracle, "panda", q, (0, 0, 0), 8000, rng),
                         (pts[:2000] + rng.normal(0, 0.01, (2000, 3))).astype(F)])
    keep = oracle.robot_filter_pointcloud("panda", oenv, q, pc, 0.005)
    assert np.array_equal(vamp.panda_0_0.filter_from_pointcloud(pc, q, env, 0.005), pc[keep])
    d = torch.from_numpy(pc).cuda()
    k = torch.empty(len(pc), dtype=torch.uint8, device="cuda")
    vamp.panda_0_0.filter_from_pointcloud_device(d.data_ptr(), len(pc), q, env, 0.005, k.data_ptr())
    vamp.context().sync()
    assert np.array_equal(k.cpu().numpy().astype(bool), keep)
