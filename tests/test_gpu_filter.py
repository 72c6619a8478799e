"""GPU point-cloud filter (vgpu_filter.hip) against the oracle's restatement of
filter_pointcloud (collision/filter.hh:175-268): the kept indices, in order, bit-exact.
Order among equal Morton codes is stable on both sides (the reference's pdqsort is unstable:
parity unpinned there)."""
import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu

F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def cases():
    rng = np.random.default_rng(11)
    yield "uniform", rng.uniform(-1, 1, (20000, 3)).astype(F), 0.02, 1.2, True
    yield "nocull", rng.uniform(-1, 1, (5000, 3)).astype(F), 0.05, 1.0, False
    # cage-sphere surfaces (SURVEY §8d config 3 style), dense: many close pairs
    c = rng.normal(size=(30000, 3)).astype(F)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    yield "sphere", (0.3 * c + np.array([0.2, -0.1, 0.5], F)).astype(F), 0.01, 1.5, True
    yield "one", np.array([[0.1, 0.2, 0.3]], F), 0.1, 1.0, True
    yield "dups", np.repeat(rng.uniform(-0.5, 0.5, (50, 3)).astype(F), 40, axis=0), 0.001, 1.0, False


@pytest.mark.parametrize("name,pc,md,rng_,cull", list(cases()), ids=[c[0] for c in cases()])
def test_filter_matches_oracle(vamp, name, pc, md, rng_, cull):
    args = (md, rng_, [0.1, 0.0, 0.2], [-0.95, -0.95, -0.95], [0.95, 0.95, 0.95], cull)
    want = O.filter_pointcloud(pc, *args)
    got = vamp.filter_pointcloud_indices(pc, *args)
    assert got.dtype == np.uint32
    np.testing.assert_array_equal(got, want)
    pts = vamp.filter_pointcloud(pc, *args)
    np.testing.assert_array_equal(pts, pc[want])


def test_filter_empty(vamp):
    assert vamp.filter_pointcloud_indices(np.zeros((0, 3), F), 0.1, 1.0, [0] * 3, [-1] * 3, [1] * 3).size == 0


def test_filter_mostly_culled_1m(vamp):
    """a 1M-point cloud wider than the workspace culls ~95 % of its points; the
    reference's n-long list then ends in ~950k copies of point 0 (filter.hh:194-214).  The GPU
    keeps one copy (exact, see vgpu_filter.hip) -- same indices as the oracle, and fast."""
    import time
    rng = np.random.default_rng(3)
    n = 1 << 20
    pc = np.empty((n, 3), F)
    pc[:, :2] = rng.uniform(-3, 3, (n, 2))
    pc[:, 2] = rng.uniform(-0.5, 2.0, n)
    args = (0.005, 1.5, [0.0, 0.0, 0.5], [-1.2, -1.2, -1.2], [1.2, 1.2, 1.2], True)
    vamp.filter_pointcloud_indices(pc[:4096], *args)  # warm the scratch pool
    t = time.perf_counter()
    got = vamp.filter_pointcloud_indices(pc, *args)
    dt = time.perf_counter() - t
    want = O.filter_pointcloud(pc, *args)
    np.testing.assert_array_equal(got, want)
    assert dt < 1.0, dt  # was O((N - kept)^2) before the tail collapse
