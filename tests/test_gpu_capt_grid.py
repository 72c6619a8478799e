"""The device point cloud's cell grid (mr-vamp_amd/csrc/vgpu_capt_grid.hip) changes no answer:
raw CAPT::collides_simd queries (collision/capt.hh:457-541) through the HIP path, with the grid at
several sizes and without it, == the C restatement bit for bit -- on queries placed where the
grid's bounds are tightest: radii within a few ulps of a point's distance, centres on and around
the cloud, huge / negative / non-finite radii, and degenerate clouds (one point, a plane, a line,
repeated points)."""
import os

import numpy as np
import pytest

from scenes import R_MAX, R_MIN, R_POINT, cage_points, raw_queries

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def boundary_queries(pts, n, seed):
    """centres at distance d from a cloud point, radius = d - r_point nudged by -4..4 ulps, and a
    spread of radii around it (bounding-sphere sizes included)."""
    rng = np.random.default_rng(seed)
    p = pts[rng.integers(0, len(pts), n)].astype(np.float64)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    d = rng.uniform(0.002, 0.3, n)
    c = (p + v * d[:, None]).astype(F)
    dd = np.linalg.norm(c.astype(np.float64) - p, axis=1)
    r = (dd - R_POINT).astype(F)
    k = rng.integers(-4, 5, n)
    r = np.array([np.float32(x) for x in r])
    for i in range(n):
        for _ in range(abs(int(k[i]))):
            r[i] = np.nextafter(r[i], np.float32(np.inf if k[i] > 0 else -np.inf))
    scale = rng.choice([0.5, 0.9, 0.99, 1.0, 1.01, 1.1, 2.0], n).astype(F)
    r2 = (r * scale).astype(F)
    big = rng.uniform(0.1, 0.4, n).astype(F)
    return np.concatenate([c, c, c]), np.concatenate([r, r2, big])


def check(vamp, oracle, pts, c, r, cells=None, layout=None):
    """layout: {"VGPU_CAPT_BRICK": "0"|"1", "VGPU_CAPT_SPLIT": "0"|"1"} (None: the defaults, bricks + split)"""
    sets = {"VGPU_CAPT_GRID_CELLS": None if cells is None else str(cells), **(layout or {})}
    old = {k: os.environ.get(k) for k in sets}
    try:
        for k, v in sets.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        env = vamp.Environment()
        env.add_pointcloud(pts, R_MIN, R_MAX, R_POINT)
        got = env.pointcloud_collides(c, r, simd=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    want = oracle.Capt(pts, R_MIN, R_MAX, R_POINT).collides(c, r, simd=True)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (f"cells={cells} layout={layout}: {len(bad)} mismatches, first {bad[:5]} "
                           f"c={c[bad[:3]]} r={r[bad[:3]]}")
    return got


@pytest.mark.parametrize("cells", [None, 0, 4096, 1 << 21])
def test_grid_boundary_queries(vamp, oracle, cells):
    pts = cage_points()
    c, r = boundary_queries(pts, 1 << 15, seed=7)
    got = check(vamp, oracle, pts, c, r, cells)
    assert 0.05 < got.mean() < 0.99
    c2, r2 = raw_queries(1 << 16, seed=11)
    check(vamp, oracle, pts, c2, r2, cells)


def test_grid_special_radii(vamp, oracle):
    pts = cage_points()
    rng = np.random.default_rng(3)
    c = pts[rng.integers(0, len(pts), 64)] + rng.normal(scale=0.03, size=(64, 3)).astype(F)
    c = np.repeat(c.astype(F), 7, axis=0)
    r = np.tile(np.array([0.0, -0.01, -1.0, np.inf, np.nan, 1e-30, 5.0], F), 64)
    check(vamp, oracle, pts, c, r)


@pytest.mark.parametrize("shape", ["one", "plane", "line", "repeats", "far"])
def test_grid_degenerate_clouds(vamp, oracle, shape):
    rng = np.random.default_rng(5)
    if shape == "one":
        pts = np.array([[0.1, 0.2, 0.3]], F)
    elif shape == "plane":
        pts = np.stack([rng.uniform(-1, 1, 3000), rng.uniform(-1, 1, 3000), np.full(3000, 0.25)], 1).astype(F)
    elif shape == "line":
        pts = np.stack([np.linspace(-1, 1, 500), np.full(500, 0.1), np.full(500, 0.4)], 1).astype(F)
    elif shape == "repeats":
        pts = np.repeat(cage_points(300, seed=9), 4, axis=0)
    else:  # a cloud 1 km from the origin: large coordinates, small cells
        pts = (cage_points(2000, seed=4) + np.array([1000.0, -700.0, 30.0], F)).astype(F)
    c, r = boundary_queries(pts, 4096, seed=2)
    check(vamp, oracle, pts, c, r)
    check(vamp, oracle, pts, c, r, cells=0)


# the grid's storage layouts (vgpu_capt.cpp capt_grid_plan): x-fastest rows or 4 x 4 x 4 bricks, one uint2
# {bounds, node} per cell or separate bound / node planes -- the same answers under each
@pytest.mark.parametrize("brick,split", [("0", "0"), ("0", "1"), ("1", "0"), ("1", "1")])
def test_grid_layouts(vamp, oracle, brick, split):
    layout = {"VGPU_CAPT_BRICK": brick, "VGPU_CAPT_SPLIT": split}
    pts = cage_points()
    c, r = boundary_queries(pts, 1 << 14, seed=13)
    check(vamp, oracle, pts, c, r, layout=layout)
    check(vamp, oracle, pts, c, r, cells=4096, layout=layout)
    far = (cage_points(2000, seed=4) + np.array([1000.0, -700.0, 30.0], F)).astype(F)
    c, r = boundary_queries(far, 4096, seed=2)
    check(vamp, oracle, far, c, r, layout=layout)


def test_grid_deep_tree(vamp, oracle):
    """40k points: a tree of depth 16, whose grid build walks with the 32-deep LDS stack (trees of depth < 16
    take the 16-deep one)"""
    pts = cage_points(40000, seed=21)
    c, r = boundary_queries(pts, 1 << 14, seed=17)
    got = check(vamp, oracle, pts, c, r)
    assert 0.05 < got.mean() < 0.99
    c2, r2 = raw_queries(1 << 15, seed=19)
    check(vamp, oracle, pts, c2, r2)
