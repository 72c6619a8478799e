"""Seeded synthetic scenes of SURVEY §8(d) shared by tests and bench (numpy only)."""
import numpy as np

F = np.float32

CAGE = np.array([(0.55, 0, 0.25), (0.35, 0.35, 0.25), (0, 0.55, 0.25), (-0.55, 0, 0.25), (-0.35, -0.35, 0.25),
                 (0, -0.55, 0.25), (0.35, -0.35, 0.25), (0.35, 0.35, 0.8), (0, 0.55, 0.8), (-0.35, 0.35, 0.8),
                 (-0.55, 0, 0.8), (-0.35, -0.35, 0.8), (0, -0.55, 0.8), (0.35, -0.35, 0.8)])
# Panda point-cloud radii (reference src/vamp/constants.py:57-77)
R_MIN, R_MAX, R_POINT = 0.012, 0.06, 0.0025


def cage_points(n=10000, seed=1):
    """Config 3: n points normal-normalised onto the 14 cage spheres (r = 0.2), tie-free."""
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    p = (CAGE[rng.integers(0, len(CAGE), n)] + 0.2 * v).astype(F)
    # the reference's pdqsort leaves equal coordinates unordered: make every axis tie-free by
    # nudging repeats up one ulp at a time (deterministic, a few points per 10k)
    for k in range(3):
        while True:
            order = np.argsort(p[:, k], kind="stable")
            col = p[order, k]
            dup = np.where(col[1:] == col[:-1])[0] + 1
            if len(dup) == 0:
                break
            p[order[dup], k] = np.nextafter(col[dup], np.float32(np.inf))
    return p


def raw_queries(n, seed=3):
    """Config 3 raw sphere queries: x, y ~ U[-1, 1], z ~ U[0, 1.2], r ~ U[0.012, 0.06]."""
    rng = np.random.default_rng(seed)
    c = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(0, 1.2, n)], 1).astype(F)
    r = rng.uniform(R_MIN, R_MAX, n).astype(F)
    return c, r


def terrain(xd=64, yd=48, seed=5):
    """A smooth heightfield: (center, scale, dims, data) in factory::heightfield::array terms.
    5 cm cells over 3.2 m x 2.4 m; height = data / scale_z + center_z = 0.125 .. 0.375 m above
    the centre (zs = 1/scale_z, sphere_heightfield.hh:25)."""
    rng = np.random.default_rng(seed)
    xs, ys = np.meshgrid(np.linspace(0, 3 * np.pi, yd), np.linspace(0, 2 * np.pi, xd))
    d = (0.5 + 0.25 * np.sin(xs + rng.uniform(0, 6)) * np.cos(ys + rng.uniform(0, 6))).astype(F)
    return (0.0, 0.0, 0.0), (0.05, 0.05, 2.0), (xd, yd), d.ravel()
