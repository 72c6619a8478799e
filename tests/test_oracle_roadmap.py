"""The PRM roadmap edge stage restated (planning/prm.hh:235-299): PRMStarNeighborParams
(roadmap.hh:42-77), the neighbour query build_roadmap runs per vertex (prm.hh:264-266) and the
adjacency it appends (prm.hh:270-275).

Pins: the k / r formulas against an independent evaluation with Python's math module; the
query against a numpy brute force with the pinned l2_norm lane order (ref_probe "l2norm",
tests/golden/ref_pins_l2.npz); the product's host-side parameter function against the oracle.
nigh (the reference's KD-tree, a CPM download absent here) is exact kNN; its order among
exactly equal distances is not pinned (ties: lower index first here).
"""
import math

import numpy as np
import pytest

F = np.float32


def l2_lanes(v):
    """FloatVector<dim>::l2_norm, dim <= 8 (avx.hh:441-452) in float32, rows of v."""
    sq = np.zeros((v.shape[0], 8), F)
    sq[:, :v.shape[1]] = v * v
    return np.sqrt(((sq[:, 0] + sq[:, 4]) + (sq[:, 2] + sq[:, 6])) + ((sq[:, 1] + sq[:, 5]) + (sq[:, 3] + sq[:, 7])))


@pytest.mark.parametrize("dim", [6, 7, 8, 14])
def test_prm_params_vs_math(oracle, dim):
    sm = oracle.SPACE_MEASURE["panda"]
    ball = math.pow(math.sqrt(math.pi), dim) / math.gamma(dim / 2 + 1)
    prm = 2.0 * math.pow(1 + 1 / dim, 1 / dim) * math.pow(sm / ball, 1 / dim)
    for n in [2, 3, 10, 100, 1000, 12345, 10 ** 5, 4 * 10 ** 6]:
        assert oracle.prm_max_neighbors(dim, n) == math.ceil((math.e + math.e / dim) * math.log(n))
        want = np.float32(2.0 * prm * math.pow(math.log(n) / n, 1 / dim))
        assert oracle.prm_neighbor_radius(dim, sm, 2.0, n) == want


def test_product_params_equal_oracle(oracle):
    """vgpu_prm_neighbor_params (host code of the product, no GPU) == the oracle."""
    from vamp_amd.roadmap import prm_neighbor_params
    for robot, dim in (("panda", 7), ("fetch", 8)):
        sm = oracle.SPACE_MEASURE[robot]
        k, r = prm_neighbor_params(dim, sm, 5000)
        assert k[0] == k[1] == 0
        for i in list(range(2, 200)) + list(range(4900, 5000)):
            assert k[i] == oracle.prm_max_neighbors(dim, i)
            assert r[i] == oracle.prm_neighbor_radius(dim, sm, 2.0, i)


def test_knn_vs_numpy_bruteforce(oracle):
    rng = np.random.default_rng(11)
    V = oracle.scale(rng.random((700, 7), dtype=F))
    V[300] = V[200]  # an exact duplicate: distance 0
    sm = oracle.SPACE_MEASURE["panda"]
    nbr, dist, cnt = oracle.roadmap_knn(V, sm)
    assert cnt[0] == cnt[1] == 0
    for i in range(2, len(V)):
        d = l2_lanes((V[:i] - V[i]).astype(F))
        k = oracle.prm_max_neighbors(7, i)
        r = oracle.prm_neighbor_radius(7, sm, 2.0, i)
        cand = np.nonzero(d <= r)[0]
        order = cand[np.lexsort((cand, d[cand]))][:k]
        assert cnt[i] == len(order), i
        assert np.array_equal(nbr[i, :cnt[i]], order.astype(np.uint32)), i
        assert np.array_equal(dist[i, :cnt[i]], d[order]), i
    assert nbr[300, 0] == 200 and dist[300, 0] == 0


def test_build_roadmap_edges_structure(oracle):
    """Append-order adjacency: symmetric, each list = own valid neighbours (query order) then
    later vertices ascending; components from union-find."""
    rng = np.random.default_rng(12)
    env = oracle.sphere_cage_env()
    q = oracle.scale(rng.random((3000, 7), dtype=F))
    V = q[oracle.fkcc_threads(env, q)][:400]
    edges, (nbr, dist, cnt, ok) = oracle.build_roadmap_edges("panda", env, V)
    n = len(V)
    pos = 0
    for i in range(n):
        own = [int(nbr[i, m]) for m in range(cnt[i]) if ok[pos + m]]
        pos += cnt[i]
        assert edges[i][:len(own)] == own
        assert all(j < i for j in own) and edges[i][len(own):] == sorted(edges[i][len(own):])
        for j in edges[i]:
            assert i in edges[j]
    comp = oracle.components(n, edges)
    for i in range(n):
        for j in edges[i]:
            assert comp[i] == comp[j]
    assert ok.sum() > 0 and (~ok).sum() > 0


def test_prm_settings_mirror(oracle):
    """vamp.PRMNeighborParams / PRMSettings (bindings/settings.cc:38-53): defaults and k/r equal the
    oracle's PRMStarNeighborParams (roadmap.hh:42-77)."""
    import vamp_amd as vamp
    p = vamp.PRMNeighborParams(7, vamp.panda.space_measure())
    st = vamp.PRMSettings(p)
    assert st.max_iterations == 100000 and st.max_samples == 100000 and p.gamma_scale == 2.0
    for n in (2, 3, 10, 1000, 123457):
        assert st.max_neighbors(n) == oracle.prm_max_neighbors(7, n)
        assert np.float32(st.neighbor_radius(n)) == np.float32(oracle.prm_neighbor_radius(7, p.space_measure, 2.0, n))


@pytest.mark.parametrize("robot,dim,n", [("fetch", 8, 3000), ("panda", 7, 2500), ("baxter", 14, 800)])
def test_cpu_kdtree_knn_equals_oracle(oracle, robot, dim, n):
    """vgpu_cpu_roadmap_knn (exact k-d tree, the CPU baseline's neighbour query) == the oracle's brute
    force, on uniform vertices with a duplicate, and on Halton vertices; any query order."""
    from vamp_amd import roadmap
    rng = np.random.default_rng(3)
    V = oracle.robot_scale(robot, rng.random((n, dim), dtype=np.float32))
    V[n // 2] = V[n // 3]
    sm = oracle.SPACE_MEASURE[robot]
    onb, od, oc = oracle.roadmap_knn(V, sm)
    qs = rng.permutation(n).astype(np.uint32)
    nb, d, c = roadmap.cpu_knn(V, qs, sm, kmax=onb.shape[1], threads=4)
    assert np.array_equal(c, oc[qs])
    mask = np.arange(onb.shape[1])[None, :] < c[:, None]
    assert np.array_equal(nb[mask], onb[qs][mask]) and np.array_equal(d[mask], od[qs][mask])
