"""GPU parity of the PRM roadmap edge stage: the causal kNN kernel and
vgpu_build_roadmap_host (neighbour queries + batched validate_motion + append-order adjacency +
union-find) against the oracle's build_roadmap restatement on the same host: identical
neighbour lists, distances, edge lists and components."""
import numpy as np
import pytest

from test_gpu_parity import gpu_env_from_oracle, random_scene

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


def knn_gpu(vamp, V, sm, kmax=None, mode=0, q_first=0, q_count=None):
    """vgpu_roadmap_knn_range on the GPU with the context's kNN method set to `mode` (0 auto, 1 brute
    force, 2 spatial index); rows are indexed from q_first"""
    import torch
    from vamp_amd import roadmap
    n, dim = V.shape
    q_count = n - q_first if q_count is None else q_count
    k, r = roadmap.prm_neighbor_params(dim, sm, n)
    kmax = kmax or int(max(1, k.max()))
    dev = torch.device("cuda", 0)
    tV = torch.from_numpy(V).to(dev)
    tk = torch.from_numpy(k.view(np.int32)).to(dev)
    tr = torch.from_numpy(r).to(dev)
    nbr = torch.zeros((max(q_count, 1), kmax), dtype=torch.int32, device=dev)
    dist = torch.zeros((max(q_count, 1), kmax), dtype=torch.float32, device=dev)
    cnt = torch.zeros(max(q_count, 1), dtype=torch.int32, device=dev)
    ctx = vamp.context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    from vamp_amd._lib import check, load
    check(load().vgpu_set_knn_mode(ctx.h, mode), ctx.h)
    try:
        check(load().vgpu_roadmap_knn_range(ctx.h, dim, tV.data_ptr(), n, q_first, q_count, tk.data_ptr(),
                                            tr.data_ptr(), kmax, nbr.data_ptr(), dist.data_ptr(), cnt.data_ptr()),
              ctx.h)
        torch.cuda.synchronize()
    finally:
        load().vgpu_set_knn_mode(ctx.h, 0)
    return nbr.cpu().numpy().view(np.uint32), dist.cpu().numpy(), cnt.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("mode", [1, 2], ids=["brute", "index"])
@pytest.mark.parametrize("robot,dim,n", [("panda", 7, 20000), ("fetch", 8, 6000), ("ur5", 6, 3000),
                                         ("baxter", 14, 3000)])
def test_knn_equals_oracle(vamp, oracle, robot, dim, n, mode):
    rng = np.random.default_rng(21)
    V = oracle.robot_scale(robot, rng.random((n, dim), dtype=F))
    V[n // 2] = V[n // 3]  # duplicate vertex (distance 0)
    sm = oracle.SPACE_MEASURE[robot]
    onb, od, oc = oracle.roadmap_knn(V, sm)
    gnb, gd, gc = knn_gpu(vamp, V, sm, onb.shape[1], mode=mode)
    assert np.array_equal(gc, oc)
    mask = np.arange(onb.shape[1])[None, :] < oc[:, None]
    assert np.array_equal(gnb[mask], onb[mask]) and np.array_equal(gd[mask], od[mask])
    assert oc[2:].min() >= 1


def test_build_roadmap_equals_oracle(vamp, oracle):
    """Vertices = start, goal, valid Halton samples (the GPU sampling stage); edges and
    components of build_roadmap on the sphere cage."""
    oenv = oracle.sphere_cage_env()
    env = gpu_env_from_oracle(vamp, oenv)
    robot = vamp.panda_0_0
    draws = vamp.halton(7, 1, 6000)
    q = robot.scale_configuration(draws)
    valid = robot.fkcc_batch(q, env)
    start, goal = q[valid][0], q[valid][1]
    V = np.concatenate([start[None], goal[None], q[valid][2:2500]]).astype(F)
    from vamp_amd import roadmap
    rm = roadmap.build_roadmap_edges(robot, env, V)
    edges, _ = oracle.build_roadmap_edges("panda", oenv, V)
    assert rm.edges == edges
    assert np.array_equal(rm.component, oracle.components(len(V), edges))
    assert rm.n_edges() > len(V)


def test_build_roadmap_end_to_end(vamp, oracle):
    """Roadmap::build_roadmap with max_iterations draws and max_samples vertices on a mixed
    primitive scene: vertex sequence and graph equal the oracle's."""
    rng = np.random.default_rng(22)
    oenv = random_scene(oracle, rng, 3, 3, 2)
    env = gpu_env_from_oracle(vamp, oenv)
    robot = vamp.panda_0_0
    s = oracle.scale(rng.random((1, 7), dtype=F))[0]
    g = oracle.scale(rng.random((1, 7), dtype=F))[0]
    from vamp_amd import roadmap
    rm = roadmap.build_roadmap(robot, s, g, env, max_iterations=4000, max_samples=1500)
    V = rm.vertices
    q = oracle.scale(oracle.halton(7, range(1, 4001)))
    want = np.concatenate([s[None], g[None], q[oracle.fkcc_threads(oenv, q)]])[:1500]
    assert np.array_equal(V, want)
    edges, _ = oracle.build_roadmap_edges("panda", oenv, V)
    assert rm.edges == edges


def test_sharded_edges_single_process_equals_oracle(vamp, oracle):
    """build_roadmap_edges_sharded (queries -> device pairs -> assemble) at world size 1."""
    import torch
    from vamp_amd import roadmap
    rng = np.random.default_rng(23)
    oenv = random_scene(oracle, rng, 4, 4, 2)
    env = gpu_env_from_oracle(vamp, oenv)
    q = oracle.robot_scale("fetch", rng.random((5000, 8), dtype=F))
    V = q[oracle.robot_fkcc_threads("fetch", oenv, q)][:2000]
    rm = roadmap.build_roadmap_edges_sharded(torch, None, vamp.fetch, env, torch.from_numpy(V).cuda())
    edges, _ = oracle.build_roadmap_edges("fetch", oenv, V)
    assert rm.edges == edges
    assert np.array_equal(rm.component, oracle.components(len(V), edges))


def _same_lists(a, b):
    (an, ad, ac), (bn, bd, bc) = a, b
    assert np.array_equal(ac, bc)
    mask = np.arange(an.shape[1])[None, :] < ac[:, None]
    assert np.array_equal(an[mask], bn[mask]) and np.array_equal(ad[mask], bd[mask])


def test_knn_index_halton_ties_and_ranges(vamp, oracle):
    """Spatial index vs the oracle on Halton vertices (the PRM vertex sequence: regular spacing,
    many near-equal distances) with exact duplicate clusters (distance-0 ties resolved by index),
    a clump of identical points larger than a tile, and query sub-ranges (one rank's share)."""
    dim, n = 8, 12000
    V = oracle.robot_scale("fetch", oracle.halton(8, range(1, n + 1)).astype(F))
    V[5000:5100] = V[4000]  # 100 copies of one vertex: one tile's box degenerates to a point
    V[7001] = V[17]
    sm = oracle.SPACE_MEASURE["fetch"]
    want = oracle.roadmap_knn(V, sm)
    kmax = want[0].shape[1]
    _same_lists(knn_gpu(vamp, V, sm, kmax, mode=2), want)
    for qf, qc in [(0, 1), (1, 5), (4990, 300), (n - 777, 777)]:
        got = knn_gpu(vamp, V, sm, kmax, mode=2, q_first=qf, q_count=qc)
        _same_lists(got, tuple(x[qf:qf + qc] for x in want))


@pytest.mark.parametrize("n", [200000, 1300000], ids=["2e5", "1.3e6"])
def test_knn_index_equals_brute_force_large(vamp, oracle, n):
    """Beyond the oracle's reach in a test, the indexed query equals the GPU brute force (which equals
    the oracle at the smaller sizes above) -- at 2e5 and at 1.3e6 Fetch vertices, the regime where
    the auto mode picks the index (include/vamp_gpu.h vgpu_set_knn_mode: from 65536)."""
    import time
    V = vamp.fetch.scale_configuration(vamp.halton(8, 1, n))
    sm = oracle.SPACE_MEASURE["fetch"]
    t = time.perf_counter()
    idx = knn_gpu(vamp, V, sm, mode=2)
    t_idx = time.perf_counter() - t
    t = time.perf_counter()
    bf = knn_gpu(vamp, V, sm, mode=1)
    t_bf = time.perf_counter() - t
    print(f"knn {n} Fetch vertices: index {t_idx * 1e3:.1f} ms, brute force {t_bf * 1e3:.1f} ms (incl. transfers)")
    _same_lists(idx, bf)
    auto = knn_gpu(vamp, V, sm, mode=0)
    _same_lists(auto, bf)


@pytest.mark.parametrize("max_iterations,max_samples", [(3000, 800), (2000, 100000)], ids=["samples", "iterations"])
def test_robot_roadmap_binding(vamp, oracle, max_iterations, max_samples):
    """vamp.<robot>.roadmap(start, goal, environment, settings, rng) (bindings/common.hh:312-321,667):
    the vertex sequence, the adjacency lists, iterations (= draws + 1, prm.hh:235,292) and the rng's
    advance equal the reference loop restated over the oracle, whichever limit ends it."""
    rng = np.random.default_rng(31)
    oenv = random_scene(oracle, rng, 3, 3, 2)
    env = gpu_env_from_oracle(vamp, oenv)
    robot = vamp.panda_0_0
    pool = oracle.scale(rng.random((64, 7), dtype=F))
    pv = oracle.fkcc_threads(oenv, pool)
    s, g = pool[pv][0], pool[pv][1]
    settings = vamp.PRMSettings(vamp.PRMNeighborParams(7, robot.space_measure()))
    settings.max_iterations, settings.max_samples = max_iterations, max_samples
    h = robot.halton()
    h.skip(10)  # draws 11 ..
    rm = robot.roadmap(s, g, env, settings, h)
    q = oracle.scale(oracle.halton(7, range(11, 11 + max_iterations)))
    ok = oracle.fkcc_threads(oenv, q)
    want = np.concatenate([s[None], g[None], q[ok]])[:max_samples]
    assert np.array_equal(rm.vertices, want) and len(rm) == len(want)
    taken = int(np.nonzero(ok)[0][max_samples - 3]) + 1 if ok.sum() >= max_samples - 2 else max_iterations
    assert h.index == 11 + taken and rm.iterations == taken + 1
    edges, _ = oracle.build_roadmap_edges("panda", oenv, want)
    assert rm.edges == edges
    assert rm.nanoseconds > 0 and np.array_equal(rm[5], want[5])


def _query_order_pairs(n, m, seed):
    """valid (vertex i, neighbour j < i) pairs in build_roadmap's query order: i ascending"""
    rng = np.random.default_rng(seed)
    i = np.sort(rng.integers(1, n, m)).astype(np.uint32) if n > 1 else np.zeros(0, np.uint32)
    j = (rng.random(len(i)) * i).astype(np.uint32)
    return np.stack([i, j], 1).astype(np.uint32)


@pytest.mark.parametrize("n,m", [(1, 0), (2, 1), (1000, 0), (1000, 5000), (300000, 2000000)])
def test_roadmap_assemble_device_equals_host(vamp, n, m):
    """vgpu_roadmap_assemble_device (vgpu_roadmap_assemble.hip: stable radix sort of the expanded pairs,
    atomicMin hooking + pointer jumping) == the host assembly: offsets, append-order adjacency and
    components (smallest index), including isolated vertices and repeated pairs."""
    import torch
    from vamp_amd import roadmap
    pairs = _query_order_pairs(n, m, 5 + n)
    if m > 10:
        pairs[5] = pairs[4]  # a repeated pair
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    tp = torch.from_numpy(pairs.view(np.int32)).to(dev).reshape(-1, 2)
    off, adj, comp = roadmap.assemble_device(torch, n, tp, ctx)
    torch.cuda.synchronize()
    ho, ha, hc = roadmap.assemble(n, pairs)
    assert np.array_equal(off.cpu().numpy(), ho)
    assert np.array_equal(adj.cpu().numpy().view(np.uint32), ha)
    assert np.array_equal(comp.cpu().numpy().view(np.uint32), hc)


def test_roadmap_assemble_device_rejects_bad_index(vamp):
    import torch
    from vamp_amd import roadmap
    from vamp_amd._lib import VgpuError
    dev = torch.device("cuda", 0)
    ctx = vamp.context(0)
    tp = torch.tensor([[1, 0], [7, 2]], dtype=torch.int32, device=dev)
    with pytest.raises(VgpuError):
        roadmap.assemble_device(torch, 5, tp, ctx)
