"""The point-cloud filter restated (collision/filter.hh:101-268), SURVEY §8f rank 4.

Pins: the Morton encoder against entries of the reference's own lookup tables
(MORTON_LUT_{X,Y,Z}_256, filter.hh:17-100) and against its table-driven encoder morton_lut
(filter.hh:106-121), which the reference treats as interchangeable with morton_pdep; the
filter loop against an independent pure-Python restatement on small clouds. filter.hh
includes pdqsort.h (a CPM download absent here), so the reference filter itself cannot be
compiled in oracle/_ref: the order among equal Morton codes (pdqsort_branchless is unstable)
is parity unpinned and both restatements use a stable sort.
"""
import ctypes as C

import numpy as np

import oracle_py as O

F = np.float32

# filter.hh:17-100, a few entries of each table
LUT_KNOWN = {
    "x": {1: 0x1, 2: 0x8, 3: 0x9, 16: 0x1000, 255: 0x00249249},
    "y": {1: 0x2, 2: 0x10, 3: 0x12, 16: 0x2000, 255: 0x00492492},
    "z": {1: 0x4, 2: 0x20, 3: 0x24, 16: 0x4000, 255: 0x00924924},
}


def spread_byte(b, lane):
    return sum(((b >> i) & 1) << (3 * i + lane) for i in range(8))


def morton_lut(x, y, z):
    """morton_lut (filter.hh:106-121) over tables built by bit spreading."""
    ans = 0
    for i in range(4, 0, -1):
        s = (i - 1) * 8
        ans = ((ans << 24) & 0xFFFFFFFF) | (spread_byte((z >> s) & 0xFF, 2) | spread_byte((y >> s) & 0xFF, 1)
                                           | spread_byte((x >> s) & 0xFF, 0))
    return ans


def test_lut_known_answers():
    for lane, axis in enumerate("xyz"):
        for b, v in LUT_KNOWN[axis].items():
            assert spread_byte(b, lane) == v
            args = [0, 0, 0]
            args[lane] = b
            assert O.morton_encode(*args) == v


def test_morton_pdep_equals_lut():
    rng = np.random.default_rng(0)
    for x, y, z in rng.integers(0, 1024, size=(2000, 3)):
        assert O.morton_encode(int(x), int(y), int(z)) == morton_lut(int(x), int(y), int(z))
    assert O.morton_encode(1023, 1023, 1023) == morton_lut(1023, 1023, 1023)


def test_remap_point_wraps_like_x86():
    assert O.remap_point(F(0.5), F(0.0), F(1.0)) == 500
    assert O.remap_point(F(1.0), F(0.0), F(1.0)) == 1000
    assert O.remap_point(F(-0.5), F(0.0), F(1.0)) == 2**32 - 500  # cvttss2si 64-bit, low word
    assert O.remap_point(F(np.nan), F(0.0), F(1.0)) == 0


def sql2(a, b):
    L = O.lib()
    L.vo_sql2_3.restype = C.c_float
    L.vo_sql2_3.argtypes = [C.c_float] * 6
    return F(L.vo_sql2_3(*(float(v) for v in a), *(float(v) for v in b)))


def filter_py(pc, min_dist, max_range, origin, wmin, wmax, cull):
    """Independent restatement of filter.hh:175-268 (stable sort on ties)."""
    n = len(pc)
    if n == 0:
        return []
    sqd, sqr = F(min_dist) * F(min_dist), F(max_range) * F(max_range)
    mn = min(F(o) - F(max_range) for o in origin)
    mx = min(F(o) + F(max_range) for o in origin)
    idx = [0] * n
    hi = 0
    for i, p in enumerate(pc):
        if not cull or (sql2(p, origin) < sqr and all(wmin[k] <= p[k] <= wmax[k] for k in range(3))):
            idx[hi] = i
            hi += 1
    for perm in [(0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1), (2, 1, 0)]:
        nmn, nmx = mx, mn
        keyed = []
        for i in idx:
            p = pc[i]
            c = [O.remap_point(p[k], mn, mx) for k in perm]
            nmn = min(nmn, F(p.min()))
            nmx = max(nmx, F(p.max()))
            keyed.append((O.morton_encode(*c), i))
        keyed.sort(key=lambda t: t[0])
        kept = [keyed[0][1]]
        for _, i in keyed[1:]:
            if sql2(pc[i], pc[kept[-1]]) > sqd:
                kept.append(i)
        idx = kept
        mx = F((float(nmx + mx)) / 2.0)
        mn = F((float(nmn + mn)) / 2.0)
    return idx


def cloud(seed, n):
    rng = np.random.default_rng(seed)
    return rng.uniform(-1.0, 1.0, size=(n, 3)).astype(F)


def test_filter_matches_python_restatement():
    for seed, n, md, cull in [(0, 200, 0.05, True), (1, 300, 0.1, False), (2, 150, 0.2, True), (3, 64, 0.0, False)]:
        pc = cloud(seed, n)
        args = (md, 1.2, [0.1, -0.1, 0.0], [-0.9, -0.9, -0.9], [0.9, 0.9, 0.9], cull)
        got = O.filter_pointcloud(pc, *args)
        assert list(got) == filter_py(pc, *args)


def test_filter_empty_and_zero_distance():
    assert O.filter_pointcloud(np.zeros((0, 3), F), 0.1, 1.0, [0, 0, 0], [-1] * 3, [1] * 3).size == 0
    pc = cloud(4, 500)
    got = O.filter_pointcloud(pc, 0.0, 10.0, [0, 0, 0], [-1] * 3, [1] * 3, cull=False)
    assert sorted(got) == list(range(500))  # distinct points, min_dist 0: nothing removed


def test_filter_adjacent_spacing_and_cull_quirk():
    pc = cloud(5, 4000)
    pc[0] = [5.0, 5.0, 5.0]  # outside the range: culled, but the tail entries name point 0
    got = O.filter_pointcloud(pc, 0.05, 1.0, [0, 0, 0], [-1] * 3, [1] * 3, cull=True)
    assert 0 in got  # reference quirk (filter.hh:194-214): the unfilled Morton tail is point 0
    for a, b in zip(got[:-1], got[1:]):  # final pass keeps each point only past the last kept one
        assert sql2(pc[b], pc[a]) > F(0.05) * F(0.05)
    kept = got[got != 0]
    assert np.all(np.einsum("ij,ij->i", pc[kept], pc[kept]) < 1.0)
