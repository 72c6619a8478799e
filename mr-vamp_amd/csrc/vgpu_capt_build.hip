// vgpu_capt_build.hip -- CAPT construction on the device (collision/capt.hh:137-398; SURVEY §8f
// rank 4, second half).  The output arrays are those of the host build (vgpu_capt.cpp) bit for
// bit: the same (coordinate, point index) order inside every node, the same median tests, the same
// affordance lists in the same order (inherited candidates first, then the new run, with the
// reference's walk-from-the-bottom quirk of capt.hh:258-270), the same leaf boxes and packing.
//
// The recursion is run level by level over the whole point set (one level = every node of one
// depth, the nodes being contiguous segments of one permutation):
//   sort      two stable radix sorts per level: (segment, index) then (segment, key(coordinate)),
//             i.e. every segment ordered by (coordinate, index) like the host comparator;
//   tests     one thread per node: (float)((double)(a + b) / 2) of the two middle coordinates;
//   lists     one wave per node: the children's affordance lists (ballot-compacted in order) --
//             a count kernel, a scan, a fill kernel (CSR per level);
//   leaves    one wave per leaf: the cell from its ancestors' tests, the representative, the
//             affordance filter (distance to the cell, internal-ball skip), the leaf box, the
//             8-wide +inf-padded vectors; count, scan (= aff_starts), fill.
// Every selection runs in list order, so the packing equals the sequential build's.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <limits>
#include <vector>

#include <hip/hip_runtime.h>

#include "vgpu_capt.hh"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vgpu_capt_build.hip: the per-node waves assume wave64 gfx950"
#endif

namespace vgpu {
namespace captdev {

constexpr int kWave = 64;
constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t ord_key(float v)
{
    if (v == 0.0f) v = 0.0f;  // -0 == +0 for the host comparator
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void pad_kernel(const float* __restrict__ pts, size_t n, size_t m, float* __restrict__ P,
                           uint32_t* __restrict__ ord)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    const float inf = __builtin_inff();
    for (int k = 0; k < 3; ++k) P[3 * i + k] = i < n ? pts[3 * i + k] : inf;
    ord[i] = (uint32_t)i;
}

__global__ void key_index_kernel(const uint32_t* __restrict__ ord, size_t m, int seg_log2,
                                 uint64_t* __restrict__ key)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    key[i] = ((uint64_t)(i >> seg_log2) << 32) | ord[i];
}

__global__ void split_keys_kernel(const uint64_t* __restrict__ sorted, size_t m, int seg_log2, int axis,
                                  const float* __restrict__ P, uint32_t* __restrict__ ord,
                                  uint64_t* __restrict__ key)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    const uint32_t id = (uint32_t)sorted[i];
    ord[i] = id;
    key[i] = ((uint64_t)(i >> seg_log2) << 32) | ord_key(P[3 * (size_t)id + axis]);
}

// median_partition (capt.hh:137-154): the float sum of the middle pair, halved in double
__global__ void tests_kernel(const uint32_t* __restrict__ ord, const float* __restrict__ P, uint32_t nodes,
                             uint32_t seg, int axis, float* __restrict__ tests_level)
{
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= nodes) return;
    const size_t mid = (size_t)s * seg + seg / 2;
    const float a = P[3 * (size_t)ord[mid - 1] + axis], b = P[3 * (size_t)ord[mid] + axis];
    tests_level[s] = (float)((double)(a + b) / 2.0);
}

// order-preserving wave compaction: positions of the lanes with `pred` among the wave's
__device__ __forceinline__ uint32_t rank_of(uint64_t ballot)
{
    const uint32_t lane = __lane_id();
    return (uint32_t)__builtin_popcountll(ballot & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
}

// the children's lists of one node (capt.hh:245-280).  mode 0 counts, mode 1 writes.
template <int MODE>
__global__ __launch_bounds__(kBlock) void lists_kernel(const uint32_t* __restrict__ ord,
                                                       const float* __restrict__ P, uint32_t nodes, uint32_t seg,
                                                       int axis, const float* __restrict__ tests_level, float r_max,
                                                       const uint32_t* __restrict__ cur_off,
                                                       const uint32_t* __restrict__ cur_ids,
                                                       uint32_t* __restrict__ next_cnt,
                                                       const uint32_t* __restrict__ next_off,
                                                       uint32_t* __restrict__ next_ids)
{
    const uint32_t s = blockIdx.x * (kBlock / kWave) + (threadIdx.x / kWave);
    if (s >= nodes) return;  // wave-uniform
    const uint32_t lane = __lane_id();
    const float test = tests_level[s];
    const float hi_lim = test + r_max, lo_lim = test - r_max;
    const size_t begin = (size_t)s * seg, mid = begin + seg / 2, end = begin + seg;
    const uint32_t p0 = cur_off[s], p1 = cur_off[s + 1];
    uint32_t lo_w = 0, hi_w = 0;  // written so far
    const uint32_t lo_base = MODE ? next_off[2 * s] : 0u, hi_base = MODE ? next_off[2 * s + 1] : 0u;
    // inherited candidates, in list order
    for (uint32_t j0 = p0; j0 < p1; j0 += kWave) {
        const uint32_t j = j0 + lane;
        uint32_t id = 0;
        float c = 0.0f;
        if (j < p1) {
            id = cur_ids[j];
            c = P[3 * (size_t)id + axis];
        }
        const uint64_t bl = __builtin_amdgcn_ballot_w64(j < p1 && c <= hi_lim);
        const uint64_t bh = __builtin_amdgcn_ballot_w64(j < p1 && c >= lo_lim);
        if (MODE) {
            if ((bl >> lane) & 1u) next_ids[lo_base + lo_w + rank_of(bl)] = id;
            if ((bh >> lane) & 1u) next_ids[hi_base + hi_w + rank_of(bh)] = id;
        }
        lo_w += (uint32_t)__builtin_popcountll(bl);
        hi_w += (uint32_t)__builtin_popcountll(bh);
    }
    // new candidates: the high half from the median up while <= hi_lim (a prefix: sorted), to
    // the low child; the low half from its BOTTOM up while >= lo_lim, to the high child
    for (size_t k0 = mid; k0 < end; k0 += kWave) {
        const size_t k = k0 + lane;
        uint32_t id = 0;
        float c = __builtin_inff();
        if (k < end) {
            id = ord[k];
            c = P[3 * (size_t)id + axis];
        }
        const uint64_t b = __builtin_amdgcn_ballot_w64(k < end && c <= hi_lim && __builtin_isfinite(c));
        if (MODE && ((b >> lane) & 1u)) next_ids[lo_base + lo_w + rank_of(b)] = id;
        lo_w += (uint32_t)__builtin_popcountll(b);
        if (b != __builtin_amdgcn_ballot_w64(k < end)) break;  // the walk stopped in this chunk
    }
    const float c_first = P[3 * (size_t)ord[begin] + axis];
    if (c_first >= lo_lim) {
        for (size_t k0 = begin; k0 < mid; k0 += kWave) {
            const size_t k = k0 + lane;
            uint32_t id = 0;
            float c = __builtin_inff();
            if (k < mid) {
                id = ord[k];
                c = P[3 * (size_t)id + axis];
            }
            const uint64_t b = __builtin_amdgcn_ballot_w64(k < mid && c >= lo_lim && __builtin_isfinite(c));
            if (MODE && ((b >> lane) & 1u)) next_ids[hi_base + hi_w + rank_of(b)] = id;
            hi_w += (uint32_t)__builtin_popcountll(b);
            if (b != __builtin_amdgcn_ballot_w64(k < mid)) break;
        }
    }
    if (!MODE && lane == 0) {
        next_cnt[2 * s] = lo_w;
        next_cnt[2 * s + 1] = hi_w;
    }
}

// Volume::extend (capt.hh:60-68) is std::min / std::max in list order: strict comparisons, so of
// equal values (+0 / -0) the one met first stays.  Wave reductions carry the list position to
// keep exactly that one.
__device__ __forceinline__ void keep_min(float& v, int& i, float v2, int i2)
{
    if (v2 < v || (v2 == v && i2 < i)) v = v2, i = i2;
}
__device__ __forceinline__ void keep_max(float& v, int& i, float v2, int i2)
{
    if (v < v2 || (v2 == v && i2 < i)) v = v2, i = i2;
}

struct Cell {
    float lo[3], up[3];
};

__device__ __forceinline__ Cell leaf_cell(uint32_t s, int nlog2, const float* __restrict__ tests)
{
    const float inf = __builtin_inff();
    Cell c{{-inf, -inf, -inf}, {inf, inf, inf}};
    for (int l = 0; l < nlog2; ++l) {
        const uint32_t node = s >> (nlog2 - l);
        const uint32_t hi = (s >> (nlog2 - 1 - l)) & 1u;
        const float t = tests[((1u << l) - 1u) + node];
        if (hi) c.lo[l % 3] = t;
        else c.up[l % 3] = t;
    }
    return c;
}

// Volume::distsq_to (capt.hh:79-86) and contained_by_internal_ball (capt.hh:70-77) in the
// reference release build's contraction (vgpu_capt.cpp)
__device__ __forceinline__ float cell_dist2(const Cell& c, const float* p)
{
    float d[3];
    for (int k = 0; k < 3; ++k) {
        const float cl = p[k] < c.lo[k] ? c.lo[k] : (c.up[k] < p[k] ? c.up[k] : p[k]);
        d[k] = p[k] - cl;
    }
    return __builtin_fmaf(d[2], d[2], __builtin_fmaf(d[0], d[0], d[1] * d[1]));
}

__device__ __forceinline__ bool cell_inside_ball(const Cell& c, const float* p, float r2)
{
    float d[3];
    for (int k = 0; k < 3; ++k) d[k] = fmaxf(p[k] - c.lo[k], c.up[k] - p[k]);
    return __builtin_fmaf(d[2], d[2], __builtin_fmaf(d[0], d[0], d[1] * d[1])) <= r2;
}

// leaves (capt.hh:284-398 via vgpu_capt.cpp leaf()): mode 0 counts 8-wide vectors, mode 1 writes
template <int MODE>
__global__ __launch_bounds__(kBlock) void leaves_kernel(const uint32_t* __restrict__ ord,
                                                        const float* __restrict__ P, uint32_t m, int nlog2,
                                                        const float* __restrict__ tests, float aff_l2,
                                                        float min_l2, const uint32_t* __restrict__ l_off,
                                                        const uint32_t* __restrict__ l_ids,
                                                        uint32_t* __restrict__ vec_cnt,
                                                        const uint32_t* __restrict__ aff_starts,
                                                        float* __restrict__ aabbs, float* __restrict__ aff)
{
    const uint32_t s = blockIdx.x * (kBlock / kWave) + (threadIdx.x / kWave);
    if (s >= m) return;  // wave-uniform
    const uint32_t lane = __lane_id();
    const float inf = __builtin_inff();
    const float* rep = &P[3 * (size_t)ord[s]];
    float lo[3] = {rep[0], rep[1], rep[2]}, up[3] = {rep[0], rep[1], rep[2]};
    int loi[3] = {-1, -1, -1}, upi[3] = {-1, -1, -1};  // list positions (the representative: -1)
    const bool finite = __builtin_isfinite(rep[0]);
    uint32_t n_sel = 0;
    if (finite) {
        const Cell cell = leaf_cell(s, nlog2, tests);
        float* out = MODE ? &aff[(size_t)aff_starts[s] * 24] : nullptr;
        if (MODE && lane == 0) out[0] = rep[0], out[8] = rep[1], out[16] = rep[2];  // the representative first
        if (!cell_inside_ball(cell, rep, min_l2)) {
            const uint32_t p0 = l_off[s], p1 = l_off[s + 1];
            for (uint32_t j0 = p0; j0 < p1; j0 += kWave) {
                const uint32_t j = j0 + lane;
                const float* q = nullptr;
                bool take = false;
                if (j < p1) {
                    q = &P[3 * (size_t)l_ids[j]];
                    take = cell_dist2(cell, q) <= aff_l2;
                }
                const uint64_t b = __builtin_amdgcn_ballot_w64(take);
                if (take) {
                    for (int k = 0; k < 3; ++k) keep_min(lo[k], loi[k], q[k], (int)j), keep_max(up[k], upi[k], q[k], (int)j);
                    if (MODE) {
                        const uint32_t e = 1u + n_sel + rank_of(b);
                        float* v = out + (size_t)(e / 8) * 24 + (e % 8);
                        v[0] = q[0], v[8] = q[1], v[16] = q[2];
                    }
                }
                n_sel += (uint32_t)__builtin_popcountll(b);
            }
        }
        if (MODE) {  // pad the last vector with +inf
            const uint32_t used = 1u + n_sel, total = (used + 7u) / 8u * 8u;
            for (uint32_t e = used + lane; e < total; e += kWave) {
                float* v = out + (size_t)(e / 8) * 24 + (e % 8);
                v[0] = v[8] = v[16] = inf;
            }
        }
    }
    if (!MODE) {
        if (lane == 0) vec_cnt[s] = finite ? (1u + n_sel + 7u) / 8u : 0u;
        return;
    }
    for (int k = 0; k < 3; ++k) {  // the leaf box over the wave, first-met value on ties
        for (int off = 32; off >= 1; off >>= 1) {
            keep_min(lo[k], loi[k], __shfl_xor(lo[k], off), __shfl_xor(loi[k], off));
            keep_max(up[k], upi[k], __shfl_xor(up[k], off), __shfl_xor(upi[k], off));
        }
    }
    if (lane == 0)
        for (int k = 0; k < 3; ++k) aabbs[6 * (size_t)s + k] = lo[k], aabbs[6 * (size_t)s + 3 + k] = up[k];
}

// aabb_top: Volume::extend over the finite leaf representatives in leaf order (vgpu_capt.cpp)
__global__ __launch_bounds__(kBlock) void top_kernel(const uint32_t* __restrict__ ord, const float* __restrict__ P,
                                                     uint32_t m, float* __restrict__ top)
{
    __shared__ float rv[6][kBlock];
    __shared__ int ri[6][kBlock];
    const float inf = __builtin_inff();
    float v[6] = {inf, inf, inf, -inf, -inf, -inf};
    int ix[6] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX, INT_MAX};
    for (uint32_t s = threadIdx.x; s < m; s += kBlock) {
        const float* p = &P[3 * (size_t)ord[s]];
        if (!__builtin_isfinite(p[0])) continue;
        for (int k = 0; k < 3; ++k) keep_min(v[k], ix[k], p[k], (int)s), keep_max(v[3 + k], ix[3 + k], p[k], (int)s);
    }
    for (int k = 0; k < 6; ++k) rv[k][threadIdx.x] = v[k], ri[k][threadIdx.x] = ix[k];
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int k = 0; k < 6; ++k) {
                float a = rv[k][threadIdx.x];
                int ai = ri[k][threadIdx.x];
                if (k < 3) keep_min(a, ai, rv[k][threadIdx.x + w], ri[k][threadIdx.x + w]);
                else keep_max(a, ai, rv[k][threadIdx.x + w], ri[k][threadIdx.x + w]);
                rv[k][threadIdx.x] = a, ri[k][threadIdx.x] = ai;
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) top[threadIdx.x] = rv[threadIdx.x][0];
}

}  // namespace captdev

#define CB_CHK(x)                                 \
    do {                                          \
        hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) {                   \
            err = e_;                             \
            goto done;                            \
        }                                         \
    } while (0)

static unsigned blocks_of(size_t threads) { return (unsigned)((threads + captdev::kBlock - 1) / captdev::kBlock); }

hipError_t capt_build_device(const float* pts, size_t n, float r_min, float r_max, float r_point, hipStream_t st,
                             CaptTree& t)
{
    using namespace captdev;
    hipError_t err = hipSuccess;
    t = CaptTree{};
    t.r_min = r_min, t.r_max = r_max, t.r_point = r_point;
    int nlog2 = 0;
    while (((size_t)1 << nlog2) < n) ++nlog2;
    t.nlog2 = nlog2;
    const size_t m = (size_t)1 << nlog2;
    const float l1 = r_max + r_point;
    const float aff_l2 = l1 * l1, min_l2 = (r_min + r_point) * (r_min + r_point);
    float *P = nullptr, *tests = nullptr, *aabbs = nullptr, *aff = nullptr, *top = nullptr;
    uint32_t *ord = nullptr, *cur_off = nullptr, *cur_ids = nullptr, *cnt = nullptr, *nxt_off = nullptr,
             *nxt_ids = nullptr, *aff_starts = nullptr, *ord2 = nullptr;  // ord2: the sorts' ping-pong twin of ord
    uint64_t *ka = nullptr, *kb = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0, cap_cur = 1, cap_nxt = 1;
    const auto t0 = std::chrono::steady_clock::now();
    if (n == 0) return hipErrorInvalidValue;
    CB_CHK(hipMalloc(&P, 3 * m * sizeof(float)));
    CB_CHK(hipMalloc(&ord, m * sizeof(uint32_t)));
    CB_CHK(hipMalloc(&ka, m * sizeof(uint64_t)));
    CB_CHK(hipMalloc(&kb, m * sizeof(uint64_t)));
    CB_CHK(hipMalloc(&tests, (m > 1 ? m - 1 : 1) * sizeof(float)));
    CB_CHK(hipMalloc(&cnt, (2 * m + 1) * sizeof(uint32_t)));
    CB_CHK(hipMalloc(&cur_off, (2 * m + 1) * sizeof(uint32_t)));
    CB_CHK(hipMalloc(&nxt_off, (2 * m + 1) * sizeof(uint32_t)));
    CB_CHK(hipMalloc(&cur_ids, cap_cur * sizeof(uint32_t)));
    CB_CHK(hipMalloc(&top, 6 * sizeof(float)));
    {
        size_t b1 = 0, b2 = 0;
        CB_CHK(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, ka, kb, (int)m, 0, 64, st));
        CB_CHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b2, ka, kb, ord, ord, (int)m, 0, 64, st));
        size_t b3 = 0;
        CB_CHK(hipcub::DeviceScan::ExclusiveSum(nullptr, b3, cnt, nxt_off, (int)(2 * m + 1), st));
        tmp_bytes = std::max(std::max(b1, b2), b3);
        CB_CHK(hipMalloc(&tmp, tmp_bytes));
    }
    {
        CB_CHK(hipMalloc(&ord2, m * sizeof(uint32_t)));
        hipLaunchKernelGGL(pad_kernel, dim3(blocks_of(m)), dim3(kBlock), 0, st, pts, n, m, P, ord);
        CB_CHK(hipGetLastError());
        CB_CHK(hipMemsetAsync(cur_off, 0, 2 * sizeof(uint32_t), st));  // the root's list is empty
        for (int l = 0; l < nlog2; ++l) {
            const int seg_log2 = nlog2 - l;
            const uint32_t nodes = 1u << l, seg = 1u << seg_log2;
            const int axis = l % 3;
            const int bits = 32 + l + 1;
            hipLaunchKernelGGL(key_index_kernel, dim3(blocks_of(m)), dim3(kBlock), 0, st, ord, m, seg_log2, ka);
            CB_CHK(hipGetLastError());
            size_t tb = tmp_bytes;
            CB_CHK(hipcub::DeviceRadixSort::SortKeys(tmp, tb, ka, kb, (int)m, 0, bits, st));
            hipLaunchKernelGGL(split_keys_kernel, dim3(blocks_of(m)), dim3(kBlock), 0, st, kb, m, seg_log2, axis, P,
                               ord, ka);
            CB_CHK(hipGetLastError());
            tb = tmp_bytes;
            CB_CHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, ka, kb, ord, ord2, (int)m, 0, bits, st));
            std::swap(ord, ord2);
            float* tl = tests + (nodes - 1);
            hipLaunchKernelGGL(tests_kernel, dim3(blocks_of(nodes)), dim3(kBlock), 0, st, ord, P, nodes, seg, axis, tl);
            CB_CHK(hipGetLastError());
            const unsigned wblocks = (unsigned)((nodes + (kBlock / kWave) - 1) / (kBlock / kWave));
            hipLaunchKernelGGL((lists_kernel<0>), dim3(wblocks), dim3(kBlock), 0, st, ord, P, nodes, seg, axis, tl,
                               r_max, cur_off, cur_ids, cnt, nullptr, nullptr);
            CB_CHK(hipGetLastError());
            CB_CHK(hipMemsetAsync(cnt + 2 * nodes, 0, sizeof(uint32_t), st));
            tb = tmp_bytes;
            CB_CHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, nxt_off, (int)(2 * nodes + 1), st));
            uint32_t total = 0;
            CB_CHK(hipMemcpyAsync(&total, nxt_off + 2 * nodes, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
            CB_CHK(hipStreamSynchronize(st));
            if (total + 1 > cap_nxt || !nxt_ids) {
                if (nxt_ids) CB_CHK(hipFree(nxt_ids));
                cap_nxt = std::max<size_t>(total + 1, 2 * cap_nxt);
                CB_CHK(hipMalloc(&nxt_ids, cap_nxt * sizeof(uint32_t)));
            }
            hipLaunchKernelGGL((lists_kernel<1>), dim3(wblocks), dim3(kBlock), 0, st, ord, P, nodes, seg, axis, tl,
                               r_max, cur_off, cur_ids, cnt, nxt_off, nxt_ids);
            CB_CHK(hipGetLastError());
            std::swap(cur_off, nxt_off);
            std::swap(cur_ids, nxt_ids);
            std::swap(cap_cur, cap_nxt);
        }
    }
    {
        // leaves: cur_off / cur_ids hold every leaf's affordance list
        CB_CHK(hipMalloc(&aabbs, 6 * m * sizeof(float)));
        CB_CHK(hipMalloc(&aff_starts, (m + 1) * sizeof(uint32_t)));
        const unsigned wblocks = (unsigned)((m + (kBlock / kWave) - 1) / (kBlock / kWave));
        hipLaunchKernelGGL((leaves_kernel<0>), dim3(wblocks), dim3(kBlock), 0, st, ord, P, (uint32_t)m, nlog2, tests,
                           aff_l2, min_l2, cur_off, cur_ids, cnt, nullptr, nullptr, nullptr);
        CB_CHK(hipGetLastError());
        CB_CHK(hipMemsetAsync(cnt + m, 0, sizeof(uint32_t), st));
        size_t tb = tmp_bytes;
        CB_CHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, aff_starts, (int)(m + 1), st));
        uint32_t n_vec = 0;
        CB_CHK(hipMemcpyAsync(&n_vec, aff_starts + m, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        CB_CHK(hipStreamSynchronize(st));
        CB_CHK(hipMalloc(&aff, std::max<size_t>(1, (size_t)n_vec * 24) * sizeof(float)));
        hipLaunchKernelGGL((leaves_kernel<1>), dim3(wblocks), dim3(kBlock), 0, st, ord, P, (uint32_t)m, nlog2, tests,
                           aff_l2, min_l2, cur_off, cur_ids, nullptr, aff_starts, aabbs, aff);
        CB_CHK(hipGetLastError());
        hipLaunchKernelGGL(top_kernel, dim3(1), dim3(kBlock), 0, st, ord, P, (uint32_t)m, top);
        CB_CHK(hipGetLastError());
        t.tests.resize(m - 1);
        t.aabbs.resize(6 * m);
        t.aff_starts.resize(m + 1);
        t.aff.resize((size_t)n_vec * 24);
        if (m > 1) CB_CHK(hipMemcpyAsync(t.tests.data(), tests, (m - 1) * sizeof(float), hipMemcpyDeviceToHost, st));
        CB_CHK(hipMemcpyAsync(t.aabbs.data(), aabbs, 6 * m * sizeof(float), hipMemcpyDeviceToHost, st));
        CB_CHK(hipMemcpyAsync(t.aff_starts.data(), aff_starts, (m + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        if (n_vec) CB_CHK(hipMemcpyAsync(t.aff.data(), aff, (size_t)n_vec * 24 * sizeof(float), hipMemcpyDeviceToHost, st));
        CB_CHK(hipMemcpyAsync(t.top, top, 6 * sizeof(float), hipMemcpyDeviceToHost, st));
        CB_CHK(hipStreamSynchronize(st));
    }
    t.build_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
done:
    (void)hipStreamSynchronize(st);
    for (void* p : {(void*)P, (void*)ord, (void*)ka, (void*)kb, (void*)tests, (void*)cnt, (void*)cur_off,
                    (void*)nxt_off, (void*)cur_ids, (void*)nxt_ids, (void*)aff_starts, (void*)aabbs, (void*)aff,
                    (void*)top, (void*)ord2, tmp})
        if (p) (void)hipFree(p);
    return err;
}

}  // namespace vgpu
