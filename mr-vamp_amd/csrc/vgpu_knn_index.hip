// vgpu_knn_index.hip -- the roadmap neighbour queries (planning/prm.hh:264-266, NN::nearest over
// vertices 0 .. i-1; nn.hh:89-95) through a spatial index, for roadmaps far beyond what the
// brute-force scan of vgpu_roadmap.hip reaches (BASELINE configs[3]: ~2.7M Fetch vertices; the
// brute force is O(n^2) pair tests).
//
// Index (rebuilt per call, all on the stream, no host sync):
//   1. per-dimension min/max of the vertices (block partials, one final block);
//   2. a Morton key per vertex: 64/dim bits per dimension, interleaved (dim 8: 8 bits each);
//   3. a stable radix sort of (key, vertex) -> perm (sorted position -> vertex);
//   4. tiles of 64 consecutive sorted positions: the tile's coordinates (row-major, vertex
//      order = sorted order), its axis-aligned box and its smallest vertex index.
// Query (default, group_kernel below): one wave per 4 consecutive sorted queries, lane = candidate,
// tiles culled per query through super-tile boxes -- MI355X, Fetch Halton vertices: 2.7M vertices
// 219 ms vs 5433 ms brute force (1400 ms with the 64-query waves), 100k 3.6 vs 11.8 ms
// (profiles/r03_knn_scale.log).
// Query (VAMP_AMD_KNN_GROUP=0, query_kernel): one wave = 64 queries consecutive in sorted order.  The wave
// visits the tiles outward from its own (home, home+1, home-1, ...) so its lists fill early;
// a tile is skipped when no lane can take anything from it: its smallest vertex index is not
// below the lane's vertex (the causal prefix), or the box's squared distance exceeds the lane's
// squared bound (k-th key or r) by more than a relative 1e-4 (the box bound is computed in
// another summation order than the candidate distance; float differences and squares are
// monotone, so the margin only has to cover the sum's rounding, <= 14 * 2^-24 relative).
// Candidates of a visited tile are held one per lane and broadcast with v_readlane; the test,
// the correctly rounded sqrt and the register top-K list are those of vgpu_roadmap.hip.
// Candidates arrive in tile order, not index order, so admission compares full keys (distance,
// index): the list ends as the k smallest keys of {j < i : d(i, j) <= r}, exactly the brute
// force's result (which scans in index order, where "strictly closer" is the same key order).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>

#include "vgpu_device.hh"

namespace vgpu {
namespace knnidx {

constexpr int kTile = 64;      // candidates per tile = one wave
constexpr int kQBlock = 256;   // four query waves per block
constexpr int kBuf = 8;        // buffered candidates per lane between insertion passes
constexpr int kMinMaxBlocks = 256;

template <int D>
constexpr int bits_per_dim() { return 64 / D; }

// l2_norm of a - b before its sqrt, in the AVX hsum order (vgpu_roadmap.hip config_sumsq)
template <int D>
__device__ __forceinline__ float sumsq(const float* a, const float* b)
{
    float v[D];
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = a[j] - b[j];
    float sq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float lo = j < D ? v[j < D ? j : 0] : 0.0f;
        if (D <= 8) {
            sq[j] = lo * lo;
        } else {
            const float hi = (j + 8 < D) ? v[(j + 8 < D) ? j + 8 : 0] : 0.0f;
            sq[j] = __builtin_fmaf(lo, lo, hi * hi);
        }
    }
    return ((sq[0] + sq[4]) + (sq[2] + sq[6])) + ((sq[1] + sq[5]) + (sq[3] + sq[7]));
}

template <int K>
__device__ __forceinline__ void list_insert(float (&bd)[K], uint32_t (&bi)[K], float cd, uint32_t ci)
{
#pragma unroll
    for (int m = 0; m < K; ++m) {
        const bool lt = cd < bd[m] || (cd == bd[m] && ci < bi[m]);
        const float td = bd[m];
        const uint32_t ti = bi[m];
        bd[m] = lt ? cd : td;
        bi[m] = lt ? ci : ti;
        cd = lt ? td : cd;
        ci = lt ? ti : ci;
    }
}

__device__ __forceinline__ float wave_min(float v)
{
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v)
{
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_umin(uint32_t v)
{
    for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// per-block partial min/max of every dimension: part[block][2D] = (min[D], max[D])
template <int D>
__global__ __launch_bounds__(256) void minmax_kernel(const float* __restrict__ V, uint32_t n, float* __restrict__ part)
{
    float lo[D], hi[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        lo[d] = __builtin_inff();
        hi[d] = -__builtin_inff();
    }
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float x = V[(size_t)i * D + d];
            lo[d] = fminf(lo[d], x);
            hi[d] = fmaxf(hi[d], x);
        }
    }
    __shared__ float s[4][2 * D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        lo[d] = wave_min(lo[d]);
        hi[d] = wave_max(hi[d]);
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            s[threadIdx.x >> 6][d] = lo[d];
            s[threadIdx.x >> 6][D + d] = hi[d];
        }
    }
    __syncthreads();
    if (threadIdx.x < 2 * D) {
        const int e = threadIdx.x;
        float v = s[0][e];
        for (int w = 1; w < 4; ++w) v = e < D ? fminf(v, s[w][e]) : fmaxf(v, s[w][e]);
        part[(size_t)blockIdx.x * 2 * D + e] = v;
    }
}

// ls[0..D) = per-dimension origin, ls[D..2D) = scale to [0, 2^B - 1] (0 for a flat or non-finite range)
template <int D>
__global__ __launch_bounds__(64) void scale_kernel(const float* __restrict__ part, uint32_t nparts, float* __restrict__ ls)
{
    const int d = threadIdx.x;
    if (d >= D) return;
    float lo = __builtin_inff(), hi = -__builtin_inff();
    for (uint32_t b = 0; b < nparts; ++b) {
        lo = fminf(lo, part[(size_t)b * 2 * D + d]);
        hi = fmaxf(hi, part[(size_t)b * 2 * D + D + d]);
    }
    const float top = (float)((1u << bits_per_dim<D>()) - 1u);
    const float span = hi - lo;
    const bool ok = span > 0.0f && span < __builtin_inff();
    ls[d] = ok ? lo : 0.0f;
    ls[D + d] = ok ? top / span : 0.0f;
}

template <int D>
__global__ __launch_bounds__(256) void key_kernel(const float* __restrict__ V, uint32_t n, const float* __restrict__ ls,
                                                  uint64_t* __restrict__ key, uint32_t* __restrict__ id)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    constexpr int B = bits_per_dim<D>();
    const float top = (float)((1u << B) - 1u);
    uint64_t k = 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float f = fminf(fmaxf((V[(size_t)i * D + d] - ls[d]) * ls[D + d], 0.0f), top);  // NaN -> 0
        const uint32_t q = (uint32_t)f;
#pragma unroll
        for (int b = 0; b < B; ++b) k |= (uint64_t)((q >> b) & 1u) << (b * D + d);
    }
    key[i] = k;
    id[i] = i;
}

// Candidate codes: each tile's coordinates quantised to 8 bits per dimension against the tile's own box,
// x' = fma(code, step, lo) with step = (hi - lo) / 255 -- D bytes per candidate instead of 4 D + 4, read for
// every candidate of a visited tile; the exact coordinates and vertex index are read only for the candidates
// whose coded distance can pass (group_kernel QC).  The tile header holds step[D] and delta, an upper bound of
// |x - x'| over the tile's candidates measured from the decoded values themselves (the same fma as the
// query side), so |d(q, x) - d(q, x')| <= delta exactly; the prefilter widens it further for the float
// rounding of both distance sums.
template <int D>
constexpr int code_words() { return (D + 3) / 4; }

// one wave per tile: sorted coordinates, the box and the smallest vertex index (+ the codes)
template <int D>
__global__ __launch_bounds__(64) void tile_kernel(const float* __restrict__ V, const uint32_t* __restrict__ perm,
                                                  uint32_t n, float* __restrict__ Vs, float* __restrict__ tbox,
                                                  uint32_t* __restrict__ tmin, uint32_t* __restrict__ qc,
                                                  float* __restrict__ qh)
{
    const uint32_t t = blockIdx.x;
    const uint32_t p = t * kTile + threadIdx.x;
    const bool ok = p < n;
    const uint32_t j = ok ? perm[p] : 0xFFFFFFFFu;
    float lo[D], hi[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float x = ok ? V[(size_t)j * D + d] : 0.0f;
        if (ok) Vs[(size_t)p * D + d] = x;
        lo[d] = wave_min(ok ? x : __builtin_inff());
        hi[d] = wave_max(ok ? x : -__builtin_inff());
    }
    const uint32_t jm = wave_umin(j);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            tbox[(size_t)t * 2 * D + d] = lo[d];
            tbox[(size_t)t * 2 * D + D + d] = hi[d];
        }
        tmin[t] = jm;
    }
    if (!qc) return;  // codes only for the coded group queries
    constexpr int W = code_words<D>();
    uint32_t word[W];
#pragma unroll
    for (int w = 0; w < W; ++w) word[w] = 0u;
    float e2 = 0.0f;
    float step[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float x = ok ? Vs[(size_t)p * D + d] : lo[d];
        float st = (hi[d] - lo[d]) * (1.0f / 255.0f);
        if (!(st > 0.0f && st < __builtin_inff())) st = 0.0f;
        step[d] = st;
        const float f = st > 0.0f ? fminf(fmaxf(__builtin_rintf((x - lo[d]) / st), 0.0f), 255.0f) : 0.0f;
        const uint32_t code = (uint32_t)f;
        word[d / 4] |= code << (8 * (d % 4));
        const float err = wave_max(ok ? __builtin_fabsf(x - __builtin_fmaf((float)code, st, lo[d])) : 0.0f);
        e2 = __builtin_fmaf(err, err, e2);
    }
#pragma unroll
    for (int w = 0; w < W; ++w) qc[((size_t)t * W + w) * kTile + threadIdx.x] = word[w];
    if (threadIdx.x == 0) {
#pragma unroll
        for (int d = 0; d < D; ++d) qh[(size_t)t * (D + 1) + d] = step[d];
        float delta = __builtin_sqrtf(e2) * 1.0001f;  // the sum's and sqrt's rounding (a few ulp) covered
        if (!(delta < __builtin_inff())) delta = __builtin_inff();  // NaN / inf coordinates: no prefilter
        qh[(size_t)t * (D + 1) + D] = delta;
    }
}

// sorted positions of the queries q_first .. q_end-1 (flag for the select)
__global__ __launch_bounds__(256) void qflag_kernel(const uint32_t* __restrict__ perm, uint32_t n, uint32_t q_first,
                                                    uint32_t q_end, uint8_t* __restrict__ flag)
{
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const uint32_t i = perm[p];
    flag[p] = (i >= q_first && i < q_end) ? 1 : 0;
}

__device__ __forceinline__ float bcast(float v, uint32_t lane)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)lane));
}
__device__ __forceinline__ uint32_t bcast(uint32_t v, uint32_t lane)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

template <int D, int K>
__global__ __launch_bounds__(kQBlock) void query_kernel(const float* __restrict__ Vs, const uint32_t* __restrict__ perm,
                                                        uint32_t n, uint32_t T, const float* __restrict__ tbox,
                                                        const uint32_t* __restrict__ tmin,
                                                        const uint32_t* __restrict__ qlist, uint32_t q_first,
                                                        uint32_t q_count, const uint32_t* __restrict__ kq,
                                                        const float* __restrict__ rq, uint32_t kmax,
                                                        uint32_t* __restrict__ nbr, float* __restrict__ dist,
                                                        uint32_t* __restrict__ cnt)
{
    __shared__ float buf_d[kBuf][kQBlock];
    __shared__ uint32_t buf_i[kBuf][kQBlock];
    const uint32_t wave = blockIdx.x * (kQBlock / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t slot = threadIdx.x;
    if (wave * 64 >= q_count) return;  // wave-uniform; the kernel has no block barrier
    const uint32_t qo = wave * 64 + lane;
    const bool inq = qo < q_count;
    const uint32_t p = inq ? (qlist ? qlist[qo] : qo) : 0u;
    const uint32_t i = inq ? perm[p] : 0xFFFFFFFFu;
    const bool live = inq && i >= 2;  // vertices 0, 1 (start, goal) query nothing (prm.hh:228-233)
    float me[D];
#pragma unroll
    for (int d = 0; d < D; ++d) me[d] = inq ? Vs[(size_t)p * D + d] : 0.0f;
    const uint32_t k = live ? min(kq[i], (uint32_t)K) : 0u;
    const float r = live ? rq[i] : -1.0f;
    float bd[K];
    uint32_t bi[K];
#pragma unroll
    for (int m = 0; m < K; ++m) {
        bd[m] = __builtin_inff();
        bi[m] = 0xFFFFFFFFu;
    }
    uint32_t c = 0, nb = 0;
    float worst = r;            // admission bound: r while fewer than k are held, else the k-th key
    uint32_t worst_i = 0xFFFFFFFFu;
    float thr = live && k ? r * r * 1.000001f : -1.0f;  // sqrt plausibility bound (vgpu_roadmap.hip)
    auto flush = [&]() {
        for (uint32_t m = 0; __builtin_amdgcn_ballot_w64(m < nb) != 0ull; ++m) {
            const bool has = m < nb;
            list_insert<K>(bd, bi, has ? buf_d[has ? m : 0][slot] : __builtin_inff(),
                           has ? buf_i[has ? m : 0][slot] : 0xFFFFFFFFu);
        }
        c = min(c + nb, k);
        nb = 0;
        float kth = r;
        uint32_t kth_i = 0xFFFFFFFFu;
#pragma unroll
        for (int m = 0; m < K; ++m)
            if ((uint32_t)m + 1 == k) {
                kth = bd[m];
                kth_i = bi[m];
            }
        worst = (c == k) ? kth : r;
        worst_i = (c == k) ? kth_i : 0xFFFFFFFFu;
        thr = live && k ? worst * worst * 1.000001f : -1.0f;
    };
    auto consider = [&](bool need, uint32_t j, float s) {
        const bool pre = need && j < i && s <= thr;
        if (__builtin_amdgcn_ballot_w64(pre) == 0ull) return;
        const float dd = __builtin_sqrtf(s);
        // nn query semantics: distance <= r; once k are held, only a smaller key displaces the k-th
        const bool take = pre && (c < k ? dd <= worst : (dd < worst || (dd == worst && j < worst_i)));
        if (take) {
            buf_d[nb][slot] = dd;
            buf_i[nb][slot] = j;
            ++nb;
        }
    };
    const uint32_t home = __builtin_amdgcn_readfirstlane(p) / kTile;
    for (uint32_t s = 0; s < 2 * T; ++s) {
        const int64_t t64 = (s & 1u) ? (int64_t)home + (int64_t)((s + 1) / 2) : (int64_t)home - (int64_t)(s / 2);
        if (t64 < 0 || t64 >= (int64_t)T) continue;
        const uint32_t t = (uint32_t)t64;
        const float* bx = tbox + (size_t)t * 2 * D;
        float lb = 0.0f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float g = fmaxf(fmaxf(bx[d] - me[d], me[d] - bx[D + d]), 0.0f);
            lb = __builtin_fmaf(g, g, lb);
        }
        const bool need = live && tmin[t] < i && lb <= thr * 1.0001f;
        if (__builtin_amdgcn_ballot_w64(need) == 0ull) continue;
        const uint32_t cp = t * kTile + lane;
        float cv[D];
#pragma unroll
        for (int d = 0; d < D; ++d) cv[d] = cp < n ? Vs[(size_t)cp * D + d] : 0.0f;
        const uint32_t cj = cp < n ? perm[cp] : 0xFFFFFFFFu;  // a missing candidate is never < i
        for (uint32_t u = 0; u < (uint32_t)kTile; u += 4) {
            float s4[4];
            uint32_t j4[4];
            bool any = false;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                float cc[D];
#pragma unroll
                for (int d = 0; d < D; ++d) cc[d] = bcast(cv[d], u + h);
                j4[h] = bcast(cj, u + h);
                s4[h] = sumsq<D>(cc, me);
                any |= need && j4[h] < i && s4[h] <= thr;
            }
            if (__builtin_amdgcn_ballot_w64(any) == 0ull) continue;
#pragma unroll
            for (int h = 0; h < 4; ++h) consider(need, j4[h], s4[h]);
            if (__builtin_amdgcn_ballot_w64(nb > kBuf - 4) != 0ull) flush();
        }
        if (__builtin_amdgcn_ballot_w64(nb != 0) != 0ull) flush();
    }
    if (inq) {
        const size_t o = (size_t)(i - q_first);
        cnt[o] = c;
#pragma unroll
        for (int m = 0; m < K; ++m) {
            if ((uint32_t)m < c) {
                nbr[o * kmax + m] = bi[m];
                dist[o * kmax + m] = bd[m];
            }
        }
    }
}

// ---- group queries (the default): one wave per kGroup consecutive sorted queries ----------------
// Each query's list lives across the wave (lane m holds its m-th key), candidates are one tile per
// visit (lane = candidate), and tiles are culled PER QUERY of the group through a two-level box
// hierarchy (super-tiles of kSuper tiles, then tiles): the 64-query waves above test every tile
// and visit any tile one of 64 queries needs, which in 8-D is most of them.  Visiting order: the
// home tile, the home super-tile, then the other super-tiles outward in chunks of 64 (one per
// lane); a super-tile / tile is visited only if some query of the group can take from it.
// Admission is the same full-key rule, so the lists are again exactly the brute force's.
constexpr int kSuper = 64;  // tiles per super-tile
// VGPU_KNN_ORDER bit 0: super-tiles visited nearest first (their box lower bound over the group's queries, one
// global order when S <= 64 * kKeySlots) instead of outward by index, each re-checked against the thresholds as
// they stand when its turn comes -- the lists tighten sooner, so fewer far tiles pass; bit 1: the same for the
// tiles inside a super-tile.  A/B on MI355X (profiles/r05l_ab.log, 2.68M vertices): 200 ms in index order, 214 ms
// with bit 0, 270 ms with both -- the selection's reductions and the key registers (57 -> 77 / 87 VGPRs: fewer
// waves) cost more than the tighter lists save; off.
#ifndef VGPU_KNN_ORDER
#define VGPU_KNN_ORDER 0
#endif
constexpr int kKeySlots = 16;
// candidate tiles held in registers per visit pipeline (2: one load in flight while a tile is tested; 3: two).
// A/B on MI355X (profiles/r05h_ab.log): 2.68M vertices 211 -> 195 ms, 100k 3.47 -> 3.23 ms with 3
#ifndef VGPU_KNN_DEPTH
#define VGPU_KNN_DEPTH 3
#endif

// one wave per super-tile: the box of its tiles' boxes and their smallest vertex index
template <int D>
__global__ __launch_bounds__(64) void super_kernel(const float* __restrict__ tbox, const uint32_t* __restrict__ tmin,
                                                   uint32_t T, float* __restrict__ sbox, uint32_t* __restrict__ smin)
{
    const uint32_t sp = blockIdx.x;
    const uint32_t t = sp * kSuper + threadIdx.x;
    const bool ok = t < T;
    float lo[D], hi[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        lo[d] = wave_min(ok ? tbox[(size_t)t * 2 * D + d] : __builtin_inff());
        hi[d] = wave_max(ok ? tbox[(size_t)t * 2 * D + D + d] : -__builtin_inff());
    }
    const uint32_t m = wave_umin(ok ? tmin[t] : 0xFFFFFFFFu);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            sbox[(size_t)sp * 2 * D + d] = lo[d];
            sbox[(size_t)sp * 2 * D + D + d] = hi[d];
        }
        smin[sp] = m;
    }
}

template <int D>
__device__ __forceinline__ float box_lb(const float* __restrict__ bx, const float* me)
{
    float lb = 0.0f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float g = fmaxf(fmaxf(bx[d] - me[d], me[d] - bx[D + d]), 0.0f);
        lb = __builtin_fmaf(g, g, lb);
    }
    return lb;
}

__device__ __forceinline__ float shfl_up1(float v) { return __shfl_up(v, 1, 64); }
__device__ __forceinline__ uint32_t shfl_up1(uint32_t v) { return (uint32_t)__shfl_up((int)v, 1, 64); }

// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share one,
// MI355X_MICROARCH.md "Workgroup dispatch"), so consecutive blocks -- neighbouring Morton-sorted query groups,
// which visit the same candidate tiles -- would pull the same tiles into 8 different L2s.  Renumbered, the
// blocks of one XCD take one contiguous run of query groups (a bijection of [0, nb) for any nb).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb)
{
    const uint32_t x = b & 7u, q = nb >> 3, r = nb & 7u;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// QC: candidates are first tested on their codes (tile_kernel) and only those that can pass for some query of
// the group read their exact coordinates and index -- the exact test and admission below are unchanged, so the
// lists are the same; the tiles' bytes per visit drop from 36 to D per candidate.  The codes of the next tile
// are in flight while the current one's exact candidates are tested.
template <int D, int QG, bool QC>
__global__ __launch_bounds__(kQBlock) void group_kernel(const float* __restrict__ Vs, const uint32_t* __restrict__ perm,
                                                        uint32_t n, uint32_t T, uint32_t S,
                                                        const float* __restrict__ tbox,
                                                        const uint32_t* __restrict__ tmin,
                                                        const float* __restrict__ sbox,
                                                        const uint32_t* __restrict__ smin,
                                                        const uint32_t* __restrict__ qc,
                                                        const float* __restrict__ qh,
                                                        const uint32_t* __restrict__ qlist, uint32_t q_first,
                                                        uint32_t q_count, const uint32_t* __restrict__ kq,
                                                        const float* __restrict__ rq, uint32_t kmax,
                                                        uint32_t* __restrict__ nbr, float* __restrict__ dist,
                                                        uint32_t* __restrict__ cnt, uint32_t* __restrict__ dbg)
{
    const uint32_t wave = xcd_block(blockIdx.x, gridDim.x) * (kQBlock / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t g0 = wave * QG;
    if (g0 >= q_count) return;  // wave-uniform; the kernel has no block barrier
    // the group's queries (wave-uniform values)
    uint32_t qi[QG], kk[QG], c[QG], wi[QG];
    float me[QG][D], wd[QG], thr[QG];
    uint32_t p0 = 0;
    // readfirstlane: the group's values are wave-uniform; kept in SGPRs they leave the VGPRs to the
    // candidates (occupancy) -- the compiler cannot prove the loads uniform by itself
    auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    auto unf = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const uint32_t qo = g0 + q;
        const bool inq = qo < q_count;
        const uint32_t p = uni(VGPU_DCLAMP(dbg, inq ? (qlist ? qlist[qo] : qo) : 0u, n, DBG_KNN_QUERY));
        if (q == 0) p0 = p;
        qi[q] = uni(inq ? VGPU_DCLAMP(dbg, perm[p], n, DBG_KNN_VERTEX) : 0xFFFFFFFFu);
        const bool live = inq && qi[q] >= 2;  // vertices 0, 1 (start, goal) query nothing (prm.hh:228-233)
#pragma unroll
        for (int d = 0; d < D; ++d) me[q][d] = unf(inq ? Vs[(size_t)p * D + d] : 0.0f);
        kk[q] = uni(live ? min(kq[qi[q]], 64u) : 0u);
        wd[q] = unf(live ? rq[qi[q]] : -1.0f);  // admission bound: r while fewer than k are held, else the k-th key
        wi[q] = 0xFFFFFFFFu;
        c[q] = 0;
        thr[q] = (live && kk[q]) ? wd[q] * wd[q] * 1.000001f : -1.0f;
    }
    // lane m holds key m of each query's list, ascending
    float bd[QG];
    uint32_t bi[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        bd[q] = __builtin_inff();
        bi[q] = 0xFFFFFFFFu;
    }
    struct Cand {
        float v[D];
        uint32_t j;
        bool live;  // wave-uniform: some lane holds a candidate
    };
    auto load = [&](uint32_t t, Cand& cd) {
        t = VGPU_DCLAMP(dbg, t, T, DBG_KNN_TILE);
        const uint32_t cp = t * kTile + lane;
        const bool ok = cp < n;
#pragma unroll
        for (int d = 0; d < D; ++d) cd.v[d] = ok ? Vs[(size_t)cp * D + d] : 0.0f;
        cd.j = ok ? perm[cp] : 0xFFFFFFFFu;  // a missing candidate is never < i
        cd.live = true;
    };
    constexpr int W = code_words<D>();
    struct Codes {
        uint32_t w[W];
    };
    auto load_codes = [&](uint32_t t, Codes& cc) {
        t = VGPU_DCLAMP(dbg, t, T, DBG_KNN_TILE);
#pragma unroll
        for (int w = 0; w < W; ++w) cc.w[w] = qc[((size_t)t * W + w) * kTile + lane];
    };
    // coded distances of tile t's candidates; exact coordinates and index only where some query can take one
    // (its threshold now -- thresholds only shrink, so a later test is no looser)
    auto refine = [&](uint32_t t, const Codes& cc, Cand& cd) {
        t = VGPU_DCLAMP(dbg, t, T, DBG_KNN_TILE);
        const float* __restrict__ h = qh + (size_t)t * (D + 1);
        const float* __restrict__ bx = tbox + (size_t)t * 2 * D;
        float xa[D];
#pragma unroll
        for (int d = 0; d < D; ++d)
            xa[d] = __builtin_fmaf((float)((cc.w[d / 4] >> (8 * (d % 4))) & 0xFFu), h[d], bx[d]);
        const float delta = h[D];
        bool pass = false;
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            // |x - me| <= |x' - me| + delta; thr >= s_exact implies |x - me| <= sqrt(thr) (1 + 2^-23); the
            // coded sum's own rounding (< 1e-6 relative) is covered by the last factor.  A dead query
            // (thr = -1) gives NaN: never passes.
            const float b = __builtin_sqrtf(thr[q]) * 1.000002f + delta;
            pass |= sumsq<D>(xa, me[q]) <= b * b * 1.00001f;
        }
        const uint32_t cp = t * kTile + lane;
        const bool ok = pass && cp < n;
#pragma unroll
        for (int d = 0; d < D; ++d) cd.v[d] = ok ? Vs[(size_t)cp * D + d] : 0.0f;
        cd.j = ok ? perm[cp] : 0xFFFFFFFFu;
        cd.live = __builtin_amdgcn_ballot_w64(ok) != 0ull;
    };
    auto consider = [&](const Cand& cd) {
        const float* cv = cd.v;
        const uint32_t cj = cd.j;
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const float s = sumsq<D>(cv, me[q]);
            uint64_t m = __builtin_amdgcn_ballot_w64(cj < qi[q] && s <= thr[q]);
            if (m == 0ull) continue;
            const float dl = __builtin_sqrtf(s);
            while (m) {
                const uint32_t b = (uint32_t)__builtin_ctzll(m);
                m &= m - 1ull;
                const float d = bcast(dl, b);
                const uint32_t j = bcast(cj, b);
                // nn query semantics: distance <= r; once k are held, only a smaller key displaces the k-th
                const bool take = c[q] < kk[q] ? d <= wd[q] : (d < wd[q] || (d == wd[q] && j < wi[q]));
                if (!take) continue;
                // every lane shuffles (a lane masked off by a short-circuit would not be read back)
                const uint32_t lt = (d < bd[q] || (d == bd[q] && j < bi[q])) ? 1u : 0u;
                const float pd = shfl_up1(bd[q]);
                const uint32_t pi = shfl_up1(bi[q]);
                const uint32_t plt_raw = shfl_up1(lt);
                const bool plt = lane > 0 && plt_raw != 0u;
                bd[q] = lt ? (plt ? pd : d) : bd[q];
                bi[q] = lt ? (plt ? pi : j) : bi[q];
                c[q] = min(c[q] + 1u, kk[q]);
                if (c[q] == kk[q]) {
                    wd[q] = bcast(bd[q], kk[q] - 1u);
                    wi[q] = bcast(bi[q], kk[q] - 1u);
                    thr[q] = wd[q] * wd[q] * 1.000001f;
                }
            }
        }
    };
    // does some query of the group need the box (smallest index mn)?
    auto need_box = [&](const float* __restrict__ bx, uint32_t mn) {
        bool need = false;
#pragma unroll
        for (int q = 0; q < QG; ++q) need |= mn < qi[q] && box_lb<D>(bx, me[q]) <= thr[q] * 1.0001f;
        return need;
    };
    // all needed tiles of super-tile sp except `skip`, the next tile's candidates loaded while the
    // current one is tested
    auto visit_super = [&](uint32_t sp, uint32_t skip) {
        sp = VGPU_DCLAMP(dbg, sp, S, DBG_KNN_SUPER);
        const uint32_t t = sp * kSuper + lane;
        if constexpr ((VGPU_KNN_ORDER & 2) && !QC) {
            // this lane's tile: its box lower bound per query (need = some query could take from it)
            float lbq[QG];
            float key = __builtin_inff();
            const bool ok = t < T && t != skip;
            const uint32_t mn = ok ? tmin[t] : 0u;
#pragma unroll
            for (int q = 0; q < QG; ++q) {
                lbq[q] = ok ? box_lb<D>(tbox + (size_t)t * 2 * D, me[q]) : __builtin_inff();
                if (mn < qi[q] && lbq[q] <= thr[q] * 1.0001f) key = fminf(key, lbq[q]);
            }
            uint64_t m = __builtin_amdgcn_ballot_w64(key < __builtin_inff());
            // the needed tile with the least bound, still needed under the current thresholds (0xFFFFFFFF: none)
            auto pick = [&]() -> uint32_t {
                bool still = false;
#pragma unroll
                for (int q = 0; q < QG; ++q) still |= mn < qi[q] && lbq[q] <= thr[q] * 1.0001f;
                m &= __builtin_amdgcn_ballot_w64(still);
                if (m == 0ull) return 0xFFFFFFFFu;
                const float k = ((m >> lane) & 1ull) ? key : __builtin_inff();
                const float kmin = wave_min(k);
                const uint32_t sel = (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(k == kmin) & m);
                m &= ~(1ull << sel);
                return sel;
            };
            Cand a, b, c;
            bool ha, hb, hc;
            auto next = [&](Cand& x, bool& h) {
                const uint32_t sel = pick();
                h = sel != 0xFFFFFFFFu;
                if (h) load(sp * kSuper + sel, x);
            };
            next(a, ha);
            next(b, hb);
            for (;;) {
                next(c, hc);
                if (!ha) break;
                consider(a);
                next(a, ha);
                if (!hb) break;
                consider(b);
                next(b, hb);
                if (!hc) break;
                consider(c);
            }
            return;
        }
        const bool need = t < T && t != skip && need_box(tbox + (size_t)t * 2 * D, tmin[t]);
        uint64_t m = __builtin_amdgcn_ballot_w64(need);
        if (m == 0ull) return;
        if constexpr (QC) {
            // two stages in flight: the next tile's codes while this tile's exact candidates are tested
            uint32_t t1 = sp * kSuper + (uint32_t)__builtin_ctzll(m);
            m &= m - 1ull;
            Codes c1;
            load_codes(t1, c1);
            Cand cur;
            refine(t1, c1, cur);
            bool has1 = m != 0ull;
            if (has1) {
                t1 = sp * kSuper + (uint32_t)__builtin_ctzll(m);
                m &= m - 1ull;
                load_codes(t1, c1);
            }
            for (;;) {
                Cand nxt;
                const bool hasn = has1;
                if (hasn) refine(t1, c1, nxt);
                has1 = m != 0ull;
                if (has1) {
                    t1 = sp * kSuper + (uint32_t)__builtin_ctzll(m);
                    m &= m - 1ull;
                    load_codes(t1, c1);
                }
                if (cur.live) consider(cur);
                if (!hasn) break;
                cur = nxt;
            }
        } else if constexpr (VGPU_KNN_DEPTH >= 3) {
            // three tiles in registers: two loads in flight while one is tested (slots rotate a, b, c)
            Cand a, b, c;
            bool ha, hb, hc;
            auto next = [&](Cand& x, bool& h) {
                h = m != 0ull;
                if (h) {
                    load(sp * kSuper + (uint32_t)__builtin_ctzll(m), x);
                    m &= m - 1ull;
                }
            };
            next(a, ha);
            next(b, hb);
            for (;;) {
                next(c, hc);
                if (!ha) break;
                consider(a);
                next(a, ha);
                if (!hb) break;
                consider(b);
                next(b, hb);
                if (!hc) break;
                consider(c);
            }
        } else {
            Cand cur, nxt;
            load(sp * kSuper + (uint32_t)__builtin_ctzll(m), cur);
            m &= m - 1ull;
            for (;;) {
                const bool more = m != 0ull;
                if (more) load(sp * kSuper + (uint32_t)__builtin_ctzll(m), nxt);
                consider(cur);
                if (!more) break;
                m &= m - 1ull;
                cur = nxt;
            }
        }
    };
    const uint32_t home_t = p0 / kTile, home_s = home_t / kSuper;
    {
        Cand h;
        load(home_t, h);
        consider(h);
    }
    visit_super(home_s, home_t);
    if constexpr ((VGPU_KNN_ORDER & 1) && !QC) {
        if (S <= 64u * kKeySlots) {
            // every super-tile's bound (lane + 64 j) into this wave's LDS row, the lane's least one in registers;
            // then the wave's least first, each re-checked when its turn comes
            __shared__ float skey[kQBlock / 64][64 * kKeySlots];
            float* row = skey[threadIdx.x >> 6];
            float kl = __builtin_inff();
            uint32_t jl = 0;
            for (uint32_t j = 0; j < (uint32_t)kKeySlots; ++j) {
                const uint32_t sp = lane + 64u * j;
                float k = __builtin_inff();
                if (sp < S && sp != home_s) {
                    const float* bx = sbox + (size_t)sp * 2 * D;
                    const uint32_t mn = smin[sp];
#pragma unroll
                    for (int q = 0; q < QG; ++q) {
                        const float lb = box_lb<D>(bx, me[q]);
                        if (mn < qi[q] && lb <= thr[q] * 1.0001f) k = fminf(k, lb);
                    }
                }
                row[sp] = k;
                if (k < kl) {
                    kl = k;
                    jl = j;
                }
            }
            for (;;) {
                const float kmin = wave_min(kl);
                if (!(kmin < __builtin_inff())) break;
                const uint32_t sl = (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(kl == kmin));
                const uint32_t js = (uint32_t)__builtin_amdgcn_readlane((int)jl, (int)sl);
                if (lane == sl) {  // drop the pick from this lane's entries, find its next least
                    row[sl + 64u * js] = __builtin_inff();
                    kl = __builtin_inff();
                    for (uint32_t j = 0; j < (uint32_t)kKeySlots; ++j) {
                        const float k = row[lane + 64u * j];
                        if (k < kl) {
                            kl = k;
                            jl = j;
                        }
                    }
                }
                const uint32_t sp = sl + 64u * js;
                if (need_box(sbox + (size_t)sp * 2 * D, smin[sp])) visit_super(sp, 0xFFFFFFFFu);
            }
            goto done;
        }
    }
    {
    const uint32_t chunks = (S + 63) / 64, home_c = home_s / 64;
    for (uint32_t st = 0; st < 2 * chunks; ++st) {
        const int64_t c64 = (st & 1u) ? (int64_t)home_c - (int64_t)((st + 1) / 2) : (int64_t)home_c + (int64_t)(st / 2);
        if (c64 < 0 || c64 >= (int64_t)chunks) continue;
        const uint32_t sp = (uint32_t)c64 * 64 + lane;
        const bool need = sp < S && sp != home_s && need_box(sbox + (size_t)sp * 2 * D, smin[sp]);
        uint64_t m = __builtin_amdgcn_ballot_w64(need);
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctzll(m);
            m &= m - 1ull;
            visit_super((uint32_t)c64 * 64 + b, 0xFFFFFFFFu);
        }
    }
    }
done:
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        if (g0 + q >= q_count) break;
        const size_t o = VGPU_DCLAMP(dbg, qi[q] - q_first, q_count, DBG_KNN_QUERY);
        if (lane == 0) cnt[o] = c[q];
        if (lane < c[q]) {
            nbr[o * kmax + lane] = bi[q];
            dist[o * kmax + lane] = bd[q];
        }
    }
}

// ---- block-cooperative group queries (VAMP_AMD_KNN_COOP=4 or 8; an A/B option, not the default) ----------
// group_kernel fetches every candidate tile once per WAVE (4 queries): at 2.7M Fetch vertices each wave
// visits ~700 tiles spread over the whole vertex set, so the tiles miss the 4 MB L2 and ~1.1 TB per call
// comes from the Infinity Cache.  Here the WV waves of a workgroup (4 * WV Morton-consecutive
// queries, whose neighbourhoods overlap) decide together which super-tiles and tiles to visit -- the union
// of their needs, a block-wide OR of each wave's ballot -- and stage each needed tile ONCE per workgroup in
// LDS (one tile per wave per batch, double buffered: the next batch's global loads are in flight while the current
// one is tested); a wave tests a staged tile only if one of its own queries needs it.  Same visiting rules
// (home super-tile first, then chunks outward), same admission: the lists are again exactly the brute
// force's.
template <int D, int QG, int WV>
__global__ __launch_bounds__(64 * WV) void coop_kernel(const float* __restrict__ Vs, const uint32_t* __restrict__ perm,
                                                       uint32_t n, uint32_t T, uint32_t S,
                                                       const float* __restrict__ tbox, const uint32_t* __restrict__ tmin,
                                                       const float* __restrict__ sbox, const uint32_t* __restrict__ smin,
                                                       const uint32_t* __restrict__ qlist, uint32_t q_first,
                                                       uint32_t q_count, const uint32_t* __restrict__ kq,
                                                       const float* __restrict__ rq, uint32_t kmax,
                                                       uint32_t* __restrict__ nbr, float* __restrict__ dist,
                                                       uint32_t* __restrict__ cnt, uint32_t* __restrict__ dbg)
{
    constexpr int NT = 64 * WV;
    constexpr int kCoopBT = WV;  // tiles per staged batch: one candidate per thread
    constexpr int CPT = kCoopBT * kTile / NT;
    __shared__ float scand[2][kCoopBT][D][kTile];  // [buffer][tile][dim][candidate]: lane reads are conflict-free
    __shared__ uint32_t sidx[2][kCoopBT][kTile];
    __shared__ uint64_t sneed[WV];
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = xcd_block(blockIdx.x, gridDim.x) * WV + w;
    const uint32_t g0 = wave * QG;
    // a wave past the queries still takes part in every barrier, with nothing to need
    const bool active = g0 < q_count;
    uint32_t qi[QG], kk[QG], c[QG], wi[QG];
    float me[QG][D], wd[QG], thr[QG];
    uint32_t p0 = 0;
    auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    auto unf = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const uint32_t qo = g0 + q;
        const bool inq = qo < q_count;
        const uint32_t p = uni(VGPU_DCLAMP(dbg, inq ? (qlist ? qlist[qo] : qo) : 0u, n, DBG_KNN_QUERY));
        if (q == 0) p0 = p;
        qi[q] = uni(inq ? VGPU_DCLAMP(dbg, perm[p], n, DBG_KNN_VERTEX) : 0u);
        const bool live = inq && qi[q] >= 2;  // vertices 0, 1 (start, goal) query nothing (prm.hh:228-233)
#pragma unroll
        for (int d = 0; d < D; ++d) me[q][d] = unf(inq ? Vs[(size_t)p * D + d] : 0.0f);
        kk[q] = uni(live ? min(kq[qi[q]], 64u) : 0u);
        wd[q] = unf(live ? rq[qi[q]] : -1.0f);
        wi[q] = 0xFFFFFFFFu;
        c[q] = 0;
        thr[q] = (live && kk[q]) ? wd[q] * wd[q] * 1.000001f : -1.0f;
    }
    float bd[QG];
    uint32_t bi[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        bd[q] = __builtin_inff();
        bi[q] = 0xFFFFFFFFu;
    }
    auto consider = [&](const float* cv, uint32_t cj) {
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const float s = sumsq<D>(cv, me[q]);
            uint64_t m = __builtin_amdgcn_ballot_w64(cj < qi[q] && s <= thr[q]);
            if (m == 0ull) continue;
            const float dl = __builtin_sqrtf(s);
            while (m) {
                const uint32_t b = (uint32_t)__builtin_ctzll(m);
                m &= m - 1ull;
                const float d = bcast(dl, b);
                const uint32_t j = bcast(cj, b);
                const bool take = c[q] < kk[q] ? d <= wd[q] : (d < wd[q] || (d == wd[q] && j < wi[q]));
                if (!take) continue;
                const uint32_t lt = (d < bd[q] || (d == bd[q] && j < bi[q])) ? 1u : 0u;
                const float pd = shfl_up1(bd[q]);
                const uint32_t pi = shfl_up1(bi[q]);
                const uint32_t plt_raw = shfl_up1(lt);
                const bool plt = lane > 0 && plt_raw != 0u;
                bd[q] = lt ? (plt ? pd : d) : bd[q];
                bi[q] = lt ? (plt ? pi : j) : bi[q];
                c[q] = min(c[q] + 1u, kk[q]);
                if (c[q] == kk[q]) {
                    wd[q] = bcast(bd[q], kk[q] - 1u);
                    wi[q] = bcast(bi[q], kk[q] - 1u);
                    thr[q] = wd[q] * wd[q] * 1.000001f;
                }
            }
        }
    };
    auto need_box = [&](const float* __restrict__ bx, uint32_t mn) {
        bool need = false;
#pragma unroll
        for (int q = 0; q < QG; ++q) need |= mn < qi[q] && box_lb<D>(bx, me[q]) <= thr[q] * 1.0001f;
        return need;
    };
    // the block-wide OR of every wave's 64-bit mask (two barriers)
    auto block_or = [&](uint64_t m) {
        if (lane == 0) sneed[w] = m;
        __syncthreads();
        uint64_t r = 0ull;
#pragma unroll
        for (int i = 0; i < WV; ++i) r |= sneed[i];
        __syncthreads();
        return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)r) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(r >> 32)) << 32);
    };
    // candidate slot e of a batch (tile e / 64 of the batch's list, candidate e % 64): staged by thread
    // e mod NT; tile lists are fixed-size arrays indexed by compile-time positions only (no scratch)
    float rv[CPT][D];
    uint32_t rj[CPT];
    auto fetch = [&](const uint32_t (&tl)[kCoopBT], int nt) {  // global -> registers
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
            const uint32_t e = threadIdx.x + (uint32_t)k * NT;
            const uint32_t tb = e / kTile;
            uint32_t tile = 0xFFFFFFFFu;
#pragma unroll
            for (int i = 0; i < kCoopBT; ++i)
                if (tb == (uint32_t)i && i < nt) tile = tl[i];
            const bool okt = tile != 0xFFFFFFFFu;
            const uint32_t cp = (okt ? VGPU_DCLAMP(dbg, tile, T, DBG_KNN_TILE) : 0u) * kTile + (e % kTile);
            const bool ok = okt && cp < n;
#pragma unroll
            for (int d = 0; d < D; ++d) rv[k][d] = ok ? Vs[(size_t)cp * D + d] : 0.0f;
            rj[k] = ok ? perm[cp] : 0xFFFFFFFFu;  // a missing candidate is never < i
        }
    };
    auto stage = [&](int buf) {  // registers -> LDS
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
            const uint32_t e = threadIdx.x + (uint32_t)k * NT;
#pragma unroll
            for (int d = 0; d < D; ++d) scand[buf][e / kTile][d][e % kTile] = rv[k][d];
            sidx[buf][e / kTile][e % kTile] = rj[k];
        }
    };
    // this wave's tests of a staged batch: only the tiles one of its own queries needs
    auto test = [&](int buf, const uint32_t (&tl)[kCoopBT], int nt, uint32_t sp, uint64_t mine) {
#pragma unroll
        for (int b = 0; b < kCoopBT; ++b) {
            if (b >= nt) break;
            if (!((mine >> (tl[b] - sp * kSuper)) & 1ull)) continue;
            float cv[D];
#pragma unroll
            for (int d = 0; d < D; ++d) cv[d] = scand[buf][b][d][lane];
            consider(cv, sidx[buf][b][lane]);
        }
    };
    // every tile of super-tile sp in the block's union of needs, staged batch by batch (double buffered,
    // the loop unrolled by two so every buffer and list index is a constant)
    auto visit_super = [&](uint32_t sp) {
        sp = VGPU_DCLAMP(dbg, sp, S, DBG_KNN_SUPER);
        const uint32_t t = sp * kSuper + lane;
        const bool need = active && t < T && need_box(tbox + (size_t)t * 2 * D, tmin[t]);
        const uint64_t mine = __builtin_amdgcn_ballot_w64(need);
        uint64_t m = block_or(mine);
        uint32_t ta[kCoopBT], tb[kCoopBT];
        int na = 0, nb = 0;
        auto take = [&](uint32_t (&tl)[kCoopBT], int& nt) {
            nt = 0;
#pragma unroll
            for (int i = 0; i < kCoopBT; ++i) {
                tl[i] = 0u;
                if (m) {
                    tl[i] = sp * kSuper + (uint32_t)__builtin_ctzll(m);
                    m &= m - 1ull;
                    nt = i + 1;
                }
            }
        };
        take(ta, na);
        if (!na) return;
        fetch(ta, na);
        for (;;) {
            stage(0);
            __syncthreads();
            take(tb, nb);
            if (nb) fetch(tb, nb);  // in flight while the staged batch is tested
            test(0, ta, na, sp, mine);
            __syncthreads();
            if (!nb) break;
            stage(1);
            __syncthreads();
            take(ta, na);
            if (na) fetch(ta, na);
            test(1, tb, nb, sp, mine);
            __syncthreads();
            if (!na) break;
        }
    };
    // the block's home super-tile first (its first query's), then the other super-tiles in chunks of 64
    // outward; a super-tile is visited when some query of the block can take from it
    const uint32_t home_s = uni(__builtin_amdgcn_readfirstlane(p0) / kTile / kSuper);
    __shared__ uint32_t shome;
    if (threadIdx.x == 0) shome = home_s;
    __syncthreads();
    const uint32_t bhome = shome;  // wave 0's
    visit_super(bhome);
    const uint32_t chunks = (S + 63) / 64, home_c = bhome / 64;
    for (uint32_t st = 0; st < 2 * chunks; ++st) {
        const int64_t c64 = (st & 1u) ? (int64_t)home_c - (int64_t)((st + 1) / 2) : (int64_t)home_c + (int64_t)(st / 2);
        if (c64 < 0 || c64 >= (int64_t)chunks) continue;
        const uint32_t sp = (uint32_t)c64 * 64 + lane;
        const bool need = active && sp < S && sp != bhome && need_box(sbox + (size_t)sp * 2 * D, smin[sp]);
        uint64_t m = block_or(__builtin_amdgcn_ballot_w64(need));
        if ((uint64_t)c64 == home_c) m &= ~(1ull << (bhome & 63u));  // visited first, never twice
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctzll(m);
            m &= m - 1ull;
            visit_super((uint32_t)c64 * 64 + b);
        }
    }
    if (!active) return;
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        if (g0 + q >= q_count) break;
        const size_t o = VGPU_DCLAMP(dbg, qi[q] - q_first, q_count, DBG_KNN_QUERY);
        if (lane == 0) cnt[o] = c[q];
        if (lane < c[q]) {
            nbr[o * kmax + lane] = bi[q];
            dist[o * kmax + lane] = bd[q];
        }
    }
}

inline size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

struct Layout {
    size_t part, ls, key0, key1, id0, perm, Vs, tbox, tmin, qc, qh, sbox, smin, flag, qlist, nsel, tmp, total;
};

template <int D>
hipError_t layout(uint32_t n, uint32_t q_count, Layout& L)
{
    const uint32_t T = (n + kTile - 1) / kTile;
    size_t tsort = 0, tsel = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tsort, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                      (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0,
                                                      D * bits_per_dim<D>());
    if (e != hipSuccess) return e;
    e = hipcub::DeviceSelect::Flagged(nullptr, tsel, hipcub::CountingInputIterator<uint32_t>(0), (uint8_t*)nullptr,
                                      (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    if (e != hipSuccess) return e;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += al256(bytes ? bytes : 1);
        return at;
    };
    L.part = take((size_t)kMinMaxBlocks * 2 * D * 4);
    L.ls = take(2 * D * 4);
    L.key0 = take((size_t)n * 8);
    L.key1 = take((size_t)n * 8);
    L.id0 = take((size_t)n * 4);
    L.perm = take((size_t)n * 4);
    L.Vs = take((size_t)n * D * 4);
    L.tbox = take((size_t)T * 2 * D * 4);
    L.tmin = take((size_t)T * 4);
    L.qc = take((size_t)T * code_words<D>() * kTile * 4);
    L.qh = take((size_t)T * (D + 1) * 4);
    const uint32_t S = (T + kSuper - 1) / kSuper;
    L.sbox = take((size_t)S * 2 * D * 4);
    L.smin = take((size_t)S * 4);
    L.flag = take(n);
    L.qlist = take((size_t)q_count * 4);
    L.nsel = take(4);
    L.tmp = take(std::max(tsort, tsel));
    L.total = o;
    return hipSuccess;
}

template <int D, int K>
hipError_t run(const float* V, uint32_t n, uint32_t q_first, uint32_t q_count, const uint32_t* k, const float* r,
               uint32_t kmax, uint32_t* nbr, float* dist, uint32_t* cnt, char* pool, size_t pool_bytes, int group,
               uint32_t* dbg, hipStream_t st)
{
    Layout L;
    hipError_t e = layout<D>(n, q_count, L);
    if (e != hipSuccess) return e;
    if (pool_bytes < L.total) return hipErrorInvalidValue;
    const uint32_t T = (n + kTile - 1) / kTile;
    float* part = (float*)(pool + L.part);
    float* ls = (float*)(pool + L.ls);
    uint64_t* key0 = (uint64_t*)(pool + L.key0);
    uint64_t* key1 = (uint64_t*)(pool + L.key1);
    uint32_t* id0 = (uint32_t*)(pool + L.id0);
    uint32_t* perm = (uint32_t*)(pool + L.perm);
    float* Vs = (float*)(pool + L.Vs);
    float* tbox = (float*)(pool + L.tbox);
    uint32_t* tmin = (uint32_t*)(pool + L.tmin);
    uint32_t* qc = (uint32_t*)(pool + L.qc);
    float* qh = (float*)(pool + L.qh);
    uint8_t* flag = (uint8_t*)(pool + L.flag);
    uint32_t* qlist = (uint32_t*)(pool + L.qlist);
    uint32_t* nsel = (uint32_t*)(pool + L.nsel);
    void* tmp = pool + L.tmp;
    const size_t tbytes = pool_bytes - L.tmp;
    const unsigned mmb = (unsigned)std::min<size_t>(kMinMaxBlocks, std::max<size_t>(1, (n + 255) / 256));
    hipLaunchKernelGGL((minmax_kernel<D>), dim3(mmb), dim3(256), 0, st, V, n, part);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((scale_kernel<D>), dim3(1), dim3(64), 0, st, part, (uint32_t)mmb, ls);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((key_kernel<D>), dim3((n + 255) / 256), dim3(256), 0, st, V, n, ls, key0, id0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = tbytes;
    e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, key0, key1, id0, perm, (int)n, 0, D * bits_per_dim<D>(), st);
    if (e != hipSuccess) return e;
    // coded candidates (VAMP_AMD_KNN_QCODE=1; an A/B option, default 0 = every visited candidate read exactly).
    // A/B on MI355X (profiles/r05g_ab.log): 2.68M vertices 216 ms exact vs 380 ms coded, 100k 3.6 vs 6.8 ms --
    // the tile's bytes were not the bound: the coded test adds a dependent load (codes -> test -> exact rows)
    // and registers, and the kernel waits on latency, not on bandwidth
    static const bool qcode = [] {
        const char* s = std::getenv("VAMP_AMD_KNN_QCODE");
        return s ? std::atoi(s) != 0 : false;
    }();
    hipLaunchKernelGGL((tile_kernel<D>), dim3(T), dim3(kTile), 0, st, V, perm, n, Vs, tbox, tmin,
                       qcode && group > 0 ? qc : nullptr, qh);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint32_t* ql = nullptr;
    if (!(q_first == 0 && q_count == n)) {
        hipLaunchKernelGGL(qflag_kernel, dim3((n + 255) / 256), dim3(256), 0, st, perm, n, q_first, q_first + q_count,
                           flag);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        tb = tbytes;
        e = hipcub::DeviceSelect::Flagged(tmp, tb, hipcub::CountingInputIterator<uint32_t>(0), flag, qlist, nsel,
                                          (int)n, st);
        if (e != hipSuccess) return e;
        ql = qlist;  // exactly q_count entries: perm is a permutation of 0 .. n-1
    }
    if (group <= 0) {  // the 64-query waves (VAMP_AMD_KNN_GROUP=0, for A/B runs)
        const unsigned grid = (unsigned)((q_count + kQBlock - 1) / kQBlock);
        hipLaunchKernelGGL((query_kernel<D, K>), dim3(grid), dim3(kQBlock), 0, st, Vs, perm, n, T, tbox, tmin, ql,
                           q_first, q_count, k, r, kmax, nbr, dist, cnt);
        return hipGetLastError();
    }
    const uint32_t S = (T + kSuper - 1) / kSuper;
    float* sbox = (float*)(pool + L.sbox);
    uint32_t* smin = (uint32_t*)(pool + L.smin);
    hipLaunchKernelGGL((super_kernel<D>), dim3(S), dim3(64), 0, st, tbox, tmin, T, sbox, smin);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint32_t QG = group >= 8 ? 8 : (group >= 4 ? 4 : (group >= 2 ? 2 : 1));
    const uint64_t waves = (q_count + QG - 1) / QG;
    // block-cooperative tiles (VAMP_AMD_KNN_COOP: waves per workgroup, 4 or 8; 0 = group_kernel, the default).
    // A/B on MI355X, 2.68M Fetch vertices (profiles/r05e_ab.log): group_kernel 212 ms, coop 4 waves 263 ms,
    // 8 waves 326 ms -- the shared tiles cost a block barrier per batch and the union of four waves' needs,
    // more than the L2 misses they save.
    static const int coop = [] {
        const char* s = std::getenv("VAMP_AMD_KNN_COOP");
        return s ? std::atoi(s) : 0;
    }();
    if (coop > 0 && QG == 4) {
        const int WV = coop >= 8 ? 8 : 4;
        const unsigned cgrid = (unsigned)((waves + WV - 1) / WV);
        if (WV == 8)
            hipLaunchKernelGGL((coop_kernel<D, 4, 8>), dim3(cgrid), dim3(512), 0, st, Vs, perm, n, T, S, tbox, tmin, sbox,
                               smin, ql, q_first, q_count, k, r, kmax, nbr, dist, cnt, dbg);
        else
            hipLaunchKernelGGL((coop_kernel<D, 4, 4>), dim3(cgrid), dim3(256), 0, st, Vs, perm, n, T, S, tbox, tmin, sbox,
                               smin, ql, q_first, q_count, k, r, kmax, nbr, dist, cnt, dbg);
        return hipGetLastError();
    }
    const unsigned grid = (unsigned)((waves + kQBlock / 64 - 1) / (kQBlock / 64));
#define VGPU_KNN_GROUP_LAUNCH(Q, C)                                                                                   \
    hipLaunchKernelGGL((group_kernel<D, Q, C>), dim3(grid), dim3(kQBlock), 0, st, Vs, perm, n, T, S, tbox, tmin,   \
                       sbox, smin, qc, qh, ql, q_first, q_count, k, r, kmax, nbr, dist, cnt, dbg)
    switch (QG * 2 + (qcode ? 1 : 0)) {
    case 2: VGPU_KNN_GROUP_LAUNCH(1, false); break;
    case 3: VGPU_KNN_GROUP_LAUNCH(1, true); break;
    case 4: VGPU_KNN_GROUP_LAUNCH(2, false); break;
    case 5: VGPU_KNN_GROUP_LAUNCH(2, true); break;
    case 8: VGPU_KNN_GROUP_LAUNCH(4, false); break;
    case 9: VGPU_KNN_GROUP_LAUNCH(4, true); break;
    case 16: VGPU_KNN_GROUP_LAUNCH(8, false); break;
    default: VGPU_KNN_GROUP_LAUNCH(8, true); break;
    }
#undef VGPU_KNN_GROUP_LAUNCH
    return hipGetLastError();
}

template <int D>
hipError_t run_dim(const float* V, uint32_t n, uint32_t qf, uint32_t qc, const uint32_t* k, const float* r,
                   uint32_t kmax, uint32_t* nbr, float* dist, uint32_t* cnt, char* pool, size_t pb, int g,
                   uint32_t* dbg, hipStream_t st)
{
    if (g > 0) return run<D, 64>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, pool, pb, g, dbg, st);  // K unused
    if (kmax <= 16) return run<D, 16>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, pool, pb, g, dbg, st);
    if (kmax <= 32) return run<D, 32>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, pool, pb, g, dbg, st);
    if (kmax <= 48) return run<D, 48>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, pool, pb, g, dbg, st);
    return run<D, 64>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, pool, pb, g, dbg, st);
}

}  // namespace knnidx
}  // namespace vgpu

extern "C" {

// pool bytes the indexed query of n vertices / q_count queries needs (0: unsupported dim)
size_t vgpu_knn_index_bytes(int dim, uint32_t n, uint32_t q_count)
{
    using namespace vgpu::knnidx;
    Layout L;
    hipError_t e = hipErrorInvalidValue;
    switch (dim) {
    case 6: e = layout<6>(n, q_count, L); break;
    case 7: e = layout<7>(n, q_count, L); break;
    case 8: e = layout<8>(n, q_count, L); break;
    case 14: e = layout<14>(n, q_count, L); break;
    default: return 0;
    }
    return e == hipSuccess ? L.total : 0;
}

// kmax <= 64, dim in {6, 7, 8, 14}, n >= 1, q_count >= 1 (checked by the caller)
hipError_t vgpu_launch_knn_index(int dim, const float* V, uint32_t n, uint32_t q_first, uint32_t q_count,
                                 const uint32_t* k, const float* r, uint32_t kmax, uint32_t* nbr, float* dist,
                                 uint32_t* cnt, void* pool, size_t pool_bytes, uint32_t* dbg, hipStream_t st)
{
    using namespace vgpu::knnidx;
    char* p = (char*)pool;
    // queries per wave of the group kernel (VAMP_AMD_KNN_GROUP: 1, 2, 4 or 8; 0 = the 64-query waves)
    static const int g = [] {
        const char* s = std::getenv("VAMP_AMD_KNN_GROUP");
        return s ? std::atoi(s) : 4;
    }();
    switch (dim) {
    case 6: return run_dim<6>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, p, pool_bytes, g, dbg, st);
    case 7: return run_dim<7>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, p, pool_bytes, g, dbg, st);
    case 8: return run_dim<8>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, p, pool_bytes, g, dbg, st);
    case 14: return run_dim<14>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, p, pool_bytes, g, dbg, st);
    default: return hipErrorInvalidValue;
    }
}

}  // extern "C"
