// vgpu_roadmap.hip -- the PRM roadmap edge stage: the neighbour queries of
// Roadmap::build_roadmap (planning/prm.hh:264-266) for a whole vertex sequence at once, and the
// gather of the candidate edges validate_motion(neighbor, vertex) checks (prm.hh:267-276).
//
// build_roadmap inserts vertex i after querying the tree of vertices 0 .. i-1 for at most
// k(i) = PRMStarNeighborParams::max_neighbors(i) neighbours within r(i) = neighbor_radius(i)
// (roadmap.hh:49-67).  The query set never depends on which edges were valid, so the queries of
// all vertices are independent: "causal" kNN, vertex i against its prefix.
//
// knn_kernel: one lane per query vertex, 256 queries per block, and the candidate prefix split
// into chunks along grid y (the work of query i grows with i: without the split a few blocks
// scan 1e5 candidates serially).  Candidates stream through LDS in tiles of 256 rows (every lane
// reads the same row: LDS broadcast).  Each lane keeps its K best (distance, index) keys sorted in
// registers; a candidate enters by one unrolled compare-exchange pass (no dynamic register
// indexing), run only when some lane of the wave takes a candidate; the correctly rounded sqrt
// runs only when some lane's squared sum is below its bound.  knn_merge_kernel combines a
// query's chunk lists into the k smallest keys.  Distance = Space<dim>::distance (nn.hh:53-57):
// the lane-wise difference's l2_norm in the AVX hsum order (pinned by ref_probe "l2norm").  Ties
// keep the lower index first (nigh's tie order is not pinned: DESIGN.md).
#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "vgpu_device.hh"

namespace vgpu {

constexpr int kKnnBlock = 256;
constexpr int kKnnBuf = 8;  // buffered candidates per lane between insertion passes

// FloatVector<D>::l2_norm of a - b (vector/avx.hh:441-452; two registers contract to
// fma(lo, lo, hi * hi), pinned by ref_probe "l2norm") before its sqrt: the squared sum in the
// AVX hsum lane order
template <int D>
__device__ __forceinline__ float config_sumsq(const float* a, const float* b)
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

// Insert (cd, ci) into the register list (bd, bi) of K entries sorted by the key (distance,
// index), by one unrolled compare-exchange pass: the carried element displaced from an earlier
// slot passes equal distances with larger indices.  No dynamic register indexing.
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

// Partial queries: block (x, y) = queries q0 .. q0+255 against the candidate chunk
// [y * S, (y + 1) * S) of their prefixes; each query's chunk list = its k smallest keys
// (distance, index) with distance <= r within the chunk.  The exact result is the k smallest keys
// over all chunks (knn_merge_kernel): the same set and order as one sequential scan.
template <int D, int K>
__global__ __launch_bounds__(kKnnBlock) void knn_kernel(const float* __restrict__ V, uint32_t n, uint32_t q_first,
                                                         uint32_t q_count, const uint32_t* __restrict__ kq,
                                                         const float* __restrict__ rq, uint32_t kmax, uint32_t S,
                                                         uint32_t C, float* __restrict__ pd,
                                                         uint32_t* __restrict__ pi, uint32_t* __restrict__ pc)
{
    __shared__ float tile[kKnnBlock * D];
    // per-lane buffers of taken candidates: inserted into the register lists in batches, so the
    // wave runs the K-slot insertion pass max-over-lanes times per batch instead of once for
    // every candidate some lane takes
    __shared__ float buf_d[kKnnBuf][kKnnBlock];
    __shared__ uint32_t buf_i[kKnnBuf][kKnnBlock];
    // heaviest query blocks (largest prefixes) first
    const uint32_t blk = gridDim.x - 1 - blockIdx.x;
    const uint32_t chunk = blockIdx.y;
    const uint32_t q_end = min(n, q_first + q_count);  // this call's queries: q_first .. q_end-1
    const uint32_t q0 = q_first + blk * kKnnBlock;
    const uint32_t last = min(q_end, q0 + kKnnBlock);  // candidates 0 .. last-2 matter to this block
    const uint32_t c_lo = chunk * S;
    if (c_lo + 1 >= last) return;  // no query of the block reaches this chunk (the merge skips it)
    const uint32_t c_hi = min(c_lo + S, last - 1);
    const uint32_t lane = threadIdx.x;
    const uint32_t i = q0 + lane;
    const bool live = i < q_end && i >= 2;  // vertices 0, 1 (start, goal) query nothing (prm.hh:228-233)
    float me[D];
#pragma unroll
    for (int j = 0; j < D; ++j) me[j] = (i < q_end) ? V[(size_t)i * D + j] : 0.0f;
    const uint32_t k = live ? min(kq[i], (uint32_t)K) : 0u;  // k, r indexed by vertex
    const float r = live ? rq[i] : -1.0f;
    float bd[K];
    uint32_t bi[K];
#pragma unroll
    for (int m = 0; m < K; ++m) {
        bd[m] = __builtin_inff();
        bi[m] = 0xFFFFFFFFu;
    }
    uint32_t c = 0, nb = 0;
    // a candidate must be within r and closer than the current k-th (when k are held); thr is a
    // bound on the squared distance below which sqrt_rn(s) <= worst is possible (w^2 (1 + 2^-20)
    // > (w + ulp(w)/2)^2), so the correctly rounded sqrt runs only for plausible candidates.
    // worst may be stale while candidates wait in the buffer: it only admits more of them, and
    // the list keeps the K smallest keys of everything inserted.
    float worst = r;
    float thr = live ? r * r * 1.000001f : -1.0f;
    auto flush = [&]() {
        for (uint32_t m = 0; __builtin_amdgcn_ballot_w64(m < nb) != 0ull; ++m) {
            const bool has = m < nb;
            list_insert<K>(bd, bi, has ? buf_d[has ? m : 0][lane] : __builtin_inff(),
                           has ? buf_i[has ? m : 0][lane] : 0xFFFFFFFFu);
        }
        c = min(c + nb, k);  // every buffered candidate is within r
        nb = 0;
        float kth = r;
#pragma unroll
        for (int m = 0; m < K; ++m)
            if ((uint32_t)m + 1 == k) kth = bd[m];
        worst = (c == k) ? kth : r;
        thr = live ? worst * worst * 1.000001f : -1.0f;
    };
    for (uint32_t t0 = c_lo; t0 < c_hi; t0 += kKnnBlock) {
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < kKnnBlock * D; e += kKnnBlock) {
            const size_t g = (size_t)t0 * D + e;
            tile[e] = (g < (size_t)n * D) ? V[g] : 0.0f;
        }
        __syncthreads();
        const uint32_t tn = min((uint32_t)kKnnBlock, c_hi - t0);
        auto consider = [&](uint32_t j, float s) {
            const bool pre = j < i && s <= thr;
            if (__builtin_amdgcn_ballot_w64(pre) == 0ull) return;
            const float d = __builtin_sqrtf(s);
            // nn query semantics: distance <= r, strictly closer than the k-th to displace it
            const bool take = pre && (c < k ? d <= worst : d < worst);
            if (take) {
                buf_d[nb][lane] = d;
                buf_i[nb][lane] = j;
                ++nb;
            }
        };
        // a step appends at most 4 per lane: flush while the buffers still have room for that
        auto maybe_flush = [&]() {
            if (__builtin_amdgcn_ballot_w64(nb > kKnnBuf - 4) != 0ull) flush();
        };
        uint32_t u = 0;
        // four candidates per step: independent LDS reads and sums in flight, one ballot when
        // none of them is plausible for any lane (the common case)
        for (; u + 4 <= tn; u += 4) {
            float s4[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) s4[h] = config_sumsq<D>(tile + (u + h) * D, me);
            bool any = false;
#pragma unroll
            for (int h = 0; h < 4; ++h) any |= (t0 + u + h < i) && s4[h] <= thr;
            if (__builtin_amdgcn_ballot_w64(any) == 0ull) continue;
#pragma unroll
            for (int h = 0; h < 4; ++h) consider(t0 + u + h, s4[h]);
            maybe_flush();
        }
        for (; u < tn; ++u) {
            consider(t0 + u, config_sumsq<D>(tile + u * D, me));
            maybe_flush();
        }
        if (__builtin_amdgcn_ballot_w64(nb != 0) != 0ull) flush();
    }
    if (i < q_end) {
        const size_t o = ((size_t)(i - q_first) * C + chunk);
        pc[o] = c;
#pragma unroll
        for (int m = 0; m < K; ++m) {
            if ((uint32_t)m < c) {
                pd[o * kmax + m] = bd[m];
                pi[o * kmax + m] = bi[m];
            }
        }
    }
}

// Final lists: the k smallest keys over the chunk lists of query i (chunks c with c * S < i)
template <int K>
__global__ __launch_bounds__(256) void knn_merge_kernel(uint32_t n, uint32_t q_first, uint32_t q_count,
                                                         const uint32_t* __restrict__ kq, uint32_t kmax, uint32_t S,
                                                         uint32_t C, const float* __restrict__ pd,
                                                         const uint32_t* __restrict__ pi,
                                                         const uint32_t* __restrict__ pc, uint32_t* __restrict__ nbr,
                                                         float* __restrict__ dist, uint32_t* __restrict__ cnt)
{
    const uint32_t o = blockIdx.x * 256 + threadIdx.x;
    if (o >= q_count) return;
    const uint32_t i = q_first + o;
    const uint32_t k = i >= 2 ? min(kq[i], (uint32_t)K) : 0u;
    float bd[K];
    uint32_t bi[K];
#pragma unroll
    for (int m = 0; m < K; ++m) {
        bd[m] = __builtin_inff();
        bi[m] = 0xFFFFFFFFu;
    }
    uint32_t total = 0;
    const uint32_t nch = k ? min(C, (i + S - 1) / S) : 0u;
    for (uint32_t ch = 0; ch < nch; ++ch) {
        const size_t b = (size_t)o * C + ch;
        const uint32_t pn = pc[b];
        total += pn;
        for (uint32_t m = 0; m < pn; ++m) list_insert<K>(bd, bi, pd[b * kmax + m], pi[b * kmax + m]);
    }
    const uint32_t c = min(total, k);
    cnt[o] = c;
#pragma unroll
    for (int m = 0; m < K; ++m) {
        if ((uint32_t)m < c) {
            nbr[(size_t)o * kmax + m] = bi[m];
            dist[(size_t)o * kmax + m] = bd[m];
        }
    }
}

// candidate edge e = (query i, its m-th neighbour): starts[e] = V[nbr], goals[e] = V[i]
// (validate_motion(neighbor.as_vector(), temp, ...), prm.hh:268)
__global__ __launch_bounds__(256) void edge_gather_kernel(const float* __restrict__ V, uint32_t q_first, uint32_t n,
                                                          int dim,
                                                          const uint32_t* __restrict__ nbr, uint32_t kmax,
                                                          const uint32_t* __restrict__ cnt,
                                                          const uint32_t* __restrict__ off,
                                                          float* __restrict__ starts, float* __restrict__ goals)
{
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t i = t / kmax;
    const uint32_t m = (uint32_t)(t - i * kmax);
    if (i >= n || m >= cnt[i]) return;
    const size_t e = (size_t)off[i] + m;
    const uint32_t j = nbr[i * kmax + m];
    const size_t v = q_first + i;  // query vertex
    for (int d = 0; d < dim; ++d) {
        starts[e * dim + d] = V[(size_t)j * dim + d];
        goals[e * dim + d] = V[v * dim + d];
    }
}

// candidate e = off[i] + m of query i -> the pair (vertex q_first + i, neighbour nbr[i][m]) packed as
// two u32 words (vertex first): the valid ones, selected in candidate order, are the pairs build_roadmap
// connects (prm.hh:268-275) in query order, nearest first
__global__ __launch_bounds__(256) void edge_pairs_kernel(uint32_t q_first, uint32_t n,
                                                         const uint32_t* __restrict__ nbr, uint32_t kmax,
                                                         const uint32_t* __restrict__ cnt,
                                                         const uint32_t* __restrict__ off,
                                                         unsigned long long* __restrict__ pairs)
{
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t i = t / kmax;
    const uint32_t m = (uint32_t)(t - i * kmax);
    if (i >= n || m >= cnt[i]) return;
    const unsigned long long v = q_first + (uint32_t)i, j = nbr[i * kmax + m];
    pairs[(size_t)off[i] + m] = v | (j << 32);
}

}  // namespace vgpu

template <int D, int K>
static hipError_t launch_knn(const float* V, uint32_t n, uint32_t qf, uint32_t qc, const uint32_t* k, const float* r,
                             uint32_t kmax, uint32_t S, uint32_t C, float* pd, uint32_t* pi, uint32_t* pc,
                             uint32_t* nbr, float* dist, uint32_t* cnt, hipStream_t st)
{
    const unsigned qb = (qc + vgpu::kKnnBlock - 1) / vgpu::kKnnBlock;
    hipLaunchKernelGGL((vgpu::knn_kernel<D, K>), dim3(qb, C), dim3(vgpu::kKnnBlock), 0, st, V, n, qf, qc, k, r, kmax,
                       S, C, pd, pi, pc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((vgpu::knn_merge_kernel<K>), dim3((qc + 255) / 256), dim3(256), 0, st, n, qf, qc, k, kmax, S, C,
                       pd, pi, pc, nbr, dist, cnt);
    return hipGetLastError();
}

template <int D>
static hipError_t knn_dim(const float* V, uint32_t n, uint32_t qf, uint32_t qc, const uint32_t* k, const float* r,
                          uint32_t kmax, uint32_t S, uint32_t C, float* pd, uint32_t* pi, uint32_t* pc, uint32_t* nbr,
                          float* dist, uint32_t* cnt, hipStream_t st)
{
    if (kmax <= 16) return launch_knn<D, 16>(V, n, qf, qc, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    if (kmax <= 32) return launch_knn<D, 32>(V, n, qf, qc, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    if (kmax <= 40) return launch_knn<D, 40>(V, n, qf, qc, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    if (kmax <= 48) return launch_knn<D, 48>(V, n, qf, qc, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    return launch_knn<D, 64>(V, n, qf, qc, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
}

extern "C" {

// Chunking of the candidate prefixes: S candidates per chunk (a multiple of the block), at most
// 4 chunks; the partial lists need q_count * C * kmax (float + u32) + q_count * C u32.
size_t vgpu_knn_chunks(size_t n, uint32_t* S)
{
    const size_t s = std::max<size_t>(8192, (n + 3) / 4);
    *S = (uint32_t)((s + vgpu::kKnnBlock - 1) / vgpu::kKnnBlock * vgpu::kKnnBlock);
    return std::max<size_t>(1, (n + *S - 1) / *S);
}

// kmax <= 64 and dim in {6, 7, 8, 14} (the robots built here) are checked by the caller
hipError_t vgpu_launch_roadmap_knn(int dim, const float* V, uint32_t n, uint32_t q_first, uint32_t q_count,
                                   const uint32_t* k, const float* r, uint32_t kmax, uint32_t S, uint32_t C, float* pd,
                                   uint32_t* pi, uint32_t* pc, uint32_t* nbr, float* dist, uint32_t* cnt,
                                   hipStream_t st)
{
    if (q_count == 0) return hipSuccess;
    switch (dim) {
    case 6: return knn_dim<6>(V, n, q_first, q_count, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    case 7: return knn_dim<7>(V, n, q_first, q_count, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    case 8: return knn_dim<8>(V, n, q_first, q_count, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    case 14: return knn_dim<14>(V, n, q_first, q_count, k, r, kmax, S, C, pd, pi, pc, nbr, dist, cnt, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t vgpu_launch_edge_gather(const float* V, uint32_t q_first, uint32_t q_count, int dim, const uint32_t* nbr,
                                   uint32_t kmax, const uint32_t* cnt, const uint32_t* off, float* starts,
                                   float* goals, hipStream_t st)
{
    const size_t threads = (size_t)q_count * kmax;
    if (threads == 0) return hipSuccess;
    hipLaunchKernelGGL(vgpu::edge_gather_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, V, q_first,
                       q_count, dim, nbr, kmax, cnt, off, starts, goals);
    return hipGetLastError();
}

// The valid candidate pairs of queries q_first .. +q_count in candidate order: all[E] (scratch) then the
// flagged selection into out[*count] (count: one device u32).  tmp == nullptr: *tmp_bytes = the
// selection's scratch size, nothing launched.
hipError_t vgpu_launch_valid_pairs(uint32_t q_first, uint32_t q_count, const uint32_t* nbr, uint32_t kmax,
                                   const uint32_t* cnt, const uint32_t* off, const uint8_t* ok, size_t E,
                                   unsigned long long* all, unsigned long long* out, uint32_t* count, void* tmp,
                                   size_t* tmp_bytes, hipStream_t st)
{
    if (!tmp)
        return hipcub::DeviceSelect::Flagged(nullptr, *tmp_bytes, all, ok, out, count, (int)std::max<size_t>(E, 1), st);
    if (E == 0) return hipMemsetAsync(count, 0, sizeof(uint32_t), st);
    const size_t threads = (size_t)q_count * kmax;
    hipLaunchKernelGGL(vgpu::edge_pairs_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, q_first,
                       q_count, nbr, kmax, cnt, off, all);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceSelect::Flagged(tmp, *tmp_bytes, all, ok, out, count, (int)E, st);
}

}  // extern "C"
