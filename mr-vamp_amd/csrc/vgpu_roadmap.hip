// vgpu_roadmap.hip -- the PRM roadmap edge stage: the neighbour queries of
// Roadmap::build_roadmap (planning/prm.hh:264-266) for a whole vertex sequence at once, and the
// gather of the candidate edges validate_motion(neighbor, vertex) checks (prm.hh:267-276).
//
// build_roadmap inserts vertex i after querying the tree of vertices 0 .. i-1 for at most
// k(i) = PRMStarNeighborParams::max_neighbors(i) neighbours within r(i) = neighbor_radius(i)
// (roadmap.hh:49-67).  The query set never depends on which edges were valid, so the queries of
// all vertices are independent: "causal" kNN, vertex i against its prefix.
//
// knn_kernel: one lane per query vertex, 256 queries per block; the candidate prefix streams
// through LDS in tiles of 256 rows (every lane reads the same row: LDS broadcast).  Each lane
// keeps its K best (distance, index) pairs sorted in registers; a candidate enters by one
// unrolled compare-exchange pass (no dynamic register indexing), executed only when some lane
// of the wave has a candidate closer than its current K-th (order = (distance, index), so
// ties keep the lower index first).  Distance = Space<dim>::distance
// (nn.hh:53-57): the lane-wise difference's l2_norm in the AVX hsum order (pinned by ref_probe
// "l2norm").  Ties keep the lower index first (nigh's tie order is not pinned: DESIGN.md).
#include "vgpu_device.hh"

namespace vgpu {

constexpr int kKnnBlock = 256;

// FloatVector<D>::l2_norm of a - b (vector/avx.hh:441-452; two registers contract to
// fma(lo, lo, hi * hi), pinned by ref_probe "l2norm")
template <int D>
__device__ __forceinline__ float config_distance(const float* a, const float* b)
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
    const float s = ((sq[0] + sq[4]) + (sq[2] + sq[6])) + ((sq[1] + sq[5]) + (sq[3] + sq[7]));
    return __builtin_sqrtf(s);
}

template <int D, int K>
__global__ __launch_bounds__(kKnnBlock) void knn_kernel(const float* __restrict__ V, uint32_t n, uint32_t q_first,
                                                         uint32_t q_count, const uint32_t* __restrict__ kq,
                                                         const float* __restrict__ rq, uint32_t kmax,
                                                         uint32_t* __restrict__ nbr, float* __restrict__ dist,
                                                         uint32_t* __restrict__ cnt)
{
    __shared__ float tile[kKnnBlock * D];
    // heaviest blocks (largest prefixes) first
    const uint32_t blk = gridDim.x - 1 - blockIdx.x;
    const uint32_t q_end = min(n, q_first + q_count);  // this call's queries: q_first .. q_end-1
    const uint32_t q0 = q_first + blk * kKnnBlock;
    const uint32_t i = q0 + threadIdx.x;
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
    uint32_t c = 0;
    // a candidate must be within r and closer than the current k-th (when k are held)
    float worst = r;
    const uint32_t last = min(q_end, q0 + kKnnBlock);  // candidates 0 .. last-2 matter to this block
    for (uint32_t t0 = 0; t0 + 1 < last; t0 += kKnnBlock) {
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < kKnnBlock * D; e += kKnnBlock) {
            const size_t g = (size_t)t0 * D + e;
            tile[e] = (g < (size_t)n * D) ? V[g] : 0.0f;
        }
        __syncthreads();
        const uint32_t tn = min((uint32_t)kKnnBlock, last - 1 - t0);
        for (uint32_t u = 0; u < tn; ++u) {
            const uint32_t j = t0 + u;
            const float d = config_distance<D>(tile + u * D, me);
            // nn query semantics: distance <= r, strictly closer than the k-th to displace it
            const bool take = live && j < i && (c < k ? d <= worst : d < worst);
            if (__builtin_amdgcn_ballot_w64(take) == 0ull) continue;
            float cd = take ? d : __builtin_inff();
            uint32_t ci = take ? j : 0xFFFFFFFFu;
#pragma unroll
            for (int m = 0; m < K; ++m) {
                // insertion by compare-exchange on the key (distance, index): the carried element
                // displaced from an earlier slot must pass equal distances with larger indices
                const bool lt = cd < bd[m] || (cd == bd[m] && ci < bi[m]);
                const float td = bd[m];
                const uint32_t ti = bi[m];
                bd[m] = lt ? cd : td;
                bi[m] = lt ? ci : ti;
                cd = lt ? td : cd;
                ci = lt ? ti : ci;
            }
            if (take) {
                c = c < k ? c + 1 : c;
                // worst = the k-th distance once k are held (bd[k-1]), else r
                float kth = r;
#pragma unroll
                for (int m = 0; m < K; ++m)
                    if ((uint32_t)m + 1 == k) kth = bd[m];
                worst = (c == k) ? kth : r;
            }
        }
    }
    if (i < q_end) {  // outputs indexed from q_first
        const size_t o = i - q_first;
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

}  // namespace vgpu

template <int D, int K>
static void launch_knn(const float* V, uint32_t n, uint32_t qf, uint32_t qc, const uint32_t* k, const float* r,
                       uint32_t kmax, uint32_t* nbr, float* dist, uint32_t* cnt, hipStream_t st)
{
    const unsigned grid = (qc + vgpu::kKnnBlock - 1) / vgpu::kKnnBlock;
    hipLaunchKernelGGL((vgpu::knn_kernel<D, K>), dim3(grid), dim3(vgpu::kKnnBlock), 0, st, V, n, qf, qc, k, r, kmax,
                       nbr, dist, cnt);
}

template <int D>
static hipError_t knn_dim(const float* V, uint32_t n, uint32_t qf, uint32_t qc, const uint32_t* k, const float* r,
                          uint32_t kmax, uint32_t* nbr, float* dist, uint32_t* cnt, hipStream_t st)
{
    if (kmax <= 16)
        launch_knn<D, 16>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, st);
    else if (kmax <= 32)
        launch_knn<D, 32>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, st);
    else if (kmax <= 48)
        launch_knn<D, 48>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, st);
    else
        launch_knn<D, 64>(V, n, qf, qc, k, r, kmax, nbr, dist, cnt, st);
    return hipGetLastError();
}

extern "C" {

// kmax <= 64 and dim in {6, 7, 8, 14} (the robots built here) are checked by the caller
hipError_t vgpu_launch_roadmap_knn(int dim, const float* V, uint32_t n, uint32_t q_first, uint32_t q_count,
                                   const uint32_t* k, const float* r, uint32_t kmax, uint32_t* nbr, float* dist,
                                   uint32_t* cnt, hipStream_t st)
{
    if (q_count == 0) return hipSuccess;
    switch (dim) {
    case 6: return knn_dim<6>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, st);
    case 7: return knn_dim<7>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, st);
    case 8: return knn_dim<8>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, st);
    case 14: return knn_dim<14>(V, n, q_first, q_count, k, r, kmax, nbr, dist, cnt, st);
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

}  // extern "C"
