// vgpu_kernels.hip -- gfx950 kernels of the motion-validation rake.
//
// Per robot (Panda today; sphere_fk lives in vgpu_fk.hip):
//   fkcc           one lane per configuration (rake group G = 1 == a configuration broadcast
//                  to all 8 reference lanes): per-configuration validity mask
//                  (fk.hh:1335-6276 interleaved_sphere_fk);
//   validate       validate_motion over a batch of edges (planning/validate.hh:23-75) in two
//                  phases with the reference's early-exit semantics:
//                    head  one 8-lane group per edge evaluates the first rake block
//                          (t = 1/8 .. 8/8, validate.hh:31-44) and computes n_e;
//                    scan  edges that survive with n_e > 1 get n_e - 1 work items;
//                    tail  one 8-lane group per (edge, back-step k) evaluates block k,
//                          reached by the reference's k sequential subtractions
//                          (validate.hh:50-56), and clears the edge's flag on a hit.
//                  On collision-heavy scenes most invalid edges die in the head block
//                  (59.5 % of the bench edges, 0.06 % later), so the tail runs only for the
//                  survivors, and adjacent groups of the tail are neighbouring blocks of one
//                  edge (correlated branches).  The edge result equals the reference's
//                  sequential loop: it is the AND of its blocks.
// All of this is VALU code: FK is 7 chained quaternion products + sparse 3x3 transforms,
// nothing is a dense contraction worth MFMA (DESIGN.md "Why no MFMA").
#include <hipcub/hipcub.hpp>

#include "vgpu_panda.hh"

namespace vgpu {

template <bool EXT>
__global__ __launch_bounds__(kBlock, VGPU_WAVES_PER_EU) void panda_fkcc_kernel(const float* __restrict__ q, size_t n, EnvView env,
                                                            float bx, float by, float bz,
                                                            uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float* qi = q + 7 * i;
    valid[i] = panda_fkcc<Grp1, EXT>(qi[0], qi[1], qi[2], qi[3], qi[4], qi[5], qi[6], env, bx, by, bz) ? 1 : 0;
}

// ---- sampling: Halton<7> draw -> scale_configuration -> fkcc (prm.hh:236-251) ----
__global__ __launch_bounds__(kBlock) void panda_sample_kernel(uint64_t first, size_t n, float* __restrict__ q)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float v[7];
    panda_sample(first + i, v);
#pragma unroll
    for (int d = 0; d < 7; ++d) q[7 * i + d] = v[d];
}

template <bool EXT>
__global__ __launch_bounds__(kBlock, VGPU_WAVES_PER_EU) void panda_sample_fkcc_kernel(
    uint64_t first, size_t n, EnvView env, float bx, float by, float bz, float* __restrict__ q,
    uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float v[7];
    panda_sample(first + i, v);
    if (q) {
#pragma unroll
        for (int d = 0; d < 7; ++d) q[7 * i + d] = v[d];
    }
    valid[i] = panda_fkcc<Grp1, EXT>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], env, bx, by, bz) ? 1 : 0;
}

template <bool EXT>
__global__ __launch_bounds__(kBlock, VGPU_WAVES_PER_EU) void panda_validate_head_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, size_t n_edges, EnvView env, float bx,
    float by, float bz, uint8_t* __restrict__ ok, int32_t* __restrict__ n_blocks, uint32_t* __restrict__ cnt)
{
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t e = tid >> 3;  // one 8-lane rake group per edge
    const int lane = (int)(tid & 7);
    if (e >= n_edges) return;   // group-uniform
    const float* s = starts + 7 * e;
    const Rake rk = rake_setup(s, goals + 7 * e);
    const float pct = (float)(lane + 1) / 8.0f;  // validate.hh:11-21
    float b[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) b[j] = __builtin_fmaf(rk.v[j], pct, s[j]);  // validate.hh:37 (contracted)
    const bool valid = panda_fkcc<Grp8, EXT>(b[0], b[1], b[2], b[3], b[4], b[5], b[6], env, bx, by, bz);
    if (lane == 0) {
        ok[e] = valid ? 1 : 0;
        if (n_blocks) n_blocks[e] = rk.n;
        cnt[e] = (valid && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
    }
}

__global__ __launch_bounds__(kBlock) void gather_rows_kernel(const float* __restrict__ q, const uint32_t* __restrict__ idx,
                                                             const uint32_t* __restrict__ count, int dim,
                                                             float* __restrict__ out)
{
    const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t j = t / (size_t)dim;
    if (j >= *count) return;
    const int d = (int)(t - j * (size_t)dim);
    out[t] = q[(size_t)idx[j] * dim + d];
}

__global__ __launch_bounds__(kBlock) void scatter_items_kernel(const uint32_t* __restrict__ cnt,
                                                               const uint32_t* __restrict__ off, size_t n_edges,
                                                               uint32_t* __restrict__ item_edge)
{
    const size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n_edges) return;
    const uint32_t c = cnt[e], o = off[e];
    for (uint32_t i = 0; i < c; ++i) item_edge[o + i] = (uint32_t)e;
}

template <bool EXT>
__global__ __launch_bounds__(kBlock, VGPU_WAVES_PER_EU) void panda_validate_tail_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, const uint32_t* __restrict__ item_edge,
    const uint32_t* __restrict__ off, size_t n_items, EnvView env, float bx, float by, float bz,
    uint8_t* __restrict__ ok)
{
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t it = tid >> 3;  // one 8-lane rake group per (edge, back-step)
    const int lane = (int)(tid & 7);
    if (it >= n_items) return;   // group-uniform
    const uint32_t e = item_edge[it];
    const int k = (int)(it - off[e]) + 1;  // back-step index 1 .. n_e - 1
    const float* s = starts + 7 * (size_t)e;
    const Rake rk = rake_setup(s, goals + 7 * (size_t)e);
    const float pct = (float)(lane + 1) / 8.0f;
    const float div = (float)(8 * (size_t)rk.n);
    float b[7], back[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        b[j] = __builtin_fmaf(rk.v[j], pct, s[j]);
        back[j] = rk.v[j] / div;  // validate.hh:50
    }
    for (int i = 0; i < k; ++i) {  // the reference's sequential subtraction chain, bit for bit
#pragma unroll
        for (int j = 0; j < 7; ++j) b[j] = b[j] - back[j];
    }
    const bool valid = panda_fkcc<Grp8, EXT>(b[0], b[1], b[2], b[3], b[4], b[5], b[6], env, bx, by, bz);
    if (lane == 0 && !valid) ok[e] = 0;  // every writer stores 0: the race is benign
}

// 64-bit total of the per-edge back-step counts: the item scan is 32-bit, so a batch whose blocks
// exceed 2^32 must be rejected before its offsets are trusted (one atomic per wave)
__global__ __launch_bounds__(kBlock) void total64_kernel(const uint32_t* __restrict__ cnt, size_t n,
                                                         unsigned long long* __restrict__ out)
{
    unsigned long long s = 0;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) s += cnt[i];
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
    // one atomic per block: same-address atomics serialise in L2 (4096 of them took ~50 us)
    __shared__ unsigned long long part[kBlock / 64];
    if (__lane_id() == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += part[w];
        if (t) atomicAdd(out, t);
    }
}

}  // namespace vgpu

static bool has_ext(const EnvView* env) { return env->n_hf > 0 || env->n_pc > 0; }

extern "C" {

hipError_t vgpu_launch_panda_fkcc(const float* q, size_t n, const EnvView* env, float bx, float by, float bz,
                                  uint8_t* valid, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + vgpu::kBlock - 1) / vgpu::kBlock);
    if (has_ext(env))
        hipLaunchKernelGGL(vgpu::panda_fkcc_kernel<true>, dim3(grid), dim3(vgpu::kBlock), 0, st, q, n, *env, bx, by,
                           bz, valid);
    else
        hipLaunchKernelGGL(vgpu::panda_fkcc_kernel<false>, dim3(grid), dim3(vgpu::kBlock), 0, st, q, n, *env, bx, by,
                           bz, valid);
    return hipGetLastError();
}

hipError_t vgpu_launch_panda_sample(uint64_t first, size_t n, float* q, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::panda_sample_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, first, n, q);
    return hipGetLastError();
}

hipError_t vgpu_launch_panda_sample_fkcc(uint64_t first, size_t n, const EnvView* env, float bx, float by, float bz,
                                         float* q, uint8_t* valid, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + vgpu::kBlock - 1) / vgpu::kBlock);
    if (has_ext(env))
        hipLaunchKernelGGL(vgpu::panda_sample_fkcc_kernel<true>, dim3(grid), dim3(vgpu::kBlock), 0, st, first, n,
                           *env, bx, by, bz, q, valid);
    else
        hipLaunchKernelGGL(vgpu::panda_sample_fkcc_kernel<false>, dim3(grid), dim3(vgpu::kBlock), 0, st, first, n,
                           *env, bx, by, bz, q, valid);
    return hipGetLastError();
}

// Compaction of valid samples (the PRM vertex stage): out_q[j] = q[idx[j]], idx ascending.
size_t vgpu_compact_bytes(size_t n)
{
    size_t tmp = 0;
    (void)hipcub::DeviceSelect::Flagged(nullptr, tmp, hipcub::CountingInputIterator<uint32_t>(0),
                                        (const uint8_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    return tmp;
}

hipError_t vgpu_launch_gather_rows(const float* q, const uint32_t* idx, const uint32_t* count, size_t max_rows,
                                   int dim, float* out, hipStream_t st)
{
    if (max_rows == 0) return hipSuccess;
    const size_t threads = max_rows * (size_t)dim;
    const unsigned grid = (unsigned)((threads + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::gather_rows_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, q, idx, count, dim, out);
    return hipGetLastError();
}

hipError_t vgpu_launch_compact(const uint8_t* valid, size_t n, uint32_t* idx_out, uint32_t* count, void* tmp,
                               size_t tmp_bytes, hipStream_t st)
{
    return hipcub::DeviceSelect::Flagged(tmp, tmp_bytes, hipcub::CountingInputIterator<uint32_t>(0), valid, idx_out,
                                         count, (int)n, st);
}

// Workspace for the two-phase validate: cnt[n_edges + 1], off[n_edges + 1], scan temp.
size_t vgpu_validate_scan_bytes(size_t n_edges)
{
    size_t tmp = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (int)(n_edges + 1));
    return tmp;
}

hipError_t vgpu_launch_scan(const uint32_t* cnt, uint32_t* off, size_t n_edges, void* scan_tmp, size_t scan_bytes,
                            hipStream_t st)
{
    return hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, cnt, off, (int)(n_edges + 1), st);
}

hipError_t vgpu_launch_panda_validate_head(const float* starts, const float* goals, size_t n_edges,
                                           const EnvView* env, float bx, float by, float bz, uint8_t* ok,
                                           int32_t* n_blocks, uint32_t* cnt, hipStream_t st)
{
    const size_t threads = n_edges * 8;
    const unsigned grid = (unsigned)((threads + vgpu::kBlock - 1) / vgpu::kBlock);
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    if (has_ext(env))
        hipLaunchKernelGGL(vgpu::panda_validate_head_kernel<true>, dim3(grid), dim3(vgpu::kBlock), 0, st, starts,
                           goals, n_edges, *env, bx, by, bz, ok, n_blocks, cnt);
    else
        hipLaunchKernelGGL(vgpu::panda_validate_head_kernel<false>, dim3(grid), dim3(vgpu::kBlock), 0, st, starts,
                           goals, n_edges, *env, bx, by, bz, ok, n_blocks, cnt);
    return hipGetLastError();
}

hipError_t vgpu_launch_total64(const uint32_t* cnt, size_t n, unsigned long long* out, hipStream_t st)
{
    hipError_t err = hipMemsetAsync(out, 0, sizeof(unsigned long long), st);
    if (err != hipSuccess || n == 0) return err;
    const size_t want = (n + vgpu::kBlock - 1) / vgpu::kBlock;
    const unsigned grid = (unsigned)(want < 256 ? want : 256);
    hipLaunchKernelGGL(vgpu::total64_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, cnt, n, out);
    return hipGetLastError();
}

hipError_t vgpu_launch_scatter_items(const uint32_t* cnt, const uint32_t* off, size_t n_edges, uint32_t* item_edge,
                                     hipStream_t st)
{
    if (n_edges == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n_edges + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::scatter_items_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, cnt, off, n_edges,
                       item_edge);
    return hipGetLastError();
}

hipError_t vgpu_launch_panda_validate_tail(const float* starts, const float* goals, size_t n_edges,
                                           size_t n_items, const EnvView* env, float bx, float by, float bz,
                                           uint8_t* ok, const uint32_t* cnt, const uint32_t* off,
                                           uint32_t* item_edge, hipStream_t st)
{
    if (n_items == 0) return hipSuccess;
    unsigned grid = (unsigned)((n_edges + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::scatter_items_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, cnt, off, n_edges,
                       item_edge);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    const size_t threads = n_items * 8;
    grid = (unsigned)((threads + vgpu::kBlock - 1) / vgpu::kBlock);
    if (has_ext(env))
        hipLaunchKernelGGL(vgpu::panda_validate_tail_kernel<true>, dim3(grid), dim3(vgpu::kBlock), 0, st, starts,
                           goals, item_edge, off, n_items, *env, bx, by, bz, ok);
    else
        hipLaunchKernelGGL(vgpu::panda_validate_tail_kernel<false>, dim3(grid), dim3(vgpu::kBlock), 0, st, starts,
                           goals, item_edge, off, n_items, *env, bx, by, bz, ok);
    return hipGetLastError();
}

}  // extern "C"
