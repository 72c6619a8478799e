// vgpu_fetch.hip -- gfx950 kernels for the Fetch (robots/fetch.hh: 8 dof, prismatic torso +
// 7 revolute joints, 111 spheres, 15 link checks + 48 self link pairs with 2586 child pairs).
//
// Same execution model as the Panda kernels (vgpu_kernels.hip): one lane per configuration
// for the mask (rake group G = 1, a configuration broadcast to the 8 reference lanes:
// prm.hh:246-249), one 8-lane DPP group per edge / back-step block for validate_motion, the
// two-phase head/tail split with the reference's early exit.  The check code is generated from
// model/fetch.json (tools/gen_kernels.py -> gen/fetch_fk.inc).  Fetch has no base offset.
#include "vgpu_rake.hh"

#include "gen/fetch_fk.inc"

#ifndef VGPU_FETCH_WAVES_PER_EU
#define VGPU_FETCH_WAVES_PER_EU 4
#endif

namespace vgpu {

constexpr int kFetchBlock = 256;
constexpr int kFetchDim = 8;
constexpr int kFetchRes = 32;  // robots/fetch.hh:13

#define FETCH_ARGS(v) v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]

__global__ __launch_bounds__(kFetchBlock) void fetch_sphere_fk_kernel(const float* __restrict__ q, size_t n,
                                                                      float* __restrict__ out, size_t ld)
{
    const size_t i = (size_t)blockIdx.x * kFetchBlock + threadIdx.x;
    if (i >= n) return;
    const float* qi = q + kFetchDim * i;
    fetch_sphere_fk_store(FETCH_ARGS(qi), 0.0f, 0.0f, 0.0f, out + i, ld);
}

template <bool EXT>
__global__ __launch_bounds__(kFetchBlock, VGPU_FETCH_WAVES_PER_EU) void fetch_fkcc_kernel(
    const float* __restrict__ q, size_t n, EnvView env, uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kFetchBlock + threadIdx.x;
    if (i >= n) return;
    const float* qi = q + kFetchDim * i;
    valid[i] = fetch_fkcc<Grp1, EXT>(FETCH_ARGS(qi), env, 0.0f, 0.0f, 0.0f) ? 1 : 0;
}

__global__ __launch_bounds__(kFetchBlock) void fetch_sample_kernel(uint64_t first, size_t n, float* __restrict__ q)
{
    const size_t i = (size_t)blockIdx.x * kFetchBlock + threadIdx.x;
    if (i >= n) return;
    float v[kFetchDim];
    sample_d<kFetchDim>(first + i, fetch_s_m, fetch_s_a, v);
#pragma unroll
    for (int d = 0; d < kFetchDim; ++d) q[kFetchDim * i + d] = v[d];
}

// PRM vertex stage (prm.hh:236-251): Halton<8> draw -> scale -> fkcc, fused
template <bool EXT>
__global__ __launch_bounds__(kFetchBlock, VGPU_FETCH_WAVES_PER_EU) void fetch_sample_fkcc_kernel(
    uint64_t first, size_t n, EnvView env, float* __restrict__ q, uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kFetchBlock + threadIdx.x;
    if (i >= n) return;
    float v[kFetchDim];
    sample_d<kFetchDim>(first + i, fetch_s_m, fetch_s_a, v);
    if (q) {
#pragma unroll
        for (int d = 0; d < kFetchDim; ++d) q[kFetchDim * i + d] = v[d];
    }
    valid[i] = fetch_fkcc<Grp1, EXT>(FETCH_ARGS(v), env, 0.0f, 0.0f, 0.0f) ? 1 : 0;
}

template <bool EXT>
__global__ __launch_bounds__(kFetchBlock, VGPU_FETCH_WAVES_PER_EU) void fetch_validate_head_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, size_t n_edges, EnvView env,
    uint8_t* __restrict__ ok, int32_t* __restrict__ n_blocks, uint32_t* __restrict__ cnt)
{
    const size_t tid = (size_t)blockIdx.x * kFetchBlock + threadIdx.x;
    const size_t e = tid >> 3;  // one 8-lane rake group per edge
    const int lane = (int)(tid & 7);
    if (e >= n_edges) return;   // group-uniform
    const float* s = starts + kFetchDim * e;
    const RakeD<kFetchDim> rk = rake_setup_d<kFetchDim, kFetchRes>(s, goals + kFetchDim * e);
    float b[kFetchDim];
    rake_block_d<kFetchDim>(s, rk, lane, 0, b);
    const bool valid = fetch_fkcc<Grp8, EXT>(FETCH_ARGS(b), env, 0.0f, 0.0f, 0.0f);
    if (lane == 0) {
        ok[e] = valid ? 1 : 0;
        if (n_blocks) n_blocks[e] = rk.n;
        cnt[e] = (valid && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
    }
}

template <bool EXT>
__global__ __launch_bounds__(kFetchBlock, VGPU_FETCH_WAVES_PER_EU) void fetch_validate_tail_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, const uint32_t* __restrict__ item_edge,
    const uint32_t* __restrict__ off, size_t n_items, EnvView env, uint8_t* __restrict__ ok)
{
    const size_t tid = (size_t)blockIdx.x * kFetchBlock + threadIdx.x;
    const size_t it = tid >> 3;  // one 8-lane rake group per (edge, back-step)
    const int lane = (int)(tid & 7);
    if (it >= n_items) return;   // group-uniform
    const uint32_t e = item_edge[it];
    const int k = (int)(it - off[e]) + 1;  // back-step index 1 .. n_e - 1
    const float* s = starts + kFetchDim * (size_t)e;
    const RakeD<kFetchDim> rk = rake_setup_d<kFetchDim, kFetchRes>(s, goals + kFetchDim * (size_t)e);
    float b[kFetchDim];
    rake_block_d<kFetchDim>(s, rk, lane, k, b);
    const bool valid = fetch_fkcc<Grp8, EXT>(FETCH_ARGS(b), env, 0.0f, 0.0f, 0.0f);
    if (lane == 0 && !valid) ok[e] = 0;  // every writer stores 0: the race is benign
}

}  // namespace vgpu

static bool fetch_has_ext(const EnvView* env) { return env->n_hf > 0 || env->n_pc > 0; }

static unsigned fetch_grid(size_t threads)
{
    return (unsigned)((threads + vgpu::kFetchBlock - 1) / vgpu::kFetchBlock);
}

extern "C" {

hipError_t vgpu_launch_fetch_sphere_fk(const float* q, size_t n, float* out, size_t ld, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(vgpu::fetch_sphere_fk_kernel, dim3(fetch_grid(n)), dim3(vgpu::kFetchBlock), 0, st, q, n, out,
                       ld);
    return hipGetLastError();
}

hipError_t vgpu_launch_fetch_fkcc(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    if (fetch_has_ext(env))
        hipLaunchKernelGGL(vgpu::fetch_fkcc_kernel<true>, dim3(fetch_grid(n)), dim3(vgpu::kFetchBlock), 0, st, q, n,
                           *env, valid);
    else
        hipLaunchKernelGGL(vgpu::fetch_fkcc_kernel<false>, dim3(fetch_grid(n)), dim3(vgpu::kFetchBlock), 0, st, q,
                           n, *env, valid);
    return hipGetLastError();
}

hipError_t vgpu_launch_fetch_sample(uint64_t first, size_t n, float* q, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(vgpu::fetch_sample_kernel, dim3(fetch_grid(n)), dim3(vgpu::kFetchBlock), 0, st, first, n, q);
    return hipGetLastError();
}

hipError_t vgpu_launch_fetch_sample_fkcc(uint64_t first, size_t n, const EnvView* env, float* q, uint8_t* valid,
                                         hipStream_t st)
{
    if (n == 0) return hipSuccess;
    if (fetch_has_ext(env))
        hipLaunchKernelGGL(vgpu::fetch_sample_fkcc_kernel<true>, dim3(fetch_grid(n)), dim3(vgpu::kFetchBlock), 0, st,
                           first, n, *env, q, valid);
    else
        hipLaunchKernelGGL(vgpu::fetch_sample_fkcc_kernel<false>, dim3(fetch_grid(n)), dim3(vgpu::kFetchBlock), 0,
                           st, first, n, *env, q, valid);
    return hipGetLastError();
}

hipError_t vgpu_launch_fetch_validate_head(const float* starts, const float* goals, size_t n_edges,
                                           const EnvView* env, uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                           hipStream_t st)
{
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess || n_edges == 0) return err;
    const unsigned grid = fetch_grid(n_edges * 8);
    if (fetch_has_ext(env))
        hipLaunchKernelGGL(vgpu::fetch_validate_head_kernel<true>, dim3(grid), dim3(vgpu::kFetchBlock), 0, st, starts,
                           goals, n_edges, *env, ok, n_blocks, cnt);
    else
        hipLaunchKernelGGL(vgpu::fetch_validate_head_kernel<false>, dim3(grid), dim3(vgpu::kFetchBlock), 0, st,
                           starts, goals, n_edges, *env, ok, n_blocks, cnt);
    return hipGetLastError();
}

hipError_t vgpu_launch_fetch_validate_tail(const float* starts, const float* goals, size_t n_items,
                                           const EnvView* env, uint8_t* ok, const uint32_t* off,
                                           const uint32_t* item_edge, hipStream_t st)
{
    if (n_items == 0) return hipSuccess;
    const unsigned grid = fetch_grid(n_items * 8);
    if (fetch_has_ext(env))
        hipLaunchKernelGGL(vgpu::fetch_validate_tail_kernel<true>, dim3(grid), dim3(vgpu::kFetchBlock), 0, st, starts,
                           goals, item_edge, off, n_items, *env, ok);
    else
        hipLaunchKernelGGL(vgpu::fetch_validate_tail_kernel<false>, dim3(grid), dim3(vgpu::kFetchBlock), 0, st,
                           starts, goals, item_edge, off, n_items, *env, ok);
    return hipGetLastError();
}

}  // extern "C"
