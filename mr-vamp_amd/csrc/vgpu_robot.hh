// vgpu_robot.hh -- the kernels of one generated robot (gen/<robot>_fk.inc), generic over a
// traits struct R, plus VGPU_ROBOT_EXPORTS(R, name) which emits `const RobotOps* vgpu_<name>_ops()`.
//
// R provides: D, kRes, kSpheres, kWavesPerEU, s_m/s_a (scale), fkcc<Grp, EXT>(v, env),
// sphere_fk_store(v, out, ld).  Same execution model as the Panda/Fetch TUs: one lane per
// configuration (rake group G = 1) for masks and sampling, one 8-lane DPP group per edge block
// for validate_motion in the two-phase head/tail split with the reference's early exit.
#pragma once

#include "vgpu_ops.hh"
#include "vgpu_rake.hh"

namespace vgpu {

constexpr int kRobotBlock = 256;

template <class R>
__global__ __launch_bounds__(kRobotBlock) void robot_sphere_fk_kernel(const float* __restrict__ q, size_t n,
                                                                      float* __restrict__ out, size_t ld)
{
    const size_t i = (size_t)blockIdx.x * kRobotBlock + threadIdx.x;
    if (i >= n) return;
    float v[R::D];
#pragma unroll
    for (int j = 0; j < R::D; ++j) v[j] = q[R::D * i + j];
    R::sphere_fk_store(v, out + i, ld);
}

template <class R, bool EXT>
__global__ __launch_bounds__(kRobotBlock, R::kWavesPerEU) void robot_fkcc_kernel(const float* __restrict__ q, size_t n,
                                                                                 EnvView env,
                                                                                 uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kRobotBlock + threadIdx.x;
    if (i >= n) return;
    float v[R::D];
#pragma unroll
    for (int j = 0; j < R::D; ++j) v[j] = q[R::D * i + j];
    valid[i] = R::template fkcc<Grp1, EXT>(v, env) ? 1 : 0;
}

template <class R>
__global__ __launch_bounds__(kRobotBlock) void robot_sample_kernel(uint64_t first, size_t n, float* __restrict__ q)
{
    const size_t i = (size_t)blockIdx.x * kRobotBlock + threadIdx.x;
    if (i >= n) return;
    float v[R::D];
    sample_d<R::D>(first + i, R::s_m, R::s_a, v);
#pragma unroll
    for (int j = 0; j < R::D; ++j) q[R::D * i + j] = v[j];
}

template <class R, bool EXT>
__global__ __launch_bounds__(kRobotBlock, R::kWavesPerEU) void robot_sample_fkcc_kernel(uint64_t first, size_t n,
                                                                                        EnvView env,
                                                                                        float* __restrict__ q,
                                                                                        uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kRobotBlock + threadIdx.x;
    if (i >= n) return;
    float v[R::D];
    sample_d<R::D>(first + i, R::s_m, R::s_a, v);
    if (q) {
#pragma unroll
        for (int j = 0; j < R::D; ++j) q[R::D * i + j] = v[j];
    }
    valid[i] = R::template fkcc<Grp1, EXT>(v, env) ? 1 : 0;
}

template <class R, bool EXT>
__global__ __launch_bounds__(kRobotBlock, R::kWavesPerEU) void robot_validate_head_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, size_t n_edges, EnvView env,
    uint8_t* __restrict__ ok, int32_t* __restrict__ n_blocks, uint32_t* __restrict__ cnt)
{
    const size_t tid = (size_t)blockIdx.x * kRobotBlock + threadIdx.x;
    const size_t e = tid >> 3;  // one 8-lane rake group per edge
    const int lane = (int)(tid & 7);
    if (e >= n_edges) return;   // group-uniform
    const float* s = starts + R::D * e;
    const RakeD<R::D> rk = rake_setup_d<R::D, R::kRes>(s, goals + R::D * e);
    float b[R::D];
    rake_block_d<R::D>(s, rk, lane, 0, b);
    const bool valid = R::template fkcc<Grp8, EXT>(b, env);
    if (lane == 0) {
        ok[e] = valid ? 1 : 0;
        if (n_blocks) n_blocks[e] = rk.n;
        cnt[e] = (valid && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
    }
}

template <class R, bool EXT>
__global__ __launch_bounds__(kRobotBlock, R::kWavesPerEU) void robot_validate_tail_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, const uint32_t* __restrict__ item_edge,
    const uint32_t* __restrict__ off, size_t n_items, EnvView env, uint8_t* __restrict__ ok)
{
    const size_t tid = (size_t)blockIdx.x * kRobotBlock + threadIdx.x;
    const size_t it = tid >> 3;
    const int lane = (int)(tid & 7);
    if (it >= n_items) return;
    const uint32_t e = item_edge[it];
    const int k = (int)(it - off[e]) + 1;
    const float* s = starts + R::D * (size_t)e;
    const RakeD<R::D> rk = rake_setup_d<R::D, R::kRes>(s, goals + R::D * (size_t)e);
    float b[R::D];
    rake_block_d<R::D>(s, rk, lane, k, b);
    const bool valid = R::template fkcc<Grp8, EXT>(b, env);
    if (lane == 0 && !valid) ok[e] = 0;  // every writer stores 0: the race is benign
}

template <class R>
__global__ __launch_bounds__(kRobotBlock) void robot_tail_counts_kernel(const float* __restrict__ starts,
                                                                        const float* __restrict__ goals, size_t n_edges,
                                                                        const uint8_t* __restrict__ ok,
                                                                        int32_t* __restrict__ n_blocks,
                                                                        uint32_t* __restrict__ cnt)
{
    const size_t e = (size_t)blockIdx.x * kRobotBlock + threadIdx.x;
    if (e >= n_edges) return;
    const RakeD<R::D> rk = rake_setup_d<R::D, R::kRes>(starts + R::D * e, goals + R::D * e);
    if (n_blocks) n_blocks[e] = rk.n;
    cnt[e] = (ok[e] && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
}

template <class R>
struct RobotHost {
    static unsigned grid(size_t threads) { return (unsigned)((threads + kRobotBlock - 1) / kRobotBlock); }
    static bool ext(const EnvView* env) { return env->n_hf > 0 || env->n_pc > 0; }

    static hipError_t sphere_fk(const float* q, size_t n, float* out, size_t ld, hipStream_t st)
    {
        if (n == 0) return hipSuccess;
        hipLaunchKernelGGL((robot_sphere_fk_kernel<R>), dim3(grid(n)), dim3(kRobotBlock), 0, st, q, n, out, ld);
        return hipGetLastError();
    }
    static hipError_t fkcc(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st)
    {
        if (n == 0) return hipSuccess;
        if (ext(env))
            hipLaunchKernelGGL((robot_fkcc_kernel<R, true>), dim3(grid(n)), dim3(kRobotBlock), 0, st, q, n, *env, valid);
        else
            hipLaunchKernelGGL((robot_fkcc_kernel<R, false>), dim3(grid(n)), dim3(kRobotBlock), 0, st, q, n, *env,
                               valid);
        return hipGetLastError();
    }
    static hipError_t sample(uint64_t first, size_t n, float* q, hipStream_t st)
    {
        if (n == 0) return hipSuccess;
        hipLaunchKernelGGL((robot_sample_kernel<R>), dim3(grid(n)), dim3(kRobotBlock), 0, st, first, n, q);
        return hipGetLastError();
    }
    static hipError_t sample_fkcc(uint64_t first, size_t n, const EnvView* env, float* q, uint8_t* valid,
                                  hipStream_t st)
    {
        if (n == 0) return hipSuccess;
        if (ext(env))
            hipLaunchKernelGGL((robot_sample_fkcc_kernel<R, true>), dim3(grid(n)), dim3(kRobotBlock), 0, st, first, n,
                               *env, q, valid);
        else
            hipLaunchKernelGGL((robot_sample_fkcc_kernel<R, false>), dim3(grid(n)), dim3(kRobotBlock), 0, st, first,
                               n, *env, q, valid);
        return hipGetLastError();
    }
    static hipError_t validate_head(const float* s, const float* g, size_t n_edges, const EnvView* env, uint8_t* ok,
                                    int32_t* n_blocks, uint32_t* cnt, hipStream_t st)
    {
        hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
        if (err != hipSuccess || n_edges == 0) return err;
        if (ext(env))
            hipLaunchKernelGGL((robot_validate_head_kernel<R, true>), dim3(grid(n_edges * 8)), dim3(kRobotBlock), 0, st,
                               s, g, n_edges, *env, ok, n_blocks, cnt);
        else
            hipLaunchKernelGGL((robot_validate_head_kernel<R, false>), dim3(grid(n_edges * 8)), dim3(kRobotBlock), 0,
                               st, s, g, n_edges, *env, ok, n_blocks, cnt);
        return hipGetLastError();
    }
    static hipError_t validate_tail(const float* s, const float* g, size_t n_items, const EnvView* env, uint8_t* ok,
                                    const uint32_t* off, const uint32_t* item_edge, hipStream_t st)
    {
        if (n_items == 0) return hipSuccess;
        if (ext(env))
            hipLaunchKernelGGL((robot_validate_tail_kernel<R, true>), dim3(grid(n_items * 8)), dim3(kRobotBlock), 0, st,
                               s, g, item_edge, off, n_items, *env, ok);
        else
            hipLaunchKernelGGL((robot_validate_tail_kernel<R, false>), dim3(grid(n_items * 8)), dim3(kRobotBlock), 0,
                               st, s, g, item_edge, off, n_items, *env, ok);
        return hipGetLastError();
    }
    static hipError_t tail_counts(const float* s, const float* g, size_t n_edges, const uint8_t* ok, int32_t* n_blocks,
                                  uint32_t* cnt, hipStream_t st)
    {
        hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
        if (err != hipSuccess || n_edges == 0) return err;
        hipLaunchKernelGGL((robot_tail_counts_kernel<R>), dim3(grid(n_edges)), dim3(kRobotBlock), 0, st, s, g, n_edges,
                           ok, n_blocks, cnt);
        return hipGetLastError();
    }
};

}  // namespace vgpu

#define VGPU_ROBOT_EXPORTS(R, NAME, STAGED)                                                                        \
    extern "C" const RobotOps* vgpu_##NAME##_ops(void)                                                             \
    {                                                                                                              \
        using H = vgpu::RobotHost<R>;                                                                              \
        static const RobotOps ops{R::D,           R::kRes,       R::kSpheres,      STAGED,           H::sphere_fk,   \
                                  H::fkcc,        H::sample,     H::sample_fkcc,   H::validate_head, H::validate_tail, \
                                  H::tail_counts};                                                                 \
        return &ops;                                                                                               \
    }
