// vgpu_attach.hh -- the attachment rake for the robots whose fkcc_attach is a generated
// interleaved_sphere_fk_attachment of D <= 8 joints (Fetch: robots/fetch.hh:42, UR5:
// robots/ur5.hh:43).  R provides D, kRes and cc<Grp, EXT>(v, env) = <robot>_attach_fkcc.
// As for the Panda (vgpu_attach.hip): the first rake block of an edge only (validate.hh:43);
// the back-step blocks go through the robot's ordinary tail.
#pragma once

#include "vgpu_rake.hh"

namespace vgpu {

constexpr int kAttBlock = 256;

template <class R, bool EXT>
__global__ __launch_bounds__(kAttBlock, 4) void att_fkcc_kernel(const float* __restrict__ q, size_t n, EnvView env,
                                                                uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kAttBlock + threadIdx.x;
    if (i >= n) return;
    float v[R::D];
#pragma unroll
    for (int j = 0; j < R::D; ++j) v[j] = q[R::D * i + j];
    valid[i] = R::template cc<Grp1, EXT>(v, env) ? 1 : 0;
}

template <class R, bool EXT>
__global__ __launch_bounds__(kAttBlock, 4) void att_head_kernel(const float* __restrict__ starts,
                                                                const float* __restrict__ goals, size_t n_edges,
                                                                EnvView env, uint8_t* __restrict__ ok,
                                                                int32_t* __restrict__ n_blocks,
                                                                uint32_t* __restrict__ cnt)
{
    const size_t tid = (size_t)blockIdx.x * kAttBlock + threadIdx.x;
    const size_t e = tid >> 3;  // one 8-lane rake group per edge
    const int lane = (int)(tid & 7);
    if (e >= n_edges) return;   // group-uniform
    const float* s = starts + R::D * e;
    const RakeD<R::D> rk = rake_setup_d<R::D, R::kRes>(s, goals + R::D * e);
    float b[R::D];
    rake_block_d<R::D>(s, rk, lane, 0, b);  // block 0: fma(v, (lane+1)/8, s) (validate.hh:37)
    const bool valid = R::template cc<Grp8, EXT>(b, env);
    if (lane == 0) {
        ok[e] = valid ? 1 : 0;
        if (n_blocks) n_blocks[e] = rk.n;
        cnt[e] = (valid && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
    }
}

template <class R>
struct AttHost {
    static hipError_t fkcc(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st)
    {
        if (n == 0) return hipSuccess;
        const unsigned grid = (unsigned)((n + kAttBlock - 1) / kAttBlock);
        if (env->n_hf > 0 || env->n_pc > 0)
            hipLaunchKernelGGL((att_fkcc_kernel<R, true>), dim3(grid), dim3(kAttBlock), 0, st, q, n, *env, valid);
        else
            hipLaunchKernelGGL((att_fkcc_kernel<R, false>), dim3(grid), dim3(kAttBlock), 0, st, q, n, *env, valid);
        return hipGetLastError();
    }
    static hipError_t head(const float* starts, const float* goals, size_t n_edges, const EnvView* env, uint8_t* ok,
                           int32_t* n_blocks, uint32_t* cnt, hipStream_t st)
    {
        hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
        if (err != hipSuccess || n_edges == 0) return err;
        const unsigned grid = (unsigned)((n_edges * 8 + kAttBlock - 1) / kAttBlock);
        if (env->n_hf > 0 || env->n_pc > 0)
            hipLaunchKernelGGL((att_head_kernel<R, true>), dim3(grid), dim3(kAttBlock), 0, st, starts, goals, n_edges,
                               *env, ok, n_blocks, cnt);
        else
            hipLaunchKernelGGL((att_head_kernel<R, false>), dim3(grid), dim3(kAttBlock), 0, st, starts, goals, n_edges,
                               *env, ok, n_blocks, cnt);
        return hipGetLastError();
    }
};

}  // namespace vgpu
