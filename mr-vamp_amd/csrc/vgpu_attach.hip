// vgpu_attach.hip -- the attachment path of the rake: Robot::fkcc_attach
// (robots/panda_base.hh:61-65 -> panda::interleaved_sphere_fk_attachment, panda/fk.hh:6278-11397).
// The reference runs it on the FIRST rake block of validate_motion only, when the environment
// carries an attachment (planning/validate.hh:43); every back-step block goes through plain fkcc,
// so the tail of an attached validate is the ordinary one (vgpu_api.cpp).
//   panda_attach_fkcc_kernel      one lane per configuration (G = 1, Robot::fkcc_attach)
//   panda_validate_head_att       one 8-lane group per edge: block 0 through fkcc_attach, n_e and
//                                 the back-step count, like panda_validate_head_kernel
// The attached spheres are posed per lane at the end-effector frame of the lane's own FK (the
// reference's set_attachment_pose, Attachment::pose) and read from the environment buffer with
// scalar loads (wave-uniform index).
#include "vgpu_panda.hh"
#include "gen/panda_attach_fk.inc"

namespace vgpu {

template <bool EXT>
__global__ __launch_bounds__(kBlock, 4) void panda_attach_fkcc_kernel(const float* __restrict__ q, size_t n,
                                                                      EnvView env, float bx, float by, float bz,
                                                                      uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float* qi = q + 7 * i;
    valid[i] = panda_attach_fkcc<Grp1, EXT>(qi[0], qi[1], qi[2], qi[3], qi[4], qi[5], qi[6], env, bx, by, bz) ? 1 : 0;
}

template <bool EXT>
__global__ __launch_bounds__(kBlock, 4) void panda_validate_head_att_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, size_t n_edges, EnvView env, float bx,
    float by, float bz, uint8_t* __restrict__ ok, int32_t* __restrict__ n_blocks, uint32_t* __restrict__ cnt)
{
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t e = tid >> 3;
    const int lane = (int)(tid & 7);
    if (e >= n_edges) return;  // group-uniform
    const float* s = starts + 7 * e;
    const Rake rk = rake_setup(s, goals + 7 * e);
    const float pct = (float)(lane + 1) / 8.0f;  // validate.hh:11-21
    float b[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) b[j] = __builtin_fmaf(rk.v[j], pct, s[j]);  // validate.hh:37
    const bool valid = panda_attach_fkcc<Grp8, EXT>(b[0], b[1], b[2], b[3], b[4], b[5], b[6], env, bx, by, bz);
    if (lane == 0) {
        ok[e] = valid ? 1 : 0;
        if (n_blocks) n_blocks[e] = rk.n;
        cnt[e] = (valid && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
    }
}

}  // namespace vgpu

static bool has_ext(const EnvView* env) { return env->n_hf > 0 || env->n_pc > 0; }

extern "C" {

hipError_t vgpu_launch_panda_fkcc_attach(const float* q, size_t n, const EnvView* env, float bx, float by, float bz,
                                         uint8_t* valid, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + vgpu::kBlock - 1) / vgpu::kBlock);
    if (has_ext(env))
        hipLaunchKernelGGL(vgpu::panda_attach_fkcc_kernel<true>, dim3(grid), dim3(vgpu::kBlock), 0, st, q, n, *env, bx,
                           by, bz, valid);
    else
        hipLaunchKernelGGL(vgpu::panda_attach_fkcc_kernel<false>, dim3(grid), dim3(vgpu::kBlock), 0, st, q, n, *env,
                           bx, by, bz, valid);
    return hipGetLastError();
}

hipError_t vgpu_launch_panda_validate_head_att(const float* starts, const float* goals, size_t n_edges,
                                               const EnvView* env, float bx, float by, float bz, uint8_t* ok,
                                               int32_t* n_blocks, uint32_t* cnt, hipStream_t st)
{
    const size_t threads = n_edges * 8;
    const unsigned grid = (unsigned)((threads + vgpu::kBlock - 1) / vgpu::kBlock);
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    if (has_ext(env))
        hipLaunchKernelGGL(vgpu::panda_validate_head_att_kernel<true>, dim3(grid), dim3(vgpu::kBlock), 0, st, starts,
                           goals, n_edges, *env, bx, by, bz, ok, n_blocks, cnt);
    else
        hipLaunchKernelGGL(vgpu::panda_validate_head_att_kernel<false>, dim3(grid), dim3(vgpu::kBlock), 0, st, starts,
                           goals, n_edges, *env, bx, by, bz, ok, n_blocks, cnt);
    return hipGetLastError();
}

}  // extern "C"
