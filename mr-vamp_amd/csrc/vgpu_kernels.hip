// vgpu_kernels.hip -- gfx950 kernels of the motion-validation rake.
//
// Three kernels per robot (Panda today):
//   sphere_fk   one lane per configuration, SoA stores: the HBM-bound FK stream
//               (reference robots/panda/fk.hh:104-1333 sphere_fk);
//   fkcc        one lane per configuration (rake group G = 1 == a configuration broadcast
//               to all 8 reference lanes): per-configuration validity mask
//               (fk.hh:1335-6276 interleaved_sphere_fk);
//   validate    one 8-lane group per edge (G = 8 == one reference rake block), looping over
//               the edge's back-steps with the reference's early exit
//               (planning/validate.hh:23-75).
// All three are VALU code: FK is 7 chained quaternion products + sparse 3x3 transforms,
// nothing here is a dense contraction worth MFMA (DESIGN.md "Why no MFMA").
#include "vgpu_device.hh"

#include "gen/panda_fk.inc"

namespace vgpu {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void panda_sphere_fk_kernel(const float* __restrict__ q, size_t n, float bx,
                                                                 float by, float bz, float* __restrict__ out,
                                                                 size_t ld)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float* qi = q + 7 * i;
    panda_sphere_fk_store(qi[0], qi[1], qi[2], qi[3], qi[4], qi[5], qi[6], bx, by, bz, out + i, ld);
}

__global__ __launch_bounds__(kBlock) void panda_fkcc_kernel(const float* __restrict__ q, size_t n, EnvView env,
                                                            float bx, float by, float bz,
                                                            uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float* qi = q + 7 * i;
    valid[i] = panda_fkcc<Grp1>(qi[0], qi[1], qi[2], qi[3], qi[4], qi[5], qi[6], env, bx, by, bz) ? 1 : 0;
}

// validate_vector (planning/validate.hh:23-65), rake = 8, resolution = 32 for the Panda.
__global__ __launch_bounds__(kBlock) void panda_validate_kernel(const float* __restrict__ starts,
                                                                const float* __restrict__ goals, size_t n_edges,
                                                                EnvView env, float bx, float by, float bz,
                                                                uint8_t* __restrict__ ok,
                                                                int32_t* __restrict__ n_blocks)
{
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t e = tid >> 3;       // one 8-lane rake group per edge
    const int lane = (int)(tid & 7);
    if (e >= n_edges) return;        // group-uniform
    const float* s = starts + 7 * e;
    const float* g = goals + 7 * e;
    float v[7], b[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) v[j] = g[j] - s[j];  // validate.hh:72
    // l2_norm in the AVX hsum lane order (vector/avx.hh:441-452), lane 7 padding = 0
    const float a = (v[0] * v[0] + v[4] * v[4]) + (v[2] * v[2] + v[6] * v[6]);
    const float c = (v[1] * v[1] + v[5] * v[5]) + (v[3] * v[3] + 0.0f);
    const float distance = __builtin_sqrtf(a + c);
    float nf = __builtin_ceilf(distance / 8.0f * 32.0f);  // validate.hh:41
    if (!(nf > 1.0f)) nf = 1.0f;
    const int n = (int)nf;
    const float pct = (float)(lane + 1) / 8.0f;  // validate.hh:11-21
#pragma unroll
    for (int j = 0; j < 7; ++j) b[j] = __builtin_fmaf(v[j], pct, s[j]);  // validate.hh:37 (contracted)
    const float div = (float)(8 * n);
    float back[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) back[j] = v[j] / div;  // validate.hh:50
    bool valid = true;
    for (int k = 0; k < n; ++k) {  // block 0, then n-1 back-steps (validate.hh:43-62)
        if (k > 0) {
#pragma unroll
            for (int j = 0; j < 7; ++j) b[j] = b[j] - back[j];
        }
        if (!panda_fkcc<Grp8>(b[0], b[1], b[2], b[3], b[4], b[5], b[6], env, bx, by, bz)) {
            valid = false;
            break;
        }
    }
    if (lane == 0) {
        ok[e] = valid ? 1 : 0;
        if (n_blocks) n_blocks[e] = n;
    }
}

}  // namespace vgpu

extern "C" {

hipError_t vgpu_launch_panda_sphere_fk(const float* q, size_t n, float bx, float by, float bz, float* out,
                                       size_t ld, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::panda_sphere_fk_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, q, n, bx, by, bz, out,
                       ld);
    return hipGetLastError();
}

hipError_t vgpu_launch_panda_fkcc(const float* q, size_t n, const EnvView* env, float bx, float by, float bz,
                                  uint8_t* valid, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::panda_fkcc_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, q, n, *env, bx, by, bz,
                       valid);
    return hipGetLastError();
}

hipError_t vgpu_launch_panda_validate(const float* starts, const float* goals, size_t n_edges, const EnvView* env,
                                      float bx, float by, float bz, uint8_t* ok, int32_t* n_blocks, hipStream_t st)
{
    if (n_edges == 0) return hipSuccess;
    const size_t threads = n_edges * 8;
    const unsigned grid = (unsigned)((threads + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::panda_validate_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, starts, goals, n_edges,
                       *env, bx, by, bz, ok, n_blocks);
    return hipGetLastError();
}

}  // extern "C"
