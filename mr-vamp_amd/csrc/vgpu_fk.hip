// vgpu_fk.hip -- the HBM-bound sphere_fk stream (reference robots/panda/fk.hh:104-1333).
//
// One lane per configuration: 7 joint loads, ~1.4k FLOP of FK, 177 coalesced SoA float stores
// (xyz[3][n_spheres][ld]) -- 736 algorithmic bytes per configuration, 1.8 FLOP/B, well under
// the ridge, so the roofline is HBM.  Built as its own translation unit WITH the SLP vectorizer
// (packed v_pk_* math: per-element IEEE results identical to the scalar ops), which the
// register-bound collision kernels in vgpu_kernels.hip are built without.
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

}  // extern "C"
