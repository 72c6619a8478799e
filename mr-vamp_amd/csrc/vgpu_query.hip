// vgpu_query.hip -- raw point-cloud queries: one lane per sphere against one CAPT of the
// environment ("raw sphere queries").
//   simd = 0: CAPT::collides(center, r) (collision/capt.hh:403-443): top-box distance test
//             against r^2, descent, leaf box against (r + r_point)^2 in the scalar Volume form
//             (fma(d2, d2, fma(d0, d0, d1*d1)), std::clamp), affordance scan;
//   simd = 1: one lane of CAPT::collides_simd (capt.hh:457-541), the form the fkcc path uses.
#include "vgpu_device.hh"

namespace vgpu {

__device__ __forceinline__ float std_clamp(float v, float lo, float hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

__device__ __forceinline__ float box_dist2_scalar(const float* b, float x, float y, float z)
{
    const float d0 = x - std_clamp(x, b[0], b[3]);
    const float d1 = y - std_clamp(y, b[1], b[4]);
    const float d2 = z - std_clamp(z, b[2], b[5]);
    return __builtin_fmaf(d2, d2, __builtin_fmaf(d0, d0, d1 * d1));
}

__device__ bool capt_scalar(const VGPU_CONST float* h, const float* __restrict__ base, float x, float y, float z,
                            float r)
{
    const float top[6] = {h[0], h[1], h[2], h[3], h[4], h[5]};
    if (box_dist2_scalar(top, x, y, z) > r * r) return false;
    const int nlog2 = (int)hdr_u(h, PC_NLOG2);
    const float* __restrict__ tests = base + hdr_u(h, PC_TESTS);
    uint32_t idx = 0;
    float a = x, b = y, c = z;
    for (int i = 0; i < nlog2; ++i) {
        idx = 2u * idx + 1u + ((a >= tests[idx]) ? 1u : 0u);
        const float t = a;
        a = b;
        b = c;
        c = t;
    }
    const uint32_t leaf = nlog2 ? idx - ((1u << nlog2) - 1u) : 0u;
    const float rr = r + h[PC_RPOINT];
    const float rsq = rr * rr;
    if (box_dist2_scalar(base + hdr_u(h, PC_AABBS) + 6u * leaf, x, y, z) > rsq) return false;
    const uint32_t* __restrict__ starts = (const uint32_t*)(base + hdr_u(h, PC_STARTS));
    const float4* __restrict__ aff = (const float4*)(base + hdr_u(h, PC_AFF));
    for (uint32_t i = starts[leaf], e = starts[leaf + 1]; i < e; ++i) {
        const float4* v = aff + 6u * i;
        const float4 x0 = v[0], x1 = v[1], y0 = v[2], y1 = v[3], z0 = v[4], z1 = v[5];
        const float px[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const float py[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
        const float pz[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
        bool any = false;
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const float dx = px[l] - x, dy = py[l] - y, dz = pz[l] - z;
            any |= __builtin_fmaf(dx, dx, __builtin_fmaf(dz, dz, dy * dy)) <= rsq;
        }
        if (any) return true;
    }
    return false;
}

__global__ __launch_bounds__(256) void capt_query_kernel(const float* __restrict__ centers,
                                                         const float* __restrict__ radii, size_t n, EnvView env,
                                                         int index, int simd, uint8_t* __restrict__ out)
{
    if (index == 0) capt_stage_lds(env);  // before any return: it ends in a barrier
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = centers[3 * i], y = centers[3 * i + 1], z = centers[3 * i + 2], r = radii[i];
    const VGPU_CONST float* h = env.pc + kExtHdr * index;
    out[i] = (simd ? capt_lane(h, env.base, x, y, z, r, index == 0 ? env.pc_lds_levels : 0)
                   : capt_scalar(h, env.base, x, y, z, r)) ? 1 : 0;
}

// filter_robot_from_pointcloud (bindings/common.hh:36-87): one lane per point.  sph = the robot's
// sphere_fk<1> output at the configuration, x[S] y[S] z[S], then the radii r[S] (staged in LDS, every
// lane reads the same sphere: broadcast).  A point is dropped when any robot sphere overlaps it -- the
// reference's SCALAR float sphere_sphere_sql2 < 0, as its release build computes it:
// fma(xs, xs, ys * ys) + fma(zs, zs, -(rs * rs)) (ref_probe "sql2s") -- or when it collides with the
// environment (the broadcast FloatVector sphere_environment_in_collision = one G = 1 lane).
constexpr int kFilterMaxSpheres = 128;
template <bool EXT>
__global__ __launch_bounds__(256) void filter_robot_kernel(const float* __restrict__ pc, size_t n, float pr,
                                                           const float* __restrict__ sph, int S, EnvView env,
                                                           uint8_t* __restrict__ keep)
{
    __shared__ float s[4 * kFilterMaxSpheres];
    for (int k = threadIdx.x; k < 4 * S; k += 256) s[k] = sph[k];
    if constexpr (EXT) capt_stage_lds(env);  // ends in a barrier (covers s[] as well)
    else __syncthreads();
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = pc[3 * i], y = pc[3 * i + 1], z = pc[3 * i + 2];
    bool hit = false;
    for (int k = 0; k < S; ++k) {
        const float xs = s[k] - x, ys = s[S + k] - y, zs = s[2 * S + k] - z, rs = s[3 * S + k] + pr;
        hit |= (__builtin_fmaf(xs, xs, ys * ys) + __builtin_fmaf(zs, zs, -(rs * rs))) < 0.0f;
    }
    if (!hit) hit = env_lane<Grp1, EXT>(env, x, y, z, pr);
    keep[i] = hit ? 0 : 1;
}

// rng::Halton<dim>::next draws first .. first + n - 1, one lane per draw (random/halton.hh:73-104)
__global__ __launch_bounds__(256) void halton_kernel(int dim, uint64_t first, size_t n, float* __restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t idx, cyc;
    halton_index(first + i, idx, cyc);
    for (int d = 0; d < dim; ++d) out[(size_t)dim * i + d] = halton_coord(idx, kHaltonPrimes[(d + cyc) % (uint32_t)dim]);
}

}  // namespace vgpu

extern "C" hipError_t vgpu_launch_halton(int dim, uint64_t first, size_t n, float* out, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(vgpu::halton_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dim, first, n, out);
    return hipGetLastError();
}

extern "C" hipError_t vgpu_launch_capt_query(const float* centers, const float* radii, size_t n, const EnvView* env,
                                             int index, int simd, uint8_t* out, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(vgpu::capt_query_kernel, dim3(grid), dim3(256), 0, st, centers, radii, n, *env, index, simd,
                       out);
    return hipGetLastError();
}

extern "C" hipError_t vgpu_launch_filter_robot(const float* pc, size_t n, float point_radius, const float* sph, int S,
                                               const EnvView* env, uint8_t* keep, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    if (S < 0 || S > vgpu::kFilterMaxSpheres) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (env->n_hf > 0 || env->n_pc > 0)
        hipLaunchKernelGGL(vgpu::filter_robot_kernel<true>, dim3(grid), dim3(256), 0, st, pc, n, point_radius, sph, S,
                           *env, keep);
    else
        hipLaunchKernelGGL(vgpu::filter_robot_kernel<false>, dim3(grid), dim3(256), 0, st, pc, n, point_radius, sph, S,
                           *env, keep);
    return hipGetLastError();
}
