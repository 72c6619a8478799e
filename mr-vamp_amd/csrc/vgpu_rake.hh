// vgpu_rake.hh -- validate_vector rake arithmetic (planning/validate.hh:23-75) for a
// configuration of D <= 8 joints (one AVX register in the reference), shared by the robot TUs
// that are not Panda (Panda keeps its tuned 7-joint copy in vgpu_panda.hh).
#pragma once

#include "vgpu_device.hh"

namespace vgpu {

template <int D>
struct RakeD {
    float v[D];
    int n;
};

// distance = l2_norm of goal - start (interface.hh:402-410): D <= 8 is one AVX register whose
// squares are summed in the hsum lane order ((l0+l4)+(l2+l6)) + ((l1+l5)+(l3+l7))
// (vector/avx.hh:441-452); D <= 16 is two registers lo/hi added lane-wise first, which the
// release build contracts to fma(lo, lo, hi * hi) (pinned by ref_probe "l2norm").  Padding
// lanes are 0.  n = max(ceil(d / 8 * resolution), 1) (validate.hh:41)
template <int D, int RES>
__device__ __forceinline__ RakeD<D> rake_setup_d(const float* __restrict__ s, const float* __restrict__ g)
{
    static_assert(D <= 16, "at most two AVX registers");
    RakeD<D> r;
#pragma unroll
    for (int j = 0; j < D; ++j) r.v[j] = g[j] - s[j];  // validate.hh:72
    float sq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float lo = j < D ? r.v[j < D ? j : 0] : 0.0f;
        if (D <= 8) {
            sq[j] = lo * lo;
        } else {
            const float hi = (j + 8 < D) ? r.v[(j + 8 < D) ? j + 8 : 0] : 0.0f;
            sq[j] = __builtin_fmaf(lo, lo, hi * hi);
        }
    }
    const float a = (sq[0] + sq[4]) + (sq[2] + sq[6]);
    const float c = (sq[1] + sq[5]) + (sq[3] + sq[7]);
    const float distance = __builtin_sqrtf(a + c);
    float nf = __builtin_ceilf(distance / 8.0f * (float)RES);
    if (!(nf > 1.0f)) nf = 1.0f;
    r.n = nf < 2147483520.0f ? (int)nf : 2147483520;
    return r;
}

// block k of an edge for rake lane `lane`: fma(v, (lane+1)/8, s) then k sequential back-step
// subtractions of v / (8 n) (validate.hh:37,50-56)
template <int D>
__device__ __forceinline__ void rake_block_d(const float* __restrict__ s, const RakeD<D>& rk, int lane, int k,
                                             float b[D])
{
    const float pct = (float)(lane + 1) / 8.0f;  // validate.hh:11-21
#pragma unroll
    for (int j = 0; j < D; ++j) b[j] = __builtin_fmaf(rk.v[j], pct, s[j]);
    if (k > 0) {
        const float div = (float)(8 * (size_t)rk.n);
        float back[D];
#pragma unroll
        for (int j = 0; j < D; ++j) back[j] = rk.v[j] / div;
        for (int i = 0; i < k; ++i) {
#pragma unroll
            for (int j = 0; j < D; ++j) b[j] = b[j] - back[j];
        }
    }
}

// Halton<D> draw k -> scale_configuration (q * s_m + s_a, one fma per joint)
template <int D>
__device__ __forceinline__ void sample_d(uint64_t k, const float* s_m, const float* s_a, float q[D])
{
    uint32_t idx, cyc;
    halton_index(k, idx, cyc);
#pragma unroll
    for (int d = 0; d < D; ++d)
        q[d] = __builtin_fmaf(halton_coord(idx, kHaltonPrimes[(d + cyc) % (uint32_t)D]), s_m[d], s_a[d]);
}

}  // namespace vgpu
