// vgpu_panda.hh -- Panda device code shared by the kernel TUs: the generated FK / check
// functions, the validate_motion rake arithmetic and the Halton sampling step.
#pragma once

#include "vgpu_device.hh"

#ifdef VGPU_FK_INC  // A/B builds of alternative generated code
#include VGPU_FK_INC
#else
#include "gen/panda_fk.inc"
#endif

#ifndef VGPU_WAVES_PER_EU
#define VGPU_WAVES_PER_EU 7  // A/B on MI355X: 4 -> 6.84 ms, 6 -> 5.96, 7 -> 5.84, 8 -> 5.96 (validate, 1M edges)
#endif

namespace vgpu {

constexpr int kBlock = 256;

// ---- sampling: Halton<7> draw -> scale_configuration -> fkcc (prm.hh:236-251) ----
__device__ __forceinline__ void panda_sample(uint64_t k, float q[7])
{
    uint32_t idx, cyc;
    halton_index(k, idx, cyc);
#pragma unroll
    for (int d = 0; d < 7; ++d)
        q[d] = __builtin_fmaf(halton_coord(idx, kHaltonPrimes[(d + cyc) % 7u]), panda_s_m[d], panda_s_a[d]);
}

// ---- validate_vector: shared rake arithmetic (validate.hh:31-50) ----------------------------
struct Rake {
    float v[7];
    int n;
};

__device__ __forceinline__ Rake rake_setup(const float* __restrict__ s, const float* __restrict__ g)
{
    Rake r;
#pragma unroll
    for (int j = 0; j < 7; ++j) r.v[j] = g[j] - s[j];  // validate.hh:72
    // l2_norm in the AVX hsum lane order (vector/avx.hh:441-452); lane 7 is padding 0
    const float a = (r.v[0] * r.v[0] + r.v[4] * r.v[4]) + (r.v[2] * r.v[2] + r.v[6] * r.v[6]);
    const float c = (r.v[1] * r.v[1] + r.v[5] * r.v[5]) + (r.v[3] * r.v[3] + 0.0f);
    const float distance = __builtin_sqrtf(a + c);
    float nf = __builtin_ceilf(distance / 8.0f * 32.0f);  // validate.hh:41
    if (!(nf > 1.0f)) nf = 1.0f;
    r.n = nf < 2147483520.0f ? (int)nf : 2147483520;
    return r;
}


// block k of an edge for rake lane `lane`: block 0 = fma(v, (lane+1)/8, s) (validate.hh:37,
// contracted), then the reference's k sequential back-step subtractions (validate.hh:50-56)
__device__ __forceinline__ void rake_block(const float* __restrict__ s, const Rake& rk, int lane, int k, float b[7])
{
    const float pct = (float)(lane + 1) / 8.0f;  // validate.hh:11-21
#pragma unroll
    for (int j = 0; j < 7; ++j) b[j] = __builtin_fmaf(rk.v[j], pct, s[j]);
    if (k > 0) {
        const float div = (float)(8 * (size_t)rk.n);
        float back[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) back[j] = rk.v[j] / div;  // validate.hh:50
        for (int i = 0; i < k; ++i) {
#pragma unroll
            for (int j = 0; j < 7; ++j) b[j] = b[j] - back[j];
        }
    }
}

}  // namespace vgpu
