// vgpu_fetch_staged.hip -- the staged collision hierarchy (vgpu_staged.hh) instantiated for the
// Fetch (robots/fetch.hh: 8 dof, 63 checks of fetch/fk.hh:1461-16079 incl. one leaf, 64-bit check
// masks), plus the Fetch validate head -> tail back-step counts.
#include "vgpu_rake.hh"
#include "vgpu_staged.hh"

#include "gen/fetch_fk.inc"

// One translation unit per part of the source kinds (VGPU_FETCH_PART, compiled in parallel: one TU with every
// kind took 12.5 min): part 0 = configurations + Halton samples (+ the tail counts), 1 = validate heads,
// 2 = validate tails, 3 = full-mask tails.  vgpu_api.cpp dispatches a kind to its part's exports.
#ifndef VGPU_FETCH_PART
#define VGPU_FETCH_PART 0
#endif
#define VGPU_CAT_(a, b) a##b
#define VGPU_CAT(a, b) VGPU_CAT_(a, b)

#ifndef VGPU_FETCH_STAGED_WAVES_PER_EU
#define VGPU_FETCH_STAGED_WAVES_PER_EU 6
#endif
// bound kernels of the validate head / tail (8-lane groups): at 6 waves/EU they spilled (r04 PMC of the
// configs[3] edge stage: 0.5 TB of scratch writes per 2.68M-vertex step)
#ifndef VGPU_FETCH_BOUND8_WAVES
#define VGPU_FETCH_BOUND8_WAVES 4
#endif
// children register classes (ChildClasses, vgpu_staged.hh) from the VGPRs each check's children kernel needs
// compiled alone (tools/probe_children_vgprs.py, gfx950, validate tails): <= 56 for 48 checks; 60-66 for
// checks 9, 10, 17, 20, 24, 26, 27, 33, 42, 48, 51, 56, 59; 73 for check 8; 90 for check 23.  Each class runs
// at an occupancy whose budget holds it in the full kernel -- which needs more than the check compiled alone:
// at 64 / 72 VGPRs classes 0 and 1 still spilled 4-63 VGPRs, at 96 / 128 (5 / 4 waves) none do (at 80 the
// validate-head kernel of class 0 still spilled 3; tests/test_kernel_resources.py).  A/B on MI355X
// (profiles/r05e_ab.log: 8/7 vs 6/5 vs 6/4 waves): edge stage 2.68M vertices 777 / 783 / 784 ms, validate
// 1.30 / 1.29 / 1.31 ms -- within a percent, and no scratch traffic.  With point clouds (EXT) classes 0 and 1
// need one wave/EU less again (kExtClassWaves)
#ifndef VGPU_FETCH_CLASS0_WAVES
#define VGPU_FETCH_CLASS0_WAVES 5
#endif
#ifndef VGPU_FETCH_CLASS1_WAVES
#define VGPU_FETCH_CLASS1_WAVES 4
#endif
#ifndef VGPU_FETCH_CLASS2_WAVES
#define VGPU_FETCH_CLASS2_WAVES 6
#endif
#ifndef VGPU_FETCH_CLASS3_WAVES
#define VGPU_FETCH_CLASS3_WAVES 5
#endif

// source kinds whose bound stage runs the mid-sphere tests (vgpu_staged.hh MidKinds; tools/gen_kernels.py
// MID_SELF_CHECKS: the head / base / torso vs arm self checks whose validate-tail items almost never confirm):
// validate heads and tails.  A/B on MI355X (profiles/r05h_ab.log): edge stage at 2.68M vertices, validation
// 424 -> 384 ms with tails only, 371 ms with heads too; 100k vertices 24.6 -> 22.3 ms; sampler unchanged
#ifndef VGPU_FETCH_MID_KINDS
#define VGPU_FETCH_MID_KINDS ((1u << 2) | (1u << 3) | (1u << 4))
#endif

namespace vgpu {

struct FetchR {
    static constexpr int D = 8;
    static constexpr int kRes = 32;  // robots/fetch.hh:13
    static constexpr int kChecks = fetch_n_checks;
    static constexpr int kWavesPerEU = VGPU_FETCH_STAGED_WAVES_PER_EU;
    static constexpr int kBoundWaves8 = VGPU_FETCH_BOUND8_WAVES;
    static constexpr int kExtBoundWaves = 3;  // point-cloud bound kernels (vgpu_staged.hh BoundWavesE)
    static constexpr int kChildWavesPerEU = VGPU_FETCH_STAGED_WAVES_PER_EU;
    using Mask = fetch_mask_t;
    static constexpr Mask kEnvChecks = fetch_env_check_bits;
    static constexpr unsigned kSourceKinds = VGPU_FETCH_PART == 0 ? 0x3u : (0x4u << (VGPU_FETCH_PART - 1));
    static constexpr int kClasses = 4;
    static constexpr int kClassOf[kChecks] = {0, 0, 0, 0, 0, 0, 0, 0, 2, 1, 1, 0, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 3, 1, 0, 1, 1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 0};
    static constexpr int kClassWaves[kClasses] = {VGPU_FETCH_CLASS0_WAVES, VGPU_FETCH_CLASS1_WAVES,
                                                  VGPU_FETCH_CLASS2_WAVES, VGPU_FETCH_CLASS3_WAVES};
    static constexpr int kExtClassWaves[kClasses] = {4, 3, 5, 5};
    static constexpr uint32_t kMidKinds = VGPU_FETCH_MID_KINDS;
    __device__ static __forceinline__ void sample(uint64_t k, float v[8]) { sample_d<8>(k, fetch_s_m, fetch_s_a, v); }
    __device__ static __forceinline__ void head(const float* s, const float* g, int lane, float v[8])
    {
        const RakeD<8> rk = rake_setup_d<8, kRes>(s, g);
        rake_block_d<8>(s, rk, lane, 0, v);
    }
    __device__ static __forceinline__ void tail(const float* s, const float* g, int lane, int k, float v[8])
    {
        const RakeD<8> rk = rake_setup_d<8, kRes>(s, g);
        rake_block_d<8>(s, rk, lane, k, v);
    }
    template <class Grp, bool EXT, bool MID = false>
    __device__ static __forceinline__ Mask bound(const float* v, const EnvView& env, const Bases&)
    {
        return fetch_bound_mask<Grp, EXT, MID>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], env, 0.0f, 0.0f, 0.0f);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool children(int c, const float* v, const EnvView& env, const Bases&)
    {
        return fetch_children<Grp, EXT>(c, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], env, 0.0f, 0.0f, 0.0f);
    }
};

#if VGPU_FETCH_PART == 0
__global__ __launch_bounds__(kStagedBlock) void fetch_tail_counts_kernel(const float* __restrict__ starts,
                                                                         const float* __restrict__ goals,
                                                                         size_t n_edges,
                                                                         const uint8_t* __restrict__ ok,
                                                                         int32_t* __restrict__ n_blocks,
                                                                         uint32_t* __restrict__ cnt)
{
    const size_t e = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    if (e >= n_edges) return;
    const RakeD<8> rk = rake_setup_d<8, FetchR::kRes>(starts + 8 * e, goals + 8 * e);
    if (n_blocks) n_blocks[e] = rk.n;
    cnt[e] = (ok[e] && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
}

#endif

}  // namespace vgpu

#define VGPU_STAGED_EXPORTS_X(R, NAME) VGPU_STAGED_EXPORTS(R, NAME)  // expands NAME before the pasting
VGPU_STAGED_EXPORTS_X(vgpu::FetchR, VGPU_CAT(fetch_p, VGPU_FETCH_PART))

#ifdef VGPU_HITSTATS
// development statistics of the VGPU_HITSTATS variant: this part's counters (each part has its own copy of
// vgpu_hitstats; its kinds' rows are the only ones it writes)
extern "C" int VGPU_CAT(VGPU_CAT(vgpu_fetch_p, VGPU_FETCH_PART), _hitstats)(unsigned int* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vgpu::vgpu_hitstats), sizeof(vgpu::vgpu_hitstats)) != hipSuccess) return -2;
    if (reset) {
        static const unsigned int zero[5][64][2] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vgpu::vgpu_hitstats), zero, sizeof(zero)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

#if VGPU_FETCH_PART == 0

#ifdef VGPU_HITSTATS
extern "C" int vgpu_fetch_p1_hitstats(unsigned int*, int);
extern "C" int vgpu_fetch_p2_hitstats(unsigned int*, int);
extern "C" int vgpu_fetch_p3_hitstats(unsigned int*, int);
// the Fetch passes' counters, laid out as vgpu_panda_hitstats's: the sum over the parts
extern "C" int vgpu_fetch_hitstats(unsigned int* out, int reset)
{
    static unsigned int part[5][64][2];
    int (*fn[4])(unsigned int*, int) = {vgpu_fetch_p0_hitstats, vgpu_fetch_p1_hitstats, vgpu_fetch_p2_hitstats,
                                        vgpu_fetch_p3_hitstats};
    for (int i = 0; i < 5 * 64 * 2; ++i) out[i] = 0;
    for (auto f : fn) {
        if (int rc = f(&part[0][0][0], reset)) return rc;
        for (int i = 0; i < 5 * 64 * 2; ++i) out[i] += (&part[0][0][0])[i];
    }
    return 0;
}
#endif

extern "C" hipError_t vgpu_launch_fetch_tail_counts(const float* starts, const float* goals, size_t n_edges,
                                                    const uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                                    hipStream_t st)
{
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess || n_edges == 0) return err;
    const unsigned grid = (unsigned)((n_edges + vgpu::kStagedBlock - 1) / vgpu::kStagedBlock);
    hipLaunchKernelGGL(vgpu::fetch_tail_counts_kernel, dim3(grid), dim3(vgpu::kStagedBlock), 0, st, starts, goals,
                       n_edges, ok, n_blocks, cnt);
    return hipGetLastError();
}
#endif
