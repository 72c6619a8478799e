// vgpu_staged.hip -- the staged collision hierarchy (vgpu_staged.hh) instantiated for the Panda
// (robots/panda_base.hh: 7 dof, 32 checks of panda/fk.hh:1335-6276, 32-bit check masks), plus
// the validate head -> tail back-step counts.
// part 0 (configurations, samples): no near-set children (their class-3 kernel as before round 6)
#if !defined(VGPU_PANDA_PART) || VGPU_PANDA_PART == 0
#define VGPU_NEAR_CHILDREN 0
#endif
#include "vgpu_panda.hh"
#include "vgpu_staged.hh"

// One translation unit per part of the source kinds (VGPU_PANDA_PART, compiled in parallel: one TU with every
// kind took ~18 min): part 0 = configurations + Halton samples (+ the head -> tail bookkeeping kernels),
// 1 = validate heads, 2 = validate tails, 3 = full-mask tails.  vgpu_api.cpp dispatches a kind to its part.
#ifndef VGPU_PANDA_PART
#define VGPU_PANDA_PART 0
#endif
#define VGPU_CAT_(a, b) a##b
#define VGPU_CAT(a, b) VGPU_CAT_(a, b)

// bound kernels: 86 VGPRs when unconstrained (Grp8 sources); at 7 waves/EU (72 VGPRs) they spilled
// 56 B/lane (~0.95 GB of scratch traffic per validate call), at 5 waves/EU none -- same speed on
// MI355X (A/B 3.31-3.40 vs 3.32-3.37 ms per 2^20-edge call), so the spill-free budget is the default
#ifndef VGPU_BOUND_WAVES_PER_EU
#define VGPU_BOUND_WAVES_PER_EU 5
#endif
// children classes (A/B on MI355X, 2^20 cage edges): class 0 at 8 waves/EU 1.5-3 % faster than 7;
// class 2 (checks 15, 21) at 6: 79 VGPRs since their children hold the link5 centres and stream the other
// link's (tools/gen_kernels.py HOLD; 105 VGPRs at 4 waves/EU before, A/B 3.50 -> 3.44 ms)
// bound stages that run the mid-sphere tests (vgpu_staged.hh MidBound, bit = SrcKindOf): the validate
// tails' (3, 4), whose bounding hits almost never confirm (tools/hitstats.py).  A/B on MI355X, two
// alternating runs (profiles/r04k_mid_ab.log): tails set B 2.40-2.42 ms vs none 2.57, set A and fkcc equal;
// head + tails: set A 1.94-1.96 vs 1.61-1.64 (head hits mostly confirm, so the mid tests are pure cost)
#ifndef VGPU_PANDA_MID_KINDS
#define VGPU_PANDA_MID_KINDS ((1u << 3) | (1u << 4))
#endif
#ifndef VGPU_PANDA_LEAD_WAVES
#define VGPU_PANDA_LEAD_WAVES 8  // 64 VGPRs, no spill (5, the bound stage budget: 67 VGPRs = 7 waves/EU; A/B set B 1.93-1.94 -> 1.90-1.91 ms)
#endif
#ifndef VGPU_PANDA_HEAD_LIST
#define VGPU_PANDA_HEAD_LIST 1
#endif
#ifndef VGPU_PANDA_CLASS0_WAVES
#define VGPU_PANDA_CLASS0_WAVES 8
#endif
#ifndef VGPU_PANDA_CLASS1_WAVES
#define VGPU_PANDA_CLASS1_WAVES 7
#endif
#ifndef VGPU_PANDA_CLASS3_WAVES
#define VGPU_PANDA_CLASS3_WAVES 6
#endif
#ifndef VGPU_PANDA_CLASS2_WAVES
#define VGPU_PANDA_CLASS2_WAVES 6
#endif

namespace vgpu {

struct PandaR {
    static constexpr int D = 7;
    static constexpr int kChecks = panda_n_checks;
    static constexpr int kWavesPerEU = VGPU_BOUND_WAVES_PER_EU;  // the bound kernels
#ifdef VGPU_CHILD_WAVES_PER_EU
    static constexpr int kChildWavesPerEU = VGPU_CHILD_WAVES_PER_EU;
#else
    static constexpr int kChildWavesPerEU = VGPU_WAVES_PER_EU;
#endif
    using Mask = panda_mask_t;
    static constexpr Mask kEnvChecks = panda_env_check_bits;
    static constexpr unsigned kSourceKinds = VGPU_PANDA_PART == 0 ? 0x3u : (0x4u << (VGPU_PANDA_PART - 1));
    // children register classes (ChildClasses): VGPRs per check when compiled alone (Grp8, gfx950):
    // most <= 49; 6, 7, 19, 20: 59-65; 15, 21: 90, 105
    // class 3 (round 6): the environment checks with near-set children (link 5: 12 children, hand: 18;
    // tools/gen_kernels.py NEAR_CHILDREN) -- their near code in the class-0 kernel spilled it at 8 waves/EU.  The
    // table is the same in every part: PandaR's members and R-only kernels (plan_kernel<PandaR>) are shared symbols
    // across the part TUs, so a per-part table broke the plan of the other parts (a 3-class part-0 table made the
    // heads miss collisions in tests/test_gpu_near.py)
    static constexpr int kClasses = 4;
    static constexpr int kClassOf[kChecks] = {0, 0, 0, 0, 0, 0, 1, 1, 3, 0, 0, 0, 0, 0, 0, 2,
                                              0, 3, 0, 1, 1, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // with a point cloud (CAPT) the near code is compiled out: link 5 and hand back in class 0 (a fourth kernel
    // there cost configs[2] 0.53 -> 0.555 ms per 2^20 configurations)
    static constexpr int kExtClasses = 3;
    static constexpr int kExtClassOf[kChecks] = {0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0, 2,
                                                 0, 0, 0, 1, 1, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    static constexpr int kClassWaves[kClasses] = {VGPU_PANDA_CLASS0_WAVES, VGPU_PANDA_CLASS1_WAVES,
                                                  VGPU_PANDA_CLASS2_WAVES, VGPU_PANDA_CLASS3_WAVES};
    __device__ static __forceinline__ void sample(uint64_t k, float v[7]) { panda_sample(k, v); }
    __device__ static __forceinline__ void head(const float* s, const float* g, int lane, float v[7])
    {
        const Rake rk = rake_setup(s, g);
        rake_block(s, rk, lane, 0, v);
    }
    __device__ static __forceinline__ void tail(const float* s, const float* g, int lane, int k, float v[7])
    {
        const Rake rk = rake_setup(s, g);
        rake_block(s, rk, lane, k, v);
    }
    // validate tails (SrcTailT, SrcTailMaskT) run the mid-sphere tests in their bound stage
    static constexpr uint32_t kMidKinds = VGPU_PANDA_MID_KINDS;
    template <class Grp, bool EXT, bool MID = false>
    __device__ static __forceinline__ Mask bound(const float* v, const EnvView& env, const Bases& b)
    {
        return panda_bound_mask<Grp, EXT, MID>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], env, b.x, b.y, b.z);
    }
    // the lead pass (vgpu_staged.hh lead_kernel): check 8, the link-5 environment check
    static constexpr int kLeadCheck = panda_lead_check;
    static constexpr int kLeadWaves = VGPU_PANDA_LEAD_WAVES;
    // after the lead pass, the heads' bound / children stages run over the compacted list of live edges
    static constexpr bool kHeadList = VGPU_PANDA_HEAD_LIST;
    template <class Grp>
    __device__ static __forceinline__ bool lead(const float* v, const EnvView& env, const Bases& b)
    {
        return panda_lead<Grp, false>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], env, b.x, b.y, b.z);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool children(int c, const float* v, const EnvView& env, const Bases& b)
    {
        return panda_children<Grp, EXT>(c, v[0], v[1], v[2], v[3], v[4], v[5], v[6], env, b.x, b.y, b.z);
    }
};

#if VGPU_PANDA_PART == 0
// validate head -> tail: back-step items for edges still valid after block 0
__global__ __launch_bounds__(kBlock) void tail_counts_kernel(const float* __restrict__ starts,
                                                             const float* __restrict__ goals, size_t n_edges,
                                                             const uint8_t* __restrict__ ok,
                                                             int32_t* __restrict__ n_blocks,
                                                             uint32_t* __restrict__ cnt)
{
    const size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n_edges) return;
    const Rake rk = rake_setup(starts + 7 * e, goals + 7 * e);
    if (n_blocks) n_blocks[e] = rk.n;
    cnt[e] = ((!ok || ok[e]) && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;  // ok = NULL: every back-step (full mask)
}

// full-mask mode: edge e's blocks at off[e] + e .. (+ n_e - 1); block 0 is the head's result, and the
// edge is valid when all of its blocks are
__global__ __launch_bounds__(kBlock) void mask_finish_kernel(size_t n_edges, const uint32_t* __restrict__ off,
                                                             uint8_t* __restrict__ ok, uint8_t* __restrict__ block_ok)
{
    const size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n_edges) return;
    const size_t base = (size_t)off[e] + e;
    const uint32_t nb = off[e + 1] - off[e] + 1u;
    uint8_t all = ok[e];
    block_ok[base] = all;
    for (uint32_t k = 1; k < nb; ++k) all &= block_ok[base + k];
    ok[e] = all;
}

#endif

}  // namespace vgpu

#define VGPU_STAGED_EXPORTS_X(R, NAME) VGPU_STAGED_EXPORTS(R, NAME)  // expands NAME before the pasting
VGPU_STAGED_EXPORTS_X(vgpu::PandaR, VGPU_CAT(panda_p, VGPU_PANDA_PART))

#ifdef VGPU_HITSTATS
// development statistics of the VGPU_HITSTATS variant: this part's counters
extern "C" int VGPU_CAT(VGPU_CAT(vgpu_panda_p, VGPU_PANDA_PART), _hitstats)(unsigned int* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vgpu::vgpu_hitstats), sizeof(vgpu::vgpu_hitstats)) != hipSuccess) return -2;
    if (reset) {
        static const unsigned int zero[5][64][2] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vgpu::vgpu_hitstats), zero, sizeof(zero)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

#if VGPU_PANDA_PART == 0

extern "C" hipError_t vgpu_launch_mask_finish(size_t n_edges, const uint32_t* off, uint8_t* ok, uint8_t* block_ok,
                                               hipStream_t st)
{
    if (n_edges == 0) return hipSuccess;
    const unsigned grid = (unsigned)((n_edges + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::mask_finish_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, n_edges, off, ok, block_ok);
    return hipGetLastError();
}

extern "C" hipError_t vgpu_launch_tail_counts(const float* starts, const float* goals, size_t n_edges,
                                              const uint8_t* ok, int32_t* n_blocks, uint32_t* cnt, hipStream_t st)
{
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess || n_edges == 0) return err;
    const unsigned grid = (unsigned)((n_edges + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::tail_counts_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, starts, goals, n_edges, ok,
                       n_blocks, cnt);
    return hipGetLastError();
}

#ifdef VGPU_HITSTATS
extern "C" int vgpu_panda_p1_hitstats(unsigned int*, int);
extern "C" int vgpu_panda_p2_hitstats(unsigned int*, int);
extern "C" int vgpu_panda_p3_hitstats(unsigned int*, int);
// development statistics of the VGPU_HITSTATS variant: out[5][64][2] (items, items with a children hit)
// per (source kind, check) since the last call, summed over the parts; reset = 1 zeroes them
extern "C" int vgpu_panda_hitstats(unsigned int* out, int reset)
{
    static unsigned int part[5][64][2];
    int (*fn[4])(unsigned int*, int) = {vgpu_panda_p0_hitstats, vgpu_panda_p1_hitstats, vgpu_panda_p2_hitstats,
                                        vgpu_panda_p3_hitstats};
    for (int i = 0; i < 5 * 64 * 2; ++i) out[i] = 0;
    for (auto f : fn) {
        if (int rc = f(&part[0][0][0], reset)) return rc;
        for (int i = 0; i < 5 * 64 * 2; ++i) out[i] += (&part[0][0][0])[i];
    }
    return 0;
}
#endif
#endif
