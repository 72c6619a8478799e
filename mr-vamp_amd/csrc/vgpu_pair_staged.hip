// vgpu_pair_staged.hip -- the two-Panda composite of BASELINE configs[4] through the staged pipeline
// (vgpu_staged.hh).  Validity = fkcc_A && fkcc_B && !inter(A, B) (oracle/vamp_oracle.c
// vo_pair_fkcc_block), an AND of three ORs over checks, so it runs as CHAINED staged passes over the
// same groups, each with its own bound -> count -> queue -> children stages and <= 64 checks:
//   pair_a    arm A's 32 Panda checks (panda/fk.hh:1335-6276) on joints 0..6 at base A
//   pair_b    arm B's 32 checks on joints 7..13 at base B (groups invalid after pair_a skip)
//   pair_i0   inter-arm link-bounding pairs 0..63 (gen/panda_pair_staged.inc, link-major order)
//   pair_i1   inter-arm pairs 64..120
// Every pass recomputes the frames it needs (lazily: a pass only evaluates its own links).  The
// 14-dof rake (two AVX registers, pinned l2_norm) feeds the head and tail sources.
#include "vgpu_rake.hh"
#include "vgpu_staged.hh"

#include "gen/panda_fk.inc"
#include "gen/panda_pair_staged.inc"

#ifndef VGPU_PAIR_BOUND_WAVES
#define VGPU_PAIR_BOUND_WAVES 5  // the arm passes' bound kernels
#endif
// the inter-arm passes' bound kernels over single configurations (fkcc): the second chunk spilled 5 VGPRs at 5
#ifndef VGPU_PAIR_INTER_BOUND_WAVES
#define VGPU_PAIR_INTER_BOUND_WAVES 4
#endif
// the inter-arm passes' bound kernels over 8-lane rake groups (validate head / tail): both arms' link
// frames are live at once -- 176 B/lane of scratch at 5 waves/EU, 12 B at 4 (128 VGPRs), none at 3
// (132); A/B on MI355X (2^20 composite edges, 2 x 2 alternating): 4 waves 10.58-10.68 ms, 3 waves
// 10.72-10.77 (profiles/r04d_pair_ab.log).  Round 5: 3, spill-free (tests/test_kernel_resources.py)
#ifndef VGPU_PAIR_INTER_BOUND8_WAVES
#define VGPU_PAIR_INTER_BOUND8_WAVES 3
#endif
// inter-arm children: both links' frames plus the held side's sphere centres (up to 30 spheres) -- 136-227
// VGPRs spilled at 6 waves/EU (80 VGPRs); they run only for the rare groups whose inter-arm bounding pairs
// overlap, so they get the registers (2 waves/EU, 256 VGPRs) rather than scratch
#ifndef VGPU_PAIR_INTER_WAVES
#define VGPU_PAIR_INTER_WAVES 2
#endif
#ifndef VGPU_PAIR_BOTH
#define VGPU_PAIR_BOTH 1
#endif
// source kinds whose arm-pass bound stage runs the mid-sphere tests (vgpu_staged.hh MidKinds): validate tails, as
// for the single Panda.  A/B on MI355X (profiles/r05m_pair_ab.log, three alternating runs): 8.50-8.60 -> 7.99-8.09
// ms per 2^20 composite edges
#ifndef VGPU_PAIR_MID_KINDS
#define VGPU_PAIR_MID_KINDS ((1u << 3) | (1u << 4))
#endif
// the combined chunks' bound kernel over 8-lane rake groups (both arms' link centres, 121 tests): it uses 94 VGPRs
// (5 waves/EU).  A/B on MI355X (profiles/r05l_pair_ab.log): forced to 6 or 7 waves it runs 8.16-8.23 vs 8.51-8.55
// ms per composite step but spills 11-26 VGPRs; holding arm A's centres in halves (arm B's FK streamed, and
// both recomputed, per half) still spilled 3-8 at 6 waves -- kept at 5, spill-free
#ifndef VGPU_PAIR_BOTH8_WAVES
#define VGPU_PAIR_BOTH8_WAVES 3
#endif

namespace vgpu {

constexpr int kPairDimS = 14;
constexpr int kPairResS = 32;  // robots/panda_base.hh:21

struct PairRakeR {  // the composite's rake blocks (validate.hh:23-56 over 14 dof)
    static constexpr int D = kPairDimS;
    static constexpr unsigned kSourceKinds = 1u | 4u | 8u;  // configurations, validate head, validate tail
    __device__ static __forceinline__ void sample(uint64_t, float v[D])
    {
#pragma unroll
        for (int j = 0; j < D; ++j) v[j] = 0.0f;  // never instantiated (kSourceKinds)
    }
    __device__ static __forceinline__ void head(const float* s, const float* g, int lane, float v[D])
    {
        const RakeD<D> rk = rake_setup_d<D, kPairResS>(s, g);
        rake_block_d<D>(s, rk, lane, 0, v);
    }
    __device__ static __forceinline__ void tail(const float* s, const float* g, int lane, int k, float v[D])
    {
        const RakeD<D> rk = rake_setup_d<D, kPairResS>(s, g);
        rake_block_d<D>(s, rk, lane, k, v);
    }
};

// one arm's Panda hierarchy; ARM 0 = joints 0..6 at (x, y, z), ARM 1 = joints 7..13 at (x2, y2, z2)
template <int ARM>
struct PairArmR : PairRakeR {
    static constexpr int kChecks = panda_n_checks;
    static constexpr int kWavesPerEU = VGPU_PAIR_BOUND_WAVES;
    static constexpr int kChildWavesPerEU = 7;
    using Mask = panda_mask_t;
    static constexpr Mask kEnvChecks = panda_env_check_bits;
    // the Panda's children register classes (vgpu_staged.hip PandaR)
    static constexpr int kClasses = 4;
    static constexpr int kClassOf[kChecks] = {0, 0, 0, 0, 0, 0, 1, 1, 3, 0, 0, 0, 0, 0, 0, 2,
                                              0, 3, 0, 1, 1, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // with a point cloud (CAPT) the near code is compiled out: link 5 and hand back in class 0 (a fourth kernel
    // there cost configs[2] 0.53 -> 0.555 ms per 2^20 configurations)
    static constexpr int kExtClasses = 3;
    static constexpr int kExtClassOf[kChecks] = {0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0, 2,
                                                 0, 0, 0, 1, 1, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    static constexpr int kClassWaves[kClasses] = {8, 7, 6, 6};
    // validate tails run the Panda's mid-sphere tests in their bound stage, as the single Panda does
    // (vgpu_staged.hip PandaR::kMidKinds)
    static constexpr uint32_t kMidKinds = VGPU_PAIR_MID_KINDS;
    template <class Grp, bool EXT, bool MID = false>
    __device__ static __forceinline__ Mask bound(const float* v, const EnvView& env, const Bases& b)
    {
        constexpr int o = 7 * ARM;
        return ARM == 0 ? panda_bound_mask<Grp, EXT, MID>(v[o], v[o + 1], v[o + 2], v[o + 3], v[o + 4], v[o + 5],
                                                           v[o + 6], env, b.x, b.y, b.z)
                        : panda_bound_mask<Grp, EXT, MID>(v[o], v[o + 1], v[o + 2], v[o + 3], v[o + 4], v[o + 5],
                                                           v[o + 6], env, b.x2, b.y2, b.z2);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool children(int c, const float* v, const EnvView& env, const Bases& b)
    {
        constexpr int o = 7 * ARM;
        return ARM == 0 ? panda_children<Grp, EXT>(c, v[o], v[o + 1], v[o + 2], v[o + 3], v[o + 4], v[o + 5],
                                                   v[o + 6], env, b.x, b.y, b.z)
                        : panda_children<Grp, EXT>(c, v[o], v[o + 1], v[o + 2], v[o + 3], v[o + 4], v[o + 5],
                                                   v[o + 6], env, b.x2, b.y2, b.z2);
    }
};

#define PAIR_Q(v) v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], v[11], v[12], v[13]

// the inter-arm checks of one chunk K (checks 64K .. 64K + kChecks - 1); no environment checks
template <int K>
struct PairInterR : PairRakeR {
    static constexpr int kFirst = K * panda_pair_chunk;
    static constexpr int kChecks = (panda_pair_n_checks - kFirst) < panda_pair_chunk ? (panda_pair_n_checks - kFirst)
                                                                                      : panda_pair_chunk;
    static constexpr int kWavesPerEU = VGPU_PAIR_INTER_BOUND_WAVES;
    static constexpr int kBoundWaves8 = (K == 0 && VGPU_PAIR_BOTH) ? VGPU_PAIR_BOTH8_WAVES : VGPU_PAIR_INTER_BOUND8_WAVES;
    static constexpr int kExtBoundWaves = 2;  // point-cloud bound kernels (vgpu_staged.hh BoundWavesE)
    static constexpr int kChildWavesPerEU = VGPU_PAIR_INTER_WAVES;
    using Mask = uint64_t;
    static constexpr Mask kEnvChecks = 0u;
    // chunk 0's bound stage also computes chunk 1's masks (vgpu_staged.hh BothChunks; VGPU_PAIR_BOTH=0: one
    // bound kernel per chunk, for A/B runs)
    static constexpr bool kBothChunks = K == 0 && VGPU_PAIR_BOTH;
    template <class Grp>
    __device__ static __forceinline__ Mask bound_both(const float* v, const Bases& b, Mask& m1)
    {
        return panda_pair_bound_both<Grp>(PAIR_Q(v), b.x, b.y, b.z, b.x2, b.y2, b.z2, m1);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ Mask bound(const float* v, const EnvView&, const Bases& b)
    {
        if constexpr (K == 0)
            return panda_pair_bound_mask_0<Grp>(PAIR_Q(v), b.x, b.y, b.z, b.x2, b.y2, b.z2);
        else
            return panda_pair_bound_mask_1<Grp>(PAIR_Q(v), b.x, b.y, b.z, b.x2, b.y2, b.z2);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool children(int c, const float* v, const EnvView&, const Bases& b)
    {
        return panda_pair_children<Grp>(kFirst + c, PAIR_Q(v), b.x, b.y, b.z, b.x2, b.y2, b.z2);
    }
};
static_assert(panda_pair_n_checks <= 2 * panda_pair_chunk, "two inter-arm chunks");

}  // namespace vgpu

// one pass per object file (the Makefile compiles this TU once per VGPU_PAIR_PASS = 0..3, in parallel)
#ifndef VGPU_PAIR_PASS
#error "compile with -DVGPU_PAIR_PASS=<0..3>"
#endif
#if VGPU_PAIR_PASS == 0
VGPU_STAGED_EXPORTS(vgpu::PairArmR<0>, pair_a)

namespace vgpu {
// validate head -> tail back-step counts of the 14-dof rake
__global__ __launch_bounds__(kStagedBlock) void pair_tail_counts_kernel(const float* __restrict__ starts,
                                                                        const float* __restrict__ goals,
                                                                        size_t n_edges, const uint8_t* __restrict__ ok,
                                                                        int32_t* __restrict__ n_blocks,
                                                                        uint32_t* __restrict__ cnt)
{
    const size_t e = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    if (e >= n_edges) return;
    const RakeD<kPairDimS> rk = rake_setup_d<kPairDimS, kPairResS>(starts + kPairDimS * e, goals + kPairDimS * e);
    if (n_blocks) n_blocks[e] = rk.n;
    cnt[e] = ((!ok || ok[e]) && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
}

}  // namespace vgpu

extern "C" hipError_t vgpu_launch_pair_tail_counts(const float* starts, const float* goals, size_t n_edges,
                                                   const uint8_t* ok, int32_t* n_blocks, uint32_t* cnt, hipStream_t st)
{
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess || n_edges == 0) return err;
    const unsigned grid = (unsigned)((n_edges + vgpu::kStagedBlock - 1) / vgpu::kStagedBlock);
    hipLaunchKernelGGL(vgpu::pair_tail_counts_kernel, dim3(grid), dim3(vgpu::kStagedBlock), 0, st, starts, goals,
                       n_edges, ok, n_blocks, cnt);
    return hipGetLastError();
}
#elif VGPU_PAIR_PASS == 1
VGPU_STAGED_EXPORTS(vgpu::PairArmR<1>, pair_b)
#elif VGPU_PAIR_PASS == 2
VGPU_STAGED_EXPORTS(vgpu::PairInterR<0>, pair_i0)
#else
VGPU_STAGED_EXPORTS(vgpu::PairInterR<1>, pair_i1)
#endif
