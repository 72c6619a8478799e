// vgpu_staged.hh -- staged evaluation of a robot's generated collision hierarchy, generic over
// the robot (Panda: 32 checks, 7 dof; Fetch: 63 checks, 8 dof).
//
// The monolithic kernels run FK and the hierarchical checks (e.g. panda/fk.hh:1335-6276) in one
// divergent pass: a wave executes a check's children whenever ANY of its groups' bounding tests
// fires, so on the bench workloads only 17 % (fkcc) / 37 % (validate head) of the Panda VALU lanes
// were active.  Here the same hierarchy runs in uniform stages:
//
//   bound     one group per rake block (G lanes): FK + all bounding tests, no children, no
//             early exit; writes a check mask (bit c = check c's bounding test fired for the
//             group) and counts the fired (group, check) pairs per check;
//   queue     scatters each fired (group, check) into check c's segment of an item list;
//             segments are padded to whole waves, so every wave holds ONE check;
//   children  one wave per 64/G items of one check: recomputes the frames that check needs and
//             tests its children; a firing child clears the group's result.  A leaf check (a
//             single-sphere link tested directly, fetch/fk.hh torso_lift_link_collision_2) has
//             no children: its bounding hit is the collision.
//
// Result: valid <=> no check has both its bounding test and one of its children firing -- the
// reference's early-exit loop is an OR over checks, so the evaluation order is free.  Groups are
// described by a Source: configurations (fkcc, G = 1), Halton samples (G = 1), first rake blocks
// of edges (validate head, G = 8), or (edge, back-step) items (validate tail, G = 8).
//
// A robot R provides: D (dof), kChecks, Mask (uint32_t / uint64_t), kEnvChecks (mask of the
// environment checks), sample(k, v), head(s, g, lane, v) and tail(s, g, lane, k, v) (the rake
// blocks), bound<Grp, EXT>(v, env, bases) -> Mask and children<Grp, EXT>(c, v, env, bases).
// VGPU_STAGED_EXPORTS(R, name) emits the extern "C" launchers vgpu_<name>_staged_*.
#pragma once

#include <type_traits>

#include "vgpu_device.hh"

namespace vgpu {

constexpr int kStagedBlock = 256;

// The device-side segment layout of one round of a staged pass (written by plan_kernel after the
// round's count + scan): each check's item segment [start, end) (wave-aligned; items [fill, end)
// are padding), laid out class-major so each children class covers one contiguous range [lo, hi).
// The host reads only the FIRST round's per-check counts back (one sync per pass): they bound
// every later round's counts, which sizes every children grid without another read-back.
constexpr int kPlanMaxChecks = 64;
constexpr int kPlanMaxClasses = 4;
struct StagedPlan {
    uint32_t start[kPlanMaxChecks], end[kPlanMaxChecks], fill[kPlanMaxChecks];
    uint32_t lo[kPlanMaxClasses], hi[kPlanMaxClasses];
    uint32_t total;
    uint32_t n_groups;  // groups of the pass (debug bounds checks)
};

// Children register classes.  A children kernel's VGPR budget is the maximum over the checks it can
// run, so one kernel over every check spills for all of them (Panda: 105 VGPRs for check 21 against
// a 72-VGPR budget at 7 waves/EU, 224 B/lane of scratch).  A robot may split its checks into
// classes (R::kClasses, R::kClassOf[c], R::kClassWaves[k]): one children kernel per class, each
// with its own occupancy.  Without them every check is class 0 at R::kChildWavesPerEU.
template <class R, class = void>
struct ChildClasses {
    static constexpr int n = 1;
    __host__ __device__ static constexpr int of(int) { return 0; }
    __host__ __device__ static constexpr int waves(int) { return R::kChildWavesPerEU; }
};
template <class R>
struct ChildClasses<R, std::void_t<decltype(R::kClassOf)>> {
    static_assert(R::kClasses <= kPlanMaxClasses, "too many children classes");
    static constexpr int n = R::kClasses;
    __host__ __device__ static constexpr int of(int c) { return R::kClassOf[c]; }
    __host__ __device__ static constexpr int waves(int k) { return R::kClassWaves[k]; }
};

// R::kExtClassOf / kExtClasses (optional): the class table of the point-cloud (EXT) instantiations -- their
// environment children run the CAPT queries, not near sets, so a robot may keep fewer classes there (the Panda's
// near-set class 3 is folded back into class 0 with a point cloud).  The host asks for the table of the pass's
// environment (vgpu_<name>_staged_class(c, ext)); plan and children kernels take it from their EXT parameter.
template <class R, bool EXT, class = void>
struct ChildClassesE : ChildClasses<R> {
};
template <class R>
struct ChildClassesE<R, true, std::void_t<decltype(R::kExtClassOf)>> {
    static_assert(R::kExtClasses <= kPlanMaxClasses, "too many children classes");
    static constexpr int n = R::kExtClasses;
    __host__ __device__ static constexpr int of(int c) { return R::kExtClassOf[c]; }
    __host__ __device__ static constexpr int waves(int k) { return R::kClassWaves[k]; }
};

// waves/EU of a children kernel: with a point cloud (EXT) at most VGPU_EXT_CHILD_WAVES -- the deferred
// queries' queue bookkeeping adds live registers: at 7 waves (72 VGPRs) the Panda / pair-arm class-0 kernels
// spilled 16-23 VGPRs (48-72 B scratch per lane); at 5 (96) none do (tests/test_kernel_resources.py).  A/B on
// MI355X, CAPT 2^20 configurations: 0.510 -> 0.518 ms kernel time (profiles/r05e_capt_ab.log)
#ifndef VGPU_EXT_CHILD_WAVES
#define VGPU_EXT_CHILD_WAVES 5
#endif
// (a robot may set its own point-cloud caps per class: R::kExtClassWaves[K])
template <class R, class = void>
struct ExtClassWaves {
    __host__ __device__ static constexpr int of(int) { return VGPU_EXT_CHILD_WAVES; }
};
template <class R>
struct ExtClassWaves<R, std::void_t<decltype(R::kExtClassWaves)>> {
    __host__ __device__ static constexpr int of(int k) { return R::kExtClassWaves[k]; }
};
template <class R, int K, bool EXT>
struct ChildWaves {
    static constexpr int w = ChildClassesE<R, EXT>::waves(K);
    static constexpr int cap = ExtClassWaves<R>::of(K);
    static constexpr int v = (EXT && w > cap) ? cap : w;
};

// Source kinds a robot's staged exports instantiate (bit k = kind k of StagedHost::with_source): all
// by default; a robot may restrict them with R::kSourceKinds (the composite has no sampler and no
// full-mask mode), which also cuts its compile time
template <class R, class = void>
struct SourceKinds {
    static constexpr unsigned v = 0x1Fu;
};
template <class R>
struct SourceKinds<R, std::void_t<decltype(R::kSourceKinds)>> {
    static constexpr unsigned v = R::kSourceKinds;
};

// ---- group sources ----------------------------------------------------------------------------
template <class R>
struct SrcConfigsT {  // fkcc: one configuration per group
    static constexpr int G = 1;
    static constexpr bool kInit = true;
    const float* q;
    __device__ __forceinline__ void load(uint32_t g, int, float v[R::D]) const
    {
        const float* p = q + R::D * (size_t)g;
#pragma unroll
        for (int j = 0; j < R::D; ++j) v[j] = p[j];
    }
    __device__ __forceinline__ uint32_t out(uint32_t g) const { return g; }
};

template <class R>
struct SrcSamplesT {  // Halton draw first + g, scaled
    static constexpr int G = 1;
    static constexpr bool kInit = true;
    uint64_t first;
    float* q_out;       // bound stage: copy of the sample (optional)
    const float* q_in;  // children stage: the bound stage's copy (else the draw is recomputed)
    __device__ __forceinline__ void load(uint32_t g, int, float v[R::D]) const
    {
        if (q_in) {
            const float* p = q_in + R::D * (size_t)g;
#pragma unroll
            for (int j = 0; j < R::D; ++j) v[j] = p[j];
        } else {
            R::sample(first + g, v);
        }
    }
    __device__ __forceinline__ uint32_t out(uint32_t g) const { return g; }
};

template <class R>
struct SrcHeadT {  // validate head: block 0 of edge g
    static constexpr int G = 8;
    static constexpr bool kInit = true;
    const float* starts;
    const float* goals;
    __device__ __forceinline__ void load(uint32_t g, int lane, float v[R::D]) const
    {
        R::head(starts + R::D * (size_t)g, goals + R::D * (size_t)g, lane, v);
    }
    __device__ __forceinline__ uint32_t out(uint32_t g) const { return g; }
};

// validate head over a compacted list: group g = block 0 of edge list[g], g < *n_live (the edges the lead pass
// left valid, ascending -- vgpu_launch_compact).  The bound stage's grid covers every edge (the live count is
// only on the device when it launches); groups past *n_live store an empty mask and leave.
template <class R>
struct SrcHeadListT {
    static constexpr int G = 8;
    static constexpr bool kInit = true;
    const float* starts;
    const float* goals;
    const uint32_t* list;
    const uint32_t* n_live;
    __device__ __forceinline__ bool live(uint32_t g) const { return g < *n_live; }
    __device__ __forceinline__ void load(uint32_t g, int lane, float v[R::D]) const
    {
        const uint32_t e = list[g];
        R::head(starts + R::D * (size_t)e, goals + R::D * (size_t)e, lane, v);
    }
    __device__ __forceinline__ uint32_t out(uint32_t g) const { return list[g]; }
};

// R::kHeadList (optional): the robot's validate heads may run over the lead pass's compacted list
template <class R, class = void>
struct HeadList {
    static constexpr bool v = false;
};
template <class R>
struct HeadList<R, std::void_t<decltype(R::kHeadList)>> {
    static constexpr bool v = R::kHeadList;
};

// groups a source leaves out (the compacted head list's tail past its device-side count)
template <class Src, class = void>
struct SrcLive {
    __device__ static __forceinline__ bool of(const Src&, uint32_t) { return true; }
};
template <class Src>
struct SrcLive<Src, std::void_t<decltype(&Src::live)>> {
    __device__ static __forceinline__ bool of(const Src& s, uint32_t g) { return s.live(g); }
};

template <class R>
struct SrcTailT {  // validate tail: item g = (edge, back-step k), result into the edge's flag
    static constexpr int G = 8;
    static constexpr bool kInit = false;  // the edge flag is shared by its items
    const float* starts;
    const float* goals;
    const uint32_t* item_edge;
    const uint32_t* off;
    __device__ __forceinline__ void load(uint32_t g, int lane, float v[R::D]) const
    {
        const uint32_t e = item_edge[g];
        const int k = (int)(g - off[e]) + 1;
        R::tail(starts + R::D * (size_t)e, goals + R::D * (size_t)e, lane, k, v);
    }
    __device__ __forceinline__ uint32_t out(uint32_t g) const { return item_edge[g]; }
};

template <class R>
struct SrcTailMaskT {  // full-mask mode: item g = (edge, back-step k), result into its own block slot
    static constexpr int G = 8;
    static constexpr bool kInit = true;  // every block gets its own flag
    const float* starts;
    const float* goals;
    const uint32_t* item_edge;
    const uint32_t* off;
    __device__ __forceinline__ void load(uint32_t g, int lane, float v[R::D]) const
    {
        const uint32_t e = item_edge[g];
        const int k = (int)(g - off[e]) + 1;
        R::tail(starts + R::D * (size_t)e, goals + R::D * (size_t)e, lane, k, v);
    }
    // block k of edge e sits at off[e] + e + k (edges laid out block 0 .. n_e - 1 in edge order)
    __device__ __forceinline__ uint32_t out(uint32_t g) const { return g + item_edge[g] + 1u; }
};

template <int G>
struct GrpOf;
template <>
struct GrpOf<1> {
    using T = Grp1;
};
template <>
struct GrpOf<8> {
    using T = Grp8;
};

// the group type of a staged kernel: with a point cloud (EXT), undecided CAPT queries are deferred
// (vgpu_device.hh capt_defer_*) -- in bound kernels under each check's bit (the generated calls pass
// it), in children kernels under kChildTag
template <int G, bool EXT, int TAG>
using StagedGrp = std::conditional_t<EXT, Deferred<typename GrpOf<G>::T, TAG>, typename GrpOf<G>::T>;

// OR of a 64-bit per-lane mask over the lane's group
template <class Grp>
__device__ __forceinline__ uint64_t group_or64(uint64_t v)
{
    return ((uint64_t)Grp::or_bits((uint32_t)(v >> 32)) << 32) | (uint64_t)Grp::or_bits((uint32_t)v);
}

template <class M>
__device__ __forceinline__ int mask_ctz(M a)
{
    if constexpr (sizeof(M) == 8) return __builtin_ctzll(a);
    else return __builtin_ctz(a);
}

template <class M>
__device__ __forceinline__ M wave_or(M m)
{
    if constexpr (sizeof(M) == 8) {
        uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
        for (int off = 32; off >= 1; off >>= 1) {
            lo |= __shfl_xor(lo, off);
            hi |= __shfl_xor(hi, off);
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        hi = __builtin_amdgcn_readfirstlane(hi);
        return ((M)hi << 32) | lo;
    } else {
        for (int off = 32; off >= 1; off >>= 1) m |= __shfl_xor(m, off);
        return __builtin_amdgcn_readfirstlane(m);
    }
}

// per-(check, block) counts of the set bits of m over the block, check-major:
// counts[c * gridDim.x + blockIdx.x]
template <class R>
__device__ __forceinline__ void block_counts(typename R::Mask m, uint32_t* __restrict__ counts)
{
    using M = typename R::Mask;
    __shared__ uint32_t cnt[R::kChecks];
    for (int i = threadIdx.x; i < R::kChecks; i += kStagedBlock) cnt[i] = 0u;
    __syncthreads();
    const M any = wave_or(m);
    for (M a = any; a; a &= a - 1) {
        const int c = mask_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        if (__lane_id() == 0) atomicAdd(&cnt[c], (uint32_t)__builtin_popcountll(b));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < R::kChecks; i += kStagedBlock) counts[(size_t)i * gridDim.x + blockIdx.x] = cnt[i];
}

// waves/EU of a bound kernel: R::kWavesPerEU, or R::kBoundWaves8 for the 8-lane rake sources (validate head
// and tail) when the robot sets it -- their rake loaders and group reductions add live registers, which
// at the sampler's occupancy spilled hundreds of bytes per lane (Fetch, the composite's inter-arm passes:
// r04 PMC, GB of scratch writes per call)
template <class R, class Src, class = void>
struct BoundWaves {
    static constexpr int v = R::kWavesPerEU;
};
template <class R, class Src>
struct BoundWaves<R, Src, std::void_t<decltype(R::kBoundWaves8)>> {
    static constexpr int v = Src::G > 1 ? R::kBoundWaves8 : R::kWavesPerEU;
};
// with a point cloud (EXT) at most R::kExtBoundWaves (optional): the deferred-query bookkeeping adds live
// registers to the bound kernels too (Fetch 8-lane: 24 VGPRs spilled at 128, the composite's inter-arm
// chunks 6-12 at 96-168)
template <class R, class = void>
struct ExtBoundCap {
    static constexpr int v = 8;
};
template <class R>
struct ExtBoundCap<R, std::void_t<decltype(R::kExtBoundWaves)>> {
    static constexpr int v = R::kExtBoundWaves;
};
template <class R, class Src, bool EXT>
struct BoundWavesE {
    static constexpr int b = BoundWaves<R, Src>::v;
    static constexpr int v = (EXT && ExtBoundCap<R>::v < b) ? ExtBoundCap<R>::v : b;
};

// source kinds, numbered (the MidBound selection and the VGPU_HITSTATS counters)
template <class Src> struct SrcKindOf;
template <class R> struct SrcKindOf<SrcConfigsT<R>> { static constexpr int v = 0; };
template <class R> struct SrcKindOf<SrcSamplesT<R>> { static constexpr int v = 1; };
template <class R> struct SrcKindOf<SrcHeadT<R>> { static constexpr int v = 2; };
template <class R> struct SrcKindOf<SrcHeadListT<R>> { static constexpr int v = 2; };
template <class R> struct SrcKindOf<SrcTailT<R>> { static constexpr int v = 3; };
template <class R> struct SrcKindOf<SrcTailMaskT<R>> { static constexpr int v = 4; };

// R::kMidKinds (optional, default none): bit k set = sources of kind k evaluate the bound stage with the
// model's mid-sphere tests, R::bound<Grp, EXT, true> (tools/gen_kernels.py MIDS).  They cut the children
// queued where bounding hits rarely confirm (a validate tail's back-steps) and cost time where they do.
template <class R, class = void>
struct MidKinds {
    static constexpr uint32_t v = 0u;
};
template <class R>
struct MidKinds<R, std::void_t<decltype(R::kMidKinds)>> {
    static constexpr uint32_t v = R::kMidKinds;
};
template <class R, class Src>
inline constexpr bool kMidBound = ((MidKinds<R>::v >> SrcKindOf<Src>::v) & 1u) != 0u;

// R::kBothChunks (optional): the bound stage of this pass also computes the NEXT chained pass's masks (the
// composite's two inter-arm chunks from one FK of both arms, R::bound_both) and stores them after its own,
// mask[n_groups + g]; the host then skips the next pass's bound kernel and hands it that half
template <class R, class = void>
struct BothChunks {
    static constexpr bool v = false;
};
template <class R>
struct BothChunks<R, std::void_t<decltype(R::kBothChunks)>> {
    static constexpr bool v = R::kBothChunks;
};

// ---- stage 1: bounding masks ---------------------------------------------------------------
template <class R, class Src, bool EXT>
__global__ __launch_bounds__(kStagedBlock, (BoundWavesE<R, Src, EXT>::v)) void bound_kernel(Src src, uint32_t n_groups, EnvView env,
                                                                             Bases bs, int chain,
                                                                             typename R::Mask* __restrict__ mask,
                                                                             uint8_t* __restrict__ valid)
{
    using Grp = StagedGrp<Src::G, EXT, -1>;
    if constexpr (EXT) {
        capt_stage_lds(env);  // the split tree's top levels into LDS (before any return)
        capt_defer_init();
    }
    const size_t tid = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const int lane = (int)(tid % Src::G);
    if (g >= n_groups) return;  // group-uniform
    // a chained pass (a later pass over the same groups, e.g. the composite's arm B after arm A): a
    // group already invalid is done -- its mask stays 0 -- and the flag is not re-initialised
    if (!SrcLive<Src>::of(src, g) || (chain && !valid[src.out(g)])) {
        if (lane == 0) {
            mask[g] = 0;
            if constexpr (BothChunks<R>::v) mask[n_groups + g] = 0;
        }
        return;
    }
    float v[R::D];
    src.load(g, lane, v);
    if constexpr (std::is_same<Src, SrcSamplesT<R>>::value) {
        if (src.q_out) {
#pragma unroll
            for (int j = 0; j < R::D; ++j) src.q_out[R::D * (size_t)g + j] = v[j];
        }
    }
    typename R::Mask m;
    [[maybe_unused]] typename R::Mask m1 = 0;
    if constexpr (BothChunks<R>::v) m = R::template bound_both<Grp>(v, bs, m1);
    else if constexpr (kMidBound<R, Src>) m = R::template bound<Grp, EXT, true>(v, env, bs);
    else m = R::template bound<Grp, EXT>(v, env, bs);
    if constexpr (EXT) m |= (typename R::Mask)group_or64<Grp>(capt_defer_finish(env.pc, env.base, env.pc_lds_levels));
    if (lane == 0) {
        mask[g] = m;
        if constexpr (BothChunks<R>::v) mask[n_groups + g] = m1;
        if constexpr (Src::kInit) {
            if (!chain) valid[src.out(g)] = 1;
        }
    }
}

// ---- lead pass (optional, R::kLeadCheck): one check, monolithic, before the bound stage ----------
// R::lead<Grp>(v, env, bases) evaluates check kLeadCheck alone -- bounding test, then its children when
// the group's bounding test fires -- and is true when the group passes it.  The pass initialises the
// flags; the bound stage then runs chained (a group the lead check invalidated skips it) and the
// rounds leave the lead check out.  Primitive environments only (no point clouds or heightfields).
template <class R, class = void>
struct LeadCheck {
    static constexpr int v = -1;
};
template <class R>
struct LeadCheck<R, std::void_t<decltype(R::kLeadCheck)>> {
    static constexpr int v = R::kLeadCheck;
};

// waves/EU of the lead kernel: R::kLeadWaves, else the bound stage's
template <class R, class Src, class = void>
struct LeadWaves {
    static constexpr int v = BoundWaves<R, Src>::v;
};
template <class R, class Src>
struct LeadWaves<R, Src, std::void_t<decltype(R::kLeadWaves)>> {
    static constexpr int v = R::kLeadWaves;
};

template <class R, class Src>
__global__ __launch_bounds__(kStagedBlock, (LeadWaves<R, Src>::v)) void lead_kernel(Src src, uint32_t n_groups,
                                                                                EnvView env, Bases bs,
                                                                                uint8_t* __restrict__ valid)
{
    using Grp = typename GrpOf<Src::G>::T;
    const size_t tid = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const int lane = (int)(tid % Src::G);
    if (g >= n_groups) return;  // group-uniform
    float v[R::D];
    src.load(g, lane, v);
    const bool ok = R::template lead<Grp>(v, env, bs);
    if (lane == 0) valid[src.out(g)] = ok ? 1 : 0;
}

// ---- rounds: the fired (group, check) pairs of a set of checks, for groups still valid ----------
// Checks run in rounds (e.g. the environment checks, then the self checks): a group invalidated by
// an earlier round contributes no work to later ones, which recovers the reference's early exit.
// count and queue run one thread per GROUP (not per lane: they only read the group's mask and
// flag), kStagedBlock groups per block; per-(check, block) counts are stored check-major,
// counts[c * blocks + block], for one flat exclusive scan.
template <class R, class Src>
__device__ __forceinline__ typename R::Mask round_bits(const Src& src, const typename R::Mask* __restrict__ mask,
                                                       uint32_t n_groups, typename R::Mask set,
                                                       const uint8_t* __restrict__ valid, uint32_t g)
{
    if (g >= n_groups) return 0u;
    const typename R::Mask m = mask[g] & set;
    return (m && valid[src.out(g)]) ? m : (typename R::Mask)0u;
}

template <class R, class Src>
__global__ __launch_bounds__(kStagedBlock) void count_kernel(Src src, const typename R::Mask* __restrict__ mask,
                                                             uint32_t n_groups, typename R::Mask set,
                                                             const uint8_t* __restrict__ valid,
                                                             uint32_t* __restrict__ counts)
{
    const uint32_t g = blockIdx.x * kStagedBlock + threadIdx.x;
    block_counts<R>(round_bits<R>(src, mask, n_groups, set, valid, g), counts);
}

// After a round's count + scan: fired[c] = offs[(c+1)*nb] - offs[c*nb]; the round's segments,
// class-major.  One lane per check computes its fired count, lane 0 lays them out.
template <class R, bool EXT>
__global__ __launch_bounds__(64) void plan_kernel(const uint32_t* __restrict__ offs, uint32_t nb, uint32_t W,
                                                  uint64_t set, uint32_t n_groups, StagedPlan* __restrict__ plan)
{
    using CC = ChildClassesE<R, EXT>;
    __shared__ uint32_t fired[R::kChecks];
    for (int k = threadIdx.x; k < R::kChecks; k += 64)
        fired[k] = offs[(size_t)(k + 1) * nb] - offs[(size_t)k * nb];
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint32_t total = 0;
    for (int cls = 0; cls < CC::n; ++cls) {
        plan->lo[cls] = total;
        for (int k = 0; k < R::kChecks; ++k) {
            if (CC::of(k) != cls) continue;
            const bool on = (set >> k) & 1u;
            plan->start[k] = total;
            plan->fill[k] = total + (on ? fired[k] : 0u);
            if (on) total += (fired[k] + W - 1) / W * W;
            plan->end[k] = total;
        }
        plan->hi[cls] = total;
    }
    plan->total = total;
    plan->n_groups = n_groups;
}

// Position of group g in check c's segment:
//   start[c] + (offs[c*nb + block] - offs[c*nb]) + rank of g among the block's groups with bit c
// -- ascending group order within each segment, no atomics.
template <class R, class Src>
__global__ __launch_bounds__(kStagedBlock) void queue_kernel(Src src, const typename R::Mask* __restrict__ mask,
                                                             uint32_t n_groups, typename R::Mask set,
                                                             const StagedPlan* __restrict__ plan,
                                                             const uint8_t* __restrict__ valid,
                                                             const uint32_t* __restrict__ offs,
                                                             uint32_t* __restrict__ items, const void* dbg)
{
    using M = typename R::Mask;
    const uint32_t g = blockIdx.x * kStagedBlock + threadIdx.x;
    const M m = round_bits<R>(src, mask, n_groups, set, valid, g);
    const int w = threadIdx.x >> 6;
    constexpr int kW = kStagedBlock / 64;
    __shared__ uint32_t wcnt[kW][R::kChecks];
    __shared__ uint32_t cbase[R::kChecks];
    const size_t nb = gridDim.x;
    for (int i = threadIdx.x; i < kW * R::kChecks; i += kStagedBlock) (&wcnt[0][0])[i] = 0u;
    // the block's first slot in every check's segment: all loads issued at once, not one per set bit
    for (int c = threadIdx.x; c < R::kChecks; c += kStagedBlock)
        cbase[c] = plan->start[c] + (offs[(size_t)c * nb + blockIdx.x] - offs[(size_t)c * nb]);
    __syncthreads();
    const M any = wave_or(m);
    for (M a = any; a; a &= a - 1) {
        const int c = mask_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        if (__lane_id() == 0) wcnt[w][c] = (uint32_t)__builtin_popcountll(b);
    }
    __syncthreads();
    const uint64_t below = (__lane_id() == 0) ? 0ull : (~0ull >> (64 - __lane_id()));
    for (M a = any; a; a &= a - 1) {
        const int c = mask_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        uint32_t base = cbase[c];
        for (int i = 0; i < w; ++i) base += wcnt[i][c];
        if ((m >> c) & 1u) {
            const uint32_t slot = base + (uint32_t)__builtin_popcountll(b & below);
            VGPU_DCHECK(dbg, slot >= plan->start[c] && slot < plan->fill[c], DBG_QUEUE_SLOT);
            if (slot < plan->total) items[slot] = g;
        }
    }
}

// ---- stage 2: children, one check per wave ------------------------------------------------------
#ifdef VGPU_HITSTATS
__device__ unsigned int vgpu_hitstats[5][64][2];
#endif
// A class's kernel covers the class's item range [lo, hi) of the plan; its grid is sized by the
// host from an upper bound (the first round's counts), so waves past hi exit at once.  The check of
// a wave is found by scanning the class's checks (compile-time list, scalar compares against the
// plan); the generated switch folds to that one case, so the kernel's registers cover only its class.
template <class R, int K, class Grp, bool EXT, int C = 0>
__device__ __forceinline__ int children_of_class(uint32_t item0, const StagedPlan* __restrict__ plan, const float* v,
                                                 const EnvView& env, const Bases& bs)
{
    if constexpr (C == R::kChecks) {
        return -1;
    } else {
        if constexpr (ChildClassesE<R, EXT>::of(C) == K) {
            if (item0 >= plan->start[C] && item0 < plan->end[C])
                return R::template children<Grp, EXT>(C, v, env, bs) ? 1 : 0;
        }
        return children_of_class<R, K, Grp, EXT, C + 1>(item0, plan, v, env, bs);
    }
}

template <class R, class Src, bool EXT, int K>
__global__ __launch_bounds__(kStagedBlock, (ChildWaves<R, K, EXT>::v)) void children_kernel(
    Src src, const StagedPlan* __restrict__ plan, const uint32_t* __restrict__ items, EnvView env, Bases bs,
    uint8_t* __restrict__ valid)
{
    using Grp = StagedGrp<Src::G, EXT, kChildTag>;
    if constexpr (EXT) {
        capt_stage_lds(env);  // the split tree's top levels into LDS (before any return)
        capt_defer_init();
    }
    const size_t tid = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    const uint32_t item = plan->lo[K] + (uint32_t)(tid / Src::G);
    const int lane = (int)(tid % Src::G);
    if (item >= plan->hi[K]) return;  // wave-uniform (segments are wave-aligned)
    const uint32_t item0 = __builtin_amdgcn_readfirstlane(item);
    // the owning check's fill (unrolled scalar compares against the plan, constant offsets: the
    // loads batch; a data-dependent scan over checks would chain one memory latency per check)
    uint32_t fill = 0;
#pragma unroll
    for (int k = 0; k < R::kChecks; ++k)
        if (ChildClassesE<R, EXT>::of(k) == K && item0 >= plan->start[k] && item0 < plan->end[k]) fill = plan->fill[k];
    if (item >= fill) return;  // segment padding (group-uniform)
    const uint32_t g = VGPU_DCLAMP(env.base, items[item], plan->n_groups, DBG_CHILD_GROUP);
    float v[R::D];
    src.load(g, lane, v);
    bool hit = children_of_class<R, K, Grp, EXT>(item0, plan, v, env, bs) > 0;
    if constexpr (EXT) hit = Grp::any(capt_defer_finish(env.pc, env.base, env.pc_lds_levels) != 0ull) || hit;
    if (hit && lane == 0) valid[src.out(g)] = 0;  // every writer stores 0: the race is benign
#ifdef VGPU_HITSTATS
    // development statistics (variant builds only): items run and items whose children hit, per
    // (source kind, check) -- how much of the children work verifies a bounding hit that is no collision
    if (lane == 0) {
        int chk = 0;
#pragma unroll
        for (int k = 0; k < R::kChecks; ++k)
            if (item0 >= plan->start[k] && item0 < plan->end[k]) chk = k;
        atomicAdd(&vgpu_hitstats[SrcKindOf<Src>::v][chk][0], 1u);
        if (hit) atomicAdd(&vgpu_hitstats[SrcKindOf<Src>::v][chk][1], 1u);
    }
#endif
}

// ---- host-side launch helpers ------------------------------------------------------------------
template <class R>
struct StagedHost {
    using M = typename R::Mask;

    template <class Src>
    static unsigned grid_of(uint32_t n_groups)
    {
        return (unsigned)(((size_t)n_groups * Src::G + kStagedBlock - 1) / kStagedBlock);
    }

    static unsigned group_blocks(uint32_t n_groups) { return (n_groups + kStagedBlock - 1) / kStagedBlock; }

    template <class Src>
    static hipError_t bound(const Src& src, uint32_t n_groups, const EnvView* env, const Bases& bs, int chain,
                            M* mask, uint8_t* valid, hipStream_t st)
    {
        if (n_groups == 0) return hipSuccess;
        const unsigned grid = grid_of<Src>(n_groups);
        if (env->n_hf > 0 || env->n_pc > 0)
            hipLaunchKernelGGL((bound_kernel<R, Src, true>), dim3(grid), dim3(kStagedBlock), 0, st, src, n_groups,
                               *env, bs, chain, mask, valid);
        else
            hipLaunchKernelGGL((bound_kernel<R, Src, false>), dim3(grid), dim3(kStagedBlock), 0, st, src, n_groups,
                               *env, bs, chain, mask, valid);
        return hipGetLastError();
    }

    template <class Src>
    static hipError_t lead(const Src& src, uint32_t n_groups, const EnvView* env, const Bases& bs, uint8_t* valid,
                           hipStream_t st)
    {
        if constexpr (LeadCheck<R>::v < 0 || !Src::kInit) {
            return hipErrorInvalidValue;
        } else {
            if (env->n_hf > 0 || env->n_pc > 0) return hipErrorInvalidValue;
            if (n_groups == 0) return hipSuccess;
            hipLaunchKernelGGL((lead_kernel<R, Src>), dim3(grid_of<Src>(n_groups)), dim3(kStagedBlock), 0, st, src,
                               n_groups, *env, bs, valid);
            return hipGetLastError();
        }
    }

    template <class Src>
    static hipError_t count(const Src& src, const M* mask, uint32_t n_groups, M set, const uint8_t* valid,
                            uint32_t* counts, hipStream_t st)
    {
        hipLaunchKernelGGL((count_kernel<R, Src>), dim3(group_blocks(n_groups)), dim3(kStagedBlock), 0, st, src, mask,
                           n_groups, set, valid, counts);
        return hipGetLastError();
    }

    template <class Src>
    static hipError_t queue(const Src& src, const M* mask, uint32_t n_groups, M set, const StagedPlan* plan,
                            const uint8_t* valid, const uint32_t* offs, uint32_t* items, const void* dbg,
                            hipStream_t st)
    {
        hipLaunchKernelGGL((queue_kernel<R, Src>), dim3(group_blocks(n_groups)), dim3(kStagedBlock), 0, st, src, mask,
                           n_groups, set, plan, valid, offs, items, dbg);
        return hipGetLastError();
    }

    // one launch per class with items; ub[k] = upper bound of class k's item count this round
    template <class Src, bool EXT, int K = 0>
    static hipError_t children_classes(const Src& src, const StagedPlan* plan, const uint32_t* ub,
                                       const uint32_t* items, const EnvView* env, const Bases& bs,
                                       uint8_t* valid, hipStream_t st)
    {
        if constexpr (K == ChildClassesE<R, EXT>::n) {
            return hipSuccess;
        } else {
            const size_t threads = (size_t)ub[K] * Src::G;
            if (threads > 0) {
                const unsigned grid = (unsigned)((threads + kStagedBlock - 1) / kStagedBlock);
                hipLaunchKernelGGL((children_kernel<R, Src, EXT, K>), dim3(grid), dim3(kStagedBlock), 0, st, src,
                                   plan, items, *env, bs, valid);
                const hipError_t err = hipGetLastError();
                if (err != hipSuccess) return err;
            }
            return children_classes<Src, EXT, K + 1>(src, plan, ub, items, env, bs, valid, st);
        }
    }

    template <class Src>
    static hipError_t children(const Src& src, const StagedPlan* plan, const uint32_t* ub, const uint32_t* items,
                               const EnvView* env, const Bases& bs, uint8_t* valid, hipStream_t st)
    {
        if (env->n_hf > 0 || env->n_pc > 0)
            return children_classes<Src, true>(src, plan, ub, items, env, bs, valid, st);
        return children_classes<Src, false>(src, plan, ub, items, env, bs, valid, st);
    }

    static hipError_t plan(const uint32_t* offs, uint32_t nb, uint32_t W, M set, uint32_t n_groups, StagedPlan* plan,
                           int ext, hipStream_t st)
    {
        if (ext)
            hipLaunchKernelGGL((plan_kernel<R, true>), dim3(1), dim3(64), 0, st, offs, nb, W, (uint64_t)set, n_groups, plan);
        else
            hipLaunchKernelGGL((plan_kernel<R, false>), dim3(1), dim3(64), 0, st, offs, nb, W, (uint64_t)set, n_groups, plan);
        return hipGetLastError();
    }

    // dispatch on the source kind: 0 configurations (s0 = q), 1 Halton samples (first, s0 = q_out
    // or NULL), 2 validate head (s0 = starts, s1 = goals), 3 validate tail (+ s2 = item_edge, s3 = off),
    // 4 full-mask tail (as 3, one result per block)
    template <class Fn>
    static hipError_t with_source(int kind, const void* s0, const void* s1, const void* s2, const void* s3,
                                  uint64_t first, Fn fn)
    {
        constexpr unsigned K = SourceKinds<R>::v;
        switch (kind) {
        case 0:
            if constexpr ((K & 1u) != 0) return fn(SrcConfigsT<R>{(const float*)s0});
            break;
        case 1:
            if constexpr ((K & 2u) != 0) return fn(SrcSamplesT<R>{first, (float*)s0, nullptr});
            break;
        case 2:  // s2, s3: the compacted list and its device-side count (HeadList robots), else NULL
            if constexpr ((K & 4u) != 0) {
                if constexpr (HeadList<R>::v) {
                    if (s2)
                        return fn(SrcHeadListT<R>{(const float*)s0, (const float*)s1, (const uint32_t*)s2,
                                                  (const uint32_t*)s3});
                }
                if (s2) break;
                return fn(SrcHeadT<R>{(const float*)s0, (const float*)s1});
            }
            break;
        case 3:
            if constexpr ((K & 8u) != 0)
                return fn(SrcTailT<R>{(const float*)s0, (const float*)s1, (const uint32_t*)s2, (const uint32_t*)s3});
            break;
        case 4:
            if constexpr ((K & 16u) != 0)
                return fn(SrcTailMaskT<R>{(const float*)s0, (const float*)s1, (const uint32_t*)s2,
                                          (const uint32_t*)s3});
            break;
        }
        return hipErrorInvalidValue;
    }
};

}  // namespace vgpu

// extern "C" launchers of one robot (masks cross the ABI as uint64_t)
#define VGPU_STAGED_EXPORTS(R, NAME)                                                                                 \
    extern "C" {                                                                                                     \
    int vgpu_##NAME##_staged_checks(void) { return R::kChecks; }                                                     \
    uint64_t vgpu_##NAME##_staged_env_checks(void) { return (uint64_t)R::kEnvChecks; }                             \
    int vgpu_##NAME##_staged_mask_bytes(void) { return (int)sizeof(typename R::Mask) * (vgpu::BothChunks<R>::v ? 2 : 1); } \
    int vgpu_##NAME##_staged_class(int c, int ext)                                                                   \
    {                                                                                                                \
        return ext ? vgpu::ChildClassesE<R, true>::of(c) : vgpu::ChildClassesE<R, false>::of(c);                    \
    }                                                                                                                \
    size_t vgpu_##NAME##_staged_plan_bytes(void) { return sizeof(vgpu::StagedPlan); }                               \
    uint32_t vgpu_##NAME##_staged_blocks(int, uint32_t n_groups)                                                     \
    {                                                                                                                \
        return vgpu::StagedHost<R>::group_blocks(n_groups); /* count / queue grid: one thread per group */          \
    }                                                                                                                \
    hipError_t vgpu_##NAME##_staged_bound(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          uint64_t first, uint32_t n_groups, const EnvView* env,                     \
                                          const float* bases, int chain, void* mask, uint8_t* valid, hipStream_t st) \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        const Bases bs{bases[0], bases[1], bases[2], bases[3], bases[4], bases[5]};                            \
        return H::with_source(kind, s0, s1, s2, s3, first, [&](auto src) {                                          \
            return H::bound(src, n_groups, env, bs, chain, (typename R::Mask*)mask, valid, st);                      \
        });                                                                                                          \
    }                                                                                                                \
    int vgpu_##NAME##_staged_lead_check(void) { return vgpu::LeadCheck<R>::v; }                                   \
    int vgpu_##NAME##_staged_head_list(void) { return vgpu::HeadList<R>::v ? 1 : 0; }                             \
    hipError_t vgpu_##NAME##_staged_lead(int kind, const void* s0, const void* s1, const void* s2, const void* s3,   \
                                         uint64_t first, uint32_t n_groups, const EnvView* env, const float* bases,  \
                                         uint8_t* valid, hipStream_t st)                                             \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        const Bases bs{bases[0], bases[1], bases[2], bases[3], bases[4], bases[5]};                            \
        return H::with_source(kind, s0, s1, s2, s3, first,                                                           \
                              [&](auto src) { return H::lead(src, n_groups, env, bs, valid, st); });                \
    }                                                                                                                \
    hipError_t vgpu_##NAME##_staged_count(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          const void* mask, uint32_t n_groups, uint64_t set, const uint8_t* valid,   \
                                          uint32_t* counts, hipStream_t st)                                          \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        if (n_groups == 0) return hipSuccess;                                                                        \
        return H::with_source(kind, s0, s1, s2, s3, 0, [&](auto src) {                                              \
            return H::count(src, (const typename R::Mask*)mask, n_groups, (typename R::Mask)set, valid, counts, st); \
        });                                                                                                          \
    }                                                                                                                \
    hipError_t vgpu_##NAME##_staged_plan(const uint32_t* offs, uint32_t nb, uint32_t W, uint64_t set,                \
                                         uint32_t n_groups, void* plan, int ext, hipStream_t st)                     \
    {                                                                                                                \
        return vgpu::StagedHost<R>::plan(offs, nb, W, (typename R::Mask)set, n_groups, (vgpu::StagedPlan*)plan, ext, \
                                         st);                                                                        \
    }                                                                                                                \
    hipError_t vgpu_##NAME##_staged_queue(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          const void* mask, uint32_t n_groups, uint64_t set, const void* plan,       \
                                          const uint8_t* valid, const uint32_t* offs, uint32_t* items,               \
                                          const void* dbg, hipStream_t st)                                           \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        if (n_groups == 0) return hipSuccess;                                                                        \
        return H::with_source(kind, s0, s1, s2, s3, 0, [&](auto src) {                                              \
            return H::queue(src, (const typename R::Mask*)mask, n_groups, (typename R::Mask)set,                     \
                            (const vgpu::StagedPlan*)plan, valid, offs, items, dbg, st);                             \
        });                                                                                                          \
    }                                                                                                                \
    hipError_t vgpu_##NAME##_staged_children(int kind, const void* s0, const void* s1, const void* s2,               \
                                             const void* s3, uint64_t first, const void* plan, const uint32_t* ub,   \
                                             const uint32_t* items, const EnvView* env, const float* bases,          \
                                             uint8_t* valid, hipStream_t st)                                         \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        const Bases bs{bases[0], bases[1], bases[2], bases[3], bases[4], bases[5]};                            \
        return H::with_source(kind, s0, s1, s2, s3, first, [&](auto src) {                                          \
            if constexpr (std::is_same<decltype(src), vgpu::SrcSamplesT<R>>::value) {                                \
                src.q_in = src.q_out; /* the samples the bound stage wrote */                                         \
                src.q_out = nullptr;                                                                                 \
            }                                                                                                        \
            return H::children(src, (const vgpu::StagedPlan*)plan, ub, items, env, bs, valid, st);                   \
        });                                                                                                          \
    }                                                                                                                \
    }
