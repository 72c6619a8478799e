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
// blocks), bound<Grp, EXT>(v, env, bx, by, bz) -> Mask and children<Grp, EXT>(c, v, env, ...).
// VGPU_STAGED_EXPORTS(R, name) emits the extern "C" launchers vgpu_<name>_staged_*.
#pragma once

#include <type_traits>

#include "vgpu_device.hh"

namespace vgpu {

constexpr int kStagedBlock = 256;
constexpr uint32_t kNoItem = 0xFFFFFFFFu;

template <class R>
struct SegTableT {
    uint32_t start[R::kChecks + 1];  // check c owns items [start[c], start[c+1]), wave-aligned
};

// ---- group sources ----------------------------------------------------------------------------
template <class R>
struct SrcConfigsT {  // fkcc: one configuration per group
    static constexpr int G = 1;
    static constexpr bool kInit = true;
    const float* q;
    __device__ void load(uint32_t g, int, float v[R::D]) const
    {
        const float* p = q + R::D * (size_t)g;
#pragma unroll
        for (int j = 0; j < R::D; ++j) v[j] = p[j];
    }
    __device__ uint32_t out(uint32_t g) const { return g; }
};

template <class R>
struct SrcSamplesT {  // Halton draw first + g, scaled
    static constexpr int G = 1;
    static constexpr bool kInit = true;
    uint64_t first;
    float* q_out;       // bound stage: copy of the sample (optional)
    const float* q_in;  // children stage: the bound stage's copy (else the draw is recomputed)
    __device__ void load(uint32_t g, int, float v[R::D]) const
    {
        if (q_in) {
            const float* p = q_in + R::D * (size_t)g;
#pragma unroll
            for (int j = 0; j < R::D; ++j) v[j] = p[j];
        } else {
            R::sample(first + g, v);
        }
    }
    __device__ uint32_t out(uint32_t g) const { return g; }
};

template <class R>
struct SrcHeadT {  // validate head: block 0 of edge g
    static constexpr int G = 8;
    static constexpr bool kInit = true;
    const float* starts;
    const float* goals;
    __device__ void load(uint32_t g, int lane, float v[R::D]) const
    {
        R::head(starts + R::D * (size_t)g, goals + R::D * (size_t)g, lane, v);
    }
    __device__ uint32_t out(uint32_t g) const { return g; }
};

template <class R>
struct SrcTailT {  // validate tail: item g = (edge, back-step k), result into the edge's flag
    static constexpr int G = 8;
    static constexpr bool kInit = false;  // the edge flag is shared by its items
    const float* starts;
    const float* goals;
    const uint32_t* item_edge;
    const uint32_t* off;
    __device__ void load(uint32_t g, int lane, float v[R::D]) const
    {
        const uint32_t e = item_edge[g];
        const int k = (int)(g - off[e]) + 1;
        R::tail(starts + R::D * (size_t)e, goals + R::D * (size_t)e, lane, k, v);
    }
    __device__ uint32_t out(uint32_t g) const { return item_edge[g]; }
};

template <class R>
struct SrcTailMaskT {  // full-mask mode: item g = (edge, back-step k), result into its own block slot
    static constexpr int G = 8;
    static constexpr bool kInit = true;  // every block gets its own flag
    const float* starts;
    const float* goals;
    const uint32_t* item_edge;
    const uint32_t* off;
    __device__ void load(uint32_t g, int lane, float v[R::D]) const
    {
        const uint32_t e = item_edge[g];
        const int k = (int)(g - off[e]) + 1;
        R::tail(starts + R::D * (size_t)e, goals + R::D * (size_t)e, lane, k, v);
    }
    // block k of edge e sits at off[e] + e + k (edges laid out block 0 .. n_e - 1 in edge order)
    __device__ uint32_t out(uint32_t g) const { return g + item_edge[g] + 1u; }
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

// ---- stage 1: bounding masks ---------------------------------------------------------------
template <class R, class Src, bool EXT>
__global__ __launch_bounds__(kStagedBlock, R::kWavesPerEU) void bound_kernel(Src src, uint32_t n_groups, EnvView env,
                                                                             float bx, float by, float bz,
                                                                             typename R::Mask* __restrict__ mask,
                                                                             uint8_t* __restrict__ valid,
                                                                             uint32_t* __restrict__ counts)
{
    using Grp = typename GrpOf<Src::G>::T;
    using M = typename R::Mask;
    if constexpr (EXT) capt_stage_lds(env);  // the split tree's top levels into LDS (before any return)
    const size_t tid = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const int lane = (int)(tid % Src::G);
    M m = 0u;
    if (g < n_groups) {  // group-uniform
        float v[R::D];
        src.load(g, lane, v);
        if constexpr (std::is_same<Src, SrcSamplesT<R>>::value) {
            if (src.q_out) {
#pragma unroll
                for (int j = 0; j < R::D; ++j) src.q_out[R::D * (size_t)g + j] = v[j];
            }
        }
        m = R::template bound<Grp, EXT>(v, env, bx, by, bz);
        if (lane == 0) {
            mask[g] = m;
            if constexpr (Src::kInit) valid[src.out(g)] = 1;
        }
    }
    // the first round's per-(check, block) counts: every group is still valid here (tail items
    // exist only for edges that passed the head)
    if (lane != 0) m = 0u;
    block_counts<R>(m, counts);
}

// ---- rounds: the fired (group, check) pairs of a set of checks, for groups still valid ----------
// Checks run in rounds (e.g. the environment checks, then the self checks): a group invalidated by
// an earlier round contributes no work to later ones, which recovers the reference's early exit.
// Both kernels use the bound kernel's grid; per-(check, block) counts are stored check-major,
// counts[c * blocks + block], for one flat exclusive scan.
template <class R, class Src>
__device__ __forceinline__ typename R::Mask round_bits(const Src& src, const typename R::Mask* __restrict__ mask,
                                                       uint32_t n_groups, typename R::Mask set,
                                                       const uint8_t* __restrict__ valid, uint32_t g, bool lead)
{
    if (!lead || g >= n_groups) return 0u;
    const typename R::Mask m = mask[g] & set;
    return (m && valid[src.out(g)]) ? m : (typename R::Mask)0u;
}

template <class R, class Src>
__global__ __launch_bounds__(kStagedBlock) void count_kernel(Src src, const typename R::Mask* __restrict__ mask,
                                                             uint32_t n_groups, typename R::Mask set,
                                                             const uint8_t* __restrict__ valid,
                                                             uint32_t* __restrict__ counts)
{
    const size_t tid = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const typename R::Mask m = round_bits<R>(src, mask, n_groups, set, valid, g, (tid % Src::G) == 0);
    block_counts<R>(m, counts);
}

// Position of group g in check c's segment:
//   seg.start[c] + (offs[c*nb + block] - offs[c*nb]) + rank of g among the block's groups with bit c
// -- ascending group order within each segment, no atomics.
template <class R, class Src>
__global__ __launch_bounds__(kStagedBlock) void queue_kernel(Src src, const typename R::Mask* __restrict__ mask,
                                                             uint32_t n_groups, typename R::Mask set,
                                                             const uint8_t* __restrict__ valid,
                                                             const uint32_t* __restrict__ offs, SegTableT<R> seg,
                                                             uint32_t* __restrict__ items)
{
    using M = typename R::Mask;
    const size_t tid = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const M m = round_bits<R>(src, mask, n_groups, set, valid, g, (tid % Src::G) == 0);
    const int w = threadIdx.x >> 6;
    __shared__ uint32_t wcnt[kStagedBlock / 64][R::kChecks];
    for (int i = threadIdx.x; i < (kStagedBlock / 64) * R::kChecks; i += kStagedBlock) (&wcnt[0][0])[i] = 0u;
    __syncthreads();
    const M any = wave_or(m);
    for (M a = any; a; a &= a - 1) {
        const int c = mask_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        if (__lane_id() == 0) wcnt[w][c] = (uint32_t)__builtin_popcountll(b);
    }
    __syncthreads();
    const uint64_t below = (__lane_id() == 0) ? 0ull : (~0ull >> (64 - __lane_id()));
    const size_t nb = gridDim.x;
    for (M a = any; a; a &= a - 1) {
        const int c = mask_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        uint32_t base = seg.start[c] + (offs[(size_t)c * nb + blockIdx.x] - offs[(size_t)c * nb]);
        for (int i = 0; i < w; ++i) base += wcnt[i][c];
        if ((m >> c) & 1u) items[base + (uint32_t)__builtin_popcountll(b & below)] = g;
    }
}

// ---- stage 2: children, one check per wave ------------------------------------------------------
template <class R, class Src, bool EXT>
__global__ __launch_bounds__(kStagedBlock, R::kChildWavesPerEU) void children_kernel(Src src, SegTableT<R> seg,
                                                                                const uint32_t* __restrict__ items,
                                                                                EnvView env, float bx, float by,
                                                                                float bz, uint8_t* __restrict__ valid)
{
    using Grp = typename GrpOf<Src::G>::T;
    if constexpr (EXT) capt_stage_lds(env);  // the split tree's top levels into LDS (before any return)
    const size_t tid = (size_t)blockIdx.x * kStagedBlock + threadIdx.x;
    const uint32_t item = (uint32_t)(tid / Src::G);
    const int lane = (int)(tid % Src::G);
    if (item >= seg.start[R::kChecks]) return;  // wave-uniform (segments are wave-aligned)
    const uint32_t item0 = __builtin_amdgcn_readfirstlane(item);
    int c = 0;
    while (item0 >= seg.start[c + 1]) ++c;  // scalar: every wave holds one check
    const uint32_t g = items[item];
    if (g == kNoItem) return;  // segment padding (group-uniform)
    float v[R::D];
    src.load(g, lane, v);
    if (R::template children<Grp, EXT>(c, v, env, bx, by, bz) && lane == 0)
        valid[src.out(g)] = 0;  // every writer stores 0: the race is benign
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

    template <class Src>
    static hipError_t bound(const Src& src, uint32_t n_groups, const EnvView* env, float bx, float by, float bz,
                            M* mask, uint8_t* valid, uint32_t* counts, hipStream_t st)
    {
        if (n_groups == 0) return hipSuccess;
        const unsigned grid = grid_of<Src>(n_groups);
        if (env->n_hf > 0 || env->n_pc > 0)
            hipLaunchKernelGGL((bound_kernel<R, Src, true>), dim3(grid), dim3(kStagedBlock), 0, st, src, n_groups,
                               *env, bx, by, bz, mask, valid, counts);
        else
            hipLaunchKernelGGL((bound_kernel<R, Src, false>), dim3(grid), dim3(kStagedBlock), 0, st, src, n_groups,
                               *env, bx, by, bz, mask, valid, counts);
        return hipGetLastError();
    }

    template <class Src>
    static hipError_t count(const Src& src, const M* mask, uint32_t n_groups, M set, const uint8_t* valid,
                            uint32_t* counts, hipStream_t st)
    {
        hipLaunchKernelGGL((count_kernel<R, Src>), dim3(grid_of<Src>(n_groups)), dim3(kStagedBlock), 0, st, src, mask,
                           n_groups, set, valid, counts);
        return hipGetLastError();
    }

    template <class Src>
    static hipError_t queue(const Src& src, const M* mask, uint32_t n_groups, M set, const uint8_t* valid,
                            const uint32_t* offs, const uint32_t* seg, uint32_t* items, uint32_t n_items,
                            hipStream_t st)
    {
        hipError_t err = hipMemsetAsync(items, 0xFF, (size_t)n_items * sizeof(uint32_t), st);
        if (err != hipSuccess) return err;
        SegTableT<R> t;
        for (int c = 0; c <= R::kChecks; ++c) t.start[c] = seg[c];
        hipLaunchKernelGGL((queue_kernel<R, Src>), dim3(grid_of<Src>(n_groups)), dim3(kStagedBlock), 0, st, src, mask,
                           n_groups, set, valid, offs, t, items);
        return hipGetLastError();
    }

    template <class Src>
    static hipError_t children(const Src& src, const uint32_t* seg, const uint32_t* items, const EnvView* env,
                               float bx, float by, float bz, uint8_t* valid, hipStream_t st)
    {
        SegTableT<R> t;
        for (int c = 0; c <= R::kChecks; ++c) t.start[c] = seg[c];
        const size_t threads = (size_t)t.start[R::kChecks] * Src::G;
        if (threads == 0) return hipSuccess;
        const unsigned grid = (unsigned)((threads + kStagedBlock - 1) / kStagedBlock);
        if (env->n_hf > 0 || env->n_pc > 0)
            hipLaunchKernelGGL((children_kernel<R, Src, true>), dim3(grid), dim3(kStagedBlock), 0, st, src, t, items,
                               *env, bx, by, bz, valid);
        else
            hipLaunchKernelGGL((children_kernel<R, Src, false>), dim3(grid), dim3(kStagedBlock), 0, st, src, t, items,
                               *env, bx, by, bz, valid);
        return hipGetLastError();
    }

    // dispatch on the source kind: 0 configurations (s0 = q), 1 Halton samples (first, s0 = q_out
    // or NULL), 2 validate head (s0 = starts, s1 = goals), 3 validate tail (+ s2 = item_edge, s3 = off),
    // 4 full-mask tail (as 3, one result per block)
    template <class Fn>
    static hipError_t with_source(int kind, const void* s0, const void* s1, const void* s2, const void* s3,
                                  uint64_t first, Fn fn)
    {
        switch (kind) {
        case 0:
            return fn(SrcConfigsT<R>{(const float*)s0});
        case 1:
            return fn(SrcSamplesT<R>{first, (float*)s0, nullptr});
        case 2:
            return fn(SrcHeadT<R>{(const float*)s0, (const float*)s1});
        case 3:
            return fn(SrcTailT<R>{(const float*)s0, (const float*)s1, (const uint32_t*)s2, (const uint32_t*)s3});
        case 4:
            return fn(SrcTailMaskT<R>{(const float*)s0, (const float*)s1, (const uint32_t*)s2, (const uint32_t*)s3});
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
    int vgpu_##NAME##_staged_mask_bytes(void) { return (int)sizeof(typename R::Mask); }                              \
    uint32_t vgpu_##NAME##_staged_blocks(int kind, uint32_t n_groups)                                                \
    {                                                                                                                \
        const size_t G = kind >= 2 ? 8 : 1;                                                                          \
        return (uint32_t)(((size_t)n_groups * G + vgpu::kStagedBlock - 1) / vgpu::kStagedBlock);                     \
    }                                                                                                                \
    hipError_t vgpu_##NAME##_staged_bound(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          uint64_t first, uint32_t n_groups, const EnvView* env, float bx, float by, \
                                          float bz, void* mask, uint8_t* valid, uint32_t* counts, hipStream_t st)    \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        return H::with_source(kind, s0, s1, s2, s3, first, [&](auto src) {                                          \
            return H::bound(src, n_groups, env, bx, by, bz, (typename R::Mask*)mask, valid, counts, st);             \
        });                                                                                                          \
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
    hipError_t vgpu_##NAME##_staged_queue(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          const void* mask, uint32_t n_groups, uint64_t set, const uint8_t* valid,   \
                                          const uint32_t* offs, const uint32_t* seg, uint32_t* items,                \
                                          uint32_t n_items, hipStream_t st)                                          \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        if (n_groups == 0) return hipSuccess;                                                                        \
        return H::with_source(kind, s0, s1, s2, s3, 0, [&](auto src) {                                              \
            return H::queue(src, (const typename R::Mask*)mask, n_groups, (typename R::Mask)set, valid, offs, seg,   \
                            items, n_items, st);                                                                     \
        });                                                                                                          \
    }                                                                                                                \
    hipError_t vgpu_##NAME##_staged_children(int kind, const void* s0, const void* s1, const void* s2,               \
                                             const void* s3, uint64_t first, const uint32_t* seg,                    \
                                             const uint32_t* items, const EnvView* env, float bx, float by,          \
                                             float bz, uint8_t* valid, hipStream_t st)                               \
    {                                                                                                                \
        using H = vgpu::StagedHost<R>;                                                                               \
        return H::with_source(kind, s0, s1, s2, s3, first, [&](auto src) {                                          \
            if constexpr (std::is_same<decltype(src), vgpu::SrcSamplesT<R>>::value) {                                \
                src.q_in = src.q_out; /* the samples the bound stage wrote */                                         \
                src.q_out = nullptr;                                                                                 \
            }                                                                                                        \
            return H::children(src, seg, items, env, bx, by, bz, valid, st);                                         \
        });                                                                                                          \
    }                                                                                                                \
    }
