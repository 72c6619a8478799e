// vgpu_staged.hip -- staged evaluation of the Panda collision hierarchy.
//
// The monolithic kernels (vgpu_kernels.hip) run FK and the 32 hierarchical checks of
// fk.hh:1335-6276 in one divergent pass: a wave executes a check's children whenever ANY of
// its groups' bounding tests fires, so on the bench workloads only 17 % (fkcc) / 37 % (validate
// head) of the VALU lanes were active.  Here the same hierarchy runs in two uniform stages:
//
//   bound     one group per rake block (G lanes): FK + all bounding tests, no children, no
//             early exit; writes a 32-bit mask (bit c = check c's bounding test fired for the
//             group) and counts the fired (group, check) pairs per check;
//   queue     scatters each fired (group, check) into check c's segment of an item list;
//             segments are padded to whole waves, so every wave holds ONE check;
//   children  one wave per 64/G items of one check: recomputes the frames that check needs and
//             tests its children; a firing child clears the group's result.
//
// Result: valid <=> no check has both its bounding test and one of its children firing -- the
// reference's early-exit loop is an OR over checks, so the evaluation order is free.  Groups are
// described by a Source: configurations (fkcc, G = 1), Halton samples (G = 1), first rake blocks
// of edges (validate head, G = 8), or (edge, back-step) items (validate tail, G = 8).
#include "vgpu_panda.hh"

namespace vgpu {

constexpr int kChecks = panda_n_checks;
constexpr uint32_t kNoItem = 0xFFFFFFFFu;

struct SegTable {
    uint32_t start[kChecks + 1];  // check c owns items [start[c], start[c+1]), wave-aligned
};

// ---- group sources ----------------------------------------------------------------------------
struct SrcConfigs {  // fkcc: one configuration per group
    static constexpr int G = 1;
    static constexpr bool kInit = true;
    const float* q;
    __device__ void load(uint32_t g, int, float v[7]) const
    {
        const float* p = q + 7 * (size_t)g;
#pragma unroll
        for (int j = 0; j < 7; ++j) v[j] = p[j];
    }
    __device__ uint32_t out(uint32_t g) const { return g; }
};

struct SrcSamples {  // Halton draw first + g, scaled
    static constexpr int G = 1;
    static constexpr bool kInit = true;
    uint64_t first;
    float* q_out;  // optional copy of the sample (written by the bound stage)
    __device__ void load(uint32_t g, int, float v[7]) const { panda_sample(first + g, v); }
    __device__ uint32_t out(uint32_t g) const { return g; }
};

struct SrcHead {  // validate head: block 0 of edge g
    static constexpr int G = 8;
    static constexpr bool kInit = true;
    const float* starts;
    const float* goals;
    __device__ void load(uint32_t g, int lane, float v[7]) const
    {
        const float* s = starts + 7 * (size_t)g;
        const Rake rk = rake_setup(s, goals + 7 * (size_t)g);
        rake_block(s, rk, lane, 0, v);
    }
    __device__ uint32_t out(uint32_t g) const { return g; }
};

struct SrcTail {  // validate tail: item g = (edge, back-step k), result into the edge's flag
    static constexpr int G = 8;
    static constexpr bool kInit = false;  // the edge flag is shared by its items
    const float* starts;
    const float* goals;
    const uint32_t* item_edge;
    const uint32_t* off;
    __device__ void load(uint32_t g, int lane, float v[7]) const
    {
        const uint32_t e = item_edge[g];
        const int k = (int)(g - off[e]) + 1;
        const float* s = starts + 7 * (size_t)e;
        const Rake rk = rake_setup(s, goals + 7 * (size_t)e);
        rake_block(s, rk, lane, k, v);
    }
    __device__ uint32_t out(uint32_t g) const { return item_edge[g]; }
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

// per-(check, block) counts of the set bits of m over the block, check-major:
// counts[c * gridDim.x + blockIdx.x]
__device__ __forceinline__ void block_counts(uint32_t m, uint32_t* __restrict__ counts)
{
    __shared__ uint32_t cnt[kChecks];
    if (threadIdx.x < kChecks) cnt[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t any = m;
    for (int off = 32; off >= 1; off >>= 1) any |= __shfl_xor(any, off);
    any = __builtin_amdgcn_readfirstlane(any);
    for (uint32_t a = any; a; a &= a - 1u) {
        const int c = __builtin_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        if (__lane_id() == 0) atomicAdd(&cnt[c], (uint32_t)__builtin_popcountll(b));
    }
    __syncthreads();
    if (threadIdx.x < kChecks) counts[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = cnt[threadIdx.x];
}

// ---- stage 1: bounding masks ---------------------------------------------------------------
template <class Src, bool EXT>
__global__ __launch_bounds__(kBlock, VGPU_WAVES_PER_EU) void bound_kernel(Src src, uint32_t n_groups, EnvView env,
                                                                          float bx, float by, float bz,
                                                                          uint32_t* __restrict__ mask,
                                                                          uint8_t* __restrict__ valid,
                                                                          uint32_t* __restrict__ counts)
{
    using Grp = typename GrpOf<Src::G>::T;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const int lane = (int)(tid % Src::G);
    uint32_t m = 0u;
    if (g < n_groups) {  // group-uniform
        float v[7];
        src.load(g, lane, v);
        if constexpr (std::is_same<Src, SrcSamples>::value) {
            if (src.q_out) {
#pragma unroll
                for (int j = 0; j < 7; ++j) src.q_out[7 * (size_t)g + j] = v[j];
            }
        }
        m = panda_bound_mask<Grp, EXT>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], env, bx, by, bz);
        if (lane == 0) {
            mask[g] = m;
            if constexpr (Src::kInit) valid[src.out(g)] = 1;
        }
    }
    // the first round's per-(check, block) counts: every group is still valid here (tail items
    // exist only for edges that passed the head)
    if (lane != 0) m = 0u;
    block_counts(m, counts);
}

// ---- rounds: the fired (group, check) pairs of a set of checks, for groups still valid ----------------
// Checks run in rounds (e.g. the environment checks, then the self checks): a group invalidated by
// an earlier round contributes no work to later ones, which recovers the reference's early exit.
// Both kernels use the bound kernel's grid; per-(check, block) counts are stored check-major,
// counts[c * blocks + block], for one flat exclusive scan.
template <class Src>
__device__ __forceinline__ uint32_t round_bits(const Src& src, const uint32_t* __restrict__ mask, uint32_t n_groups,
                                               uint32_t set, const uint8_t* __restrict__ valid, uint32_t g,
                                               bool lead)
{
    if (!lead || g >= n_groups) return 0u;
    const uint32_t m = mask[g] & set;
    return (m && valid[src.out(g)]) ? m : 0u;
}

template <class Src>
__global__ __launch_bounds__(kBlock) void count_kernel(Src src, const uint32_t* __restrict__ mask, uint32_t n_groups,
                                                       uint32_t set, const uint8_t* __restrict__ valid,
                                                       uint32_t* __restrict__ counts)
{
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const uint32_t m = round_bits(src, mask, n_groups, set, valid, g, (tid % Src::G) == 0);
    block_counts(m, counts);
}

// Position of group g in check c's segment:
//   seg.start[c] + (offs[c*nb + block] - offs[c*nb]) + rank of g among the block's groups with bit c
// -- ascending group order within each segment, no atomics.
template <class Src>
__global__ __launch_bounds__(kBlock) void queue_kernel(Src src, const uint32_t* __restrict__ mask, uint32_t n_groups,
                                                       uint32_t set, const uint8_t* __restrict__ valid,
                                                       const uint32_t* __restrict__ offs, SegTable seg,
                                                       uint32_t* __restrict__ items)
{
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t g = (uint32_t)(tid / Src::G);
    const uint32_t m = round_bits(src, mask, n_groups, set, valid, g, (tid % Src::G) == 0);
    const int w = threadIdx.x >> 6;
    __shared__ uint32_t wcnt[kBlock / 64][kChecks];
    for (int i = threadIdx.x; i < (kBlock / 64) * kChecks; i += kBlock) (&wcnt[0][0])[i] = 0u;
    __syncthreads();
    uint32_t any = m;
    for (int off = 32; off >= 1; off >>= 1) any |= __shfl_xor(any, off);
    any = __builtin_amdgcn_readfirstlane(any);
    for (uint32_t a = any; a; a &= a - 1u) {
        const int c = __builtin_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        if (__lane_id() == 0) wcnt[w][c] = (uint32_t)__builtin_popcountll(b);
    }
    __syncthreads();
    const uint64_t below = (__lane_id() == 0) ? 0ull : (~0ull >> (64 - __lane_id()));
    const size_t nb = gridDim.x;
    for (uint32_t a = any; a; a &= a - 1u) {
        const int c = __builtin_ctz(a);
        const uint64_t b = __builtin_amdgcn_ballot_w64((m >> c) & 1u);
        uint32_t base = seg.start[c] + (offs[(size_t)c * nb + blockIdx.x] - offs[(size_t)c * nb]);
        for (int i = 0; i < w; ++i) base += wcnt[i][c];
        if ((m >> c) & 1u) items[base + (uint32_t)__builtin_popcountll(b & below)] = g;
    }
}

// ---- stage 2: children, one check per wave ------------------------------------------------------
template <class Src, bool EXT>
__global__ __launch_bounds__(kBlock, VGPU_WAVES_PER_EU) void children_kernel(Src src, SegTable seg,
                                                                             const uint32_t* __restrict__ items,
                                                                             EnvView env, float bx, float by,
                                                                             float bz, uint8_t* __restrict__ valid)
{
    using Grp = typename GrpOf<Src::G>::T;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t item = (uint32_t)(tid / Src::G);
    const int lane = (int)(tid % Src::G);
    if (item >= seg.start[kChecks]) return;  // wave-uniform (segments are wave-aligned)
    const uint32_t item0 = __builtin_amdgcn_readfirstlane(item);
    int c = 0;
    while (item0 >= seg.start[c + 1]) ++c;  // scalar: every wave holds one check
    const uint32_t g = items[item];
    if (g == kNoItem) return;  // segment padding (group-uniform)
    float v[7];
    src.load(g, lane, v);
    if (panda_children<Grp, EXT>(c, v[0], v[1], v[2], v[3], v[4], v[5], v[6], env, bx, by, bz) && lane == 0)
        valid[src.out(g)] = 0;  // every writer stores 0: the race is benign
}

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
    cnt[e] = (ok[e] && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
}

}  // namespace vgpu

// ---- host-side launch helpers (called by vgpu_api.cpp) ------------------------------------------
// A staged pass over n_groups groups of one source:
//   bound (per-block counts) -> exclusive scan -> [caller: D2H check totals, segment table]
//   -> queue -> children
// The caller owns the workspace: mask[n_groups], counts/offs[kChecks * blocks + 1], items[].
namespace {
template <class Src>
hipError_t launch_bound(const Src& src, uint32_t n_groups, const EnvView* env, float bx, float by, float bz,
                        uint32_t* mask, uint8_t* valid, uint32_t* counts, hipStream_t st)
{
    const size_t threads = (size_t)n_groups * Src::G;
    const unsigned grid = (unsigned)((threads + vgpu::kBlock - 1) / vgpu::kBlock);
    if (n_groups == 0) return hipSuccess;
    if (env->n_hf > 0 || env->n_pc > 0)
        hipLaunchKernelGGL((vgpu::bound_kernel<Src, true>), dim3(grid), dim3(vgpu::kBlock), 0, st, src, n_groups,
                           *env, bx, by, bz, mask, valid, counts);
    else
        hipLaunchKernelGGL((vgpu::bound_kernel<Src, false>), dim3(grid), dim3(vgpu::kBlock), 0, st, src, n_groups,
                           *env, bx, by, bz, mask, valid, counts);
    return hipGetLastError();
}

template <class Src>
hipError_t launch_count(const Src& src, const uint32_t* mask, uint32_t n_groups, uint32_t set, const uint8_t* valid,
                        uint32_t* counts, hipStream_t st)
{
    const unsigned grid = (unsigned)(((size_t)n_groups * Src::G + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL((vgpu::count_kernel<Src>), dim3(grid), dim3(vgpu::kBlock), 0, st, src, mask, n_groups, set,
                       valid, counts);
    return hipGetLastError();
}

template <class Src>
hipError_t launch_queue(const Src& src, const uint32_t* mask, uint32_t n_groups, uint32_t set, const uint8_t* valid,
                        const uint32_t* offs, const uint32_t* seg, uint32_t* items, uint32_t n_items, hipStream_t st)
{
    hipError_t err = hipMemsetAsync(items, 0xFF, (size_t)n_items * sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    vgpu::SegTable t;
    for (int c = 0; c <= vgpu::kChecks; ++c) t.start[c] = seg[c];
    const unsigned grid = (unsigned)(((size_t)n_groups * Src::G + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL((vgpu::queue_kernel<Src>), dim3(grid), dim3(vgpu::kBlock), 0, st, src, mask, n_groups, set,
                       valid, offs, t, items);
    return hipGetLastError();
}

template <class Src>
hipError_t launch_children(const Src& src, const uint32_t* seg, const uint32_t* items, const EnvView* env, float bx,
                           float by, float bz, uint8_t* valid, hipStream_t st)
{
    vgpu::SegTable t;
    for (int c = 0; c <= vgpu::kChecks; ++c) t.start[c] = seg[c];
    const size_t threads = (size_t)t.start[vgpu::kChecks] * Src::G;
    if (threads == 0) return hipSuccess;
    const unsigned grid = (unsigned)((threads + vgpu::kBlock - 1) / vgpu::kBlock);
    if (env->n_hf > 0 || env->n_pc > 0)
        hipLaunchKernelGGL((vgpu::children_kernel<Src, true>), dim3(grid), dim3(vgpu::kBlock), 0, st, src, t, items,
                           *env, bx, by, bz, valid);
    else
        hipLaunchKernelGGL((vgpu::children_kernel<Src, false>), dim3(grid), dim3(vgpu::kBlock), 0, st, src, t, items,
                           *env, bx, by, bz, valid);
    return hipGetLastError();
}

// dispatch on the source kind: 0 configurations (src0 = q), 1 Halton samples (first, src0 = q_out
// or NULL), 2 validate head (src0 = starts, src1 = goals), 3 validate tail (+ src2 = item_edge,
// src3 = off)
template <class Fn>
hipError_t with_source(int kind, const void* s0, const void* s1, const void* s2, const void* s3, uint64_t first,
                       Fn fn)
{
    switch (kind) {
    case 0:
        return fn(vgpu::SrcConfigs{(const float*)s0});
    case 1:
        return fn(vgpu::SrcSamples{first, (float*)s0});
    case 2:
        return fn(vgpu::SrcHead{(const float*)s0, (const float*)s1});
    case 3:
        return fn(vgpu::SrcTail{(const float*)s0, (const float*)s1, (const uint32_t*)s2, (const uint32_t*)s3});
    }
    return hipErrorInvalidValue;
}
}  // namespace

extern "C" {

int vgpu_staged_checks(void) { return vgpu::kChecks; }

// bit c set for the environment checks (the rest are self checks), in check order
uint32_t vgpu_staged_env_checks(void) { return panda_env_check_bits; }

uint32_t vgpu_staged_blocks(int kind, uint32_t n_groups)
{
    const size_t G = kind >= 2 ? 8 : 1;
    return (uint32_t)(((size_t)n_groups * G + vgpu::kBlock - 1) / vgpu::kBlock);
}

hipError_t vgpu_launch_staged_bound(int kind, const void* s0, const void* s1, const void* s2, const void* s3,
                                    uint64_t first, uint32_t n_groups, const EnvView* env, float bx, float by,
                                    float bz, uint32_t* mask, uint8_t* valid, uint32_t* counts, hipStream_t st)
{
    return with_source(kind, s0, s1, s2, s3, first,
                       [&](auto src) { return launch_bound(src, n_groups, env, bx, by, bz, mask, valid, counts, st); });
}

hipError_t vgpu_launch_staged_count(int kind, const void* s0, const void* s1, const void* s2, const void* s3,
                                    const uint32_t* mask, uint32_t n_groups, uint32_t set, const uint8_t* valid,
                                    uint32_t* counts, hipStream_t st)
{
    if (n_groups == 0) return hipSuccess;
    return with_source(kind, s0, s1, s2, s3, 0,
                       [&](auto src) { return launch_count(src, mask, n_groups, set, valid, counts, st); });
}

hipError_t vgpu_launch_staged_queue(int kind, const void* s0, const void* s1, const void* s2, const void* s3,
                                    const uint32_t* mask, uint32_t n_groups, uint32_t set, const uint8_t* valid,
                                    const uint32_t* offs, const uint32_t* seg, uint32_t* items, uint32_t n_items,
                                    hipStream_t st)
{
    if (n_groups == 0) return hipSuccess;
    return with_source(kind, s0, s1, s2, s3, 0, [&](auto src) {
        return launch_queue(src, mask, n_groups, set, valid, offs, seg, items, n_items, st);
    });
}

hipError_t vgpu_launch_staged_children(int kind, const void* s0, const void* s1, const void* s2, const void* s3,
                                       uint64_t first, const uint32_t* seg, const uint32_t* items,
                                       const EnvView* env, float bx, float by, float bz, uint8_t* valid,
                                       hipStream_t st)
{
    return with_source(kind, s0, s1, s2, s3, first, [&](auto src) {
        if constexpr (std::is_same<decltype(src), vgpu::SrcSamples>::value) src.q_out = nullptr;
        return launch_children(src, seg, items, env, bx, by, bz, valid, st);
    });
}

hipError_t vgpu_launch_tail_counts(const float* starts, const float* goals, size_t n_edges, const uint8_t* ok,
                                   int32_t* n_blocks, uint32_t* cnt, hipStream_t st)
{
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess || n_edges == 0) return err;
    const unsigned grid = (unsigned)((n_edges + vgpu::kBlock - 1) / vgpu::kBlock);
    hipLaunchKernelGGL(vgpu::tail_counts_kernel, dim3(grid), dim3(vgpu::kBlock), 0, st, starts, goals, n_edges, ok,
                       n_blocks, cnt);
    return hipGetLastError();
}

}  // extern "C"
