// vgpu_pair.hip -- gfx950 kernels for the two-Panda composite of BASELINE configs[4]
// (14 dof = arm A joints 0..6 at base A, arm B joints 7..13 at base B).
//
// The reference has no composite robot (SURVEY §0 finding 10); validity is composed from its
// primitives exactly as oracle/vamp_oracle.c vo_pair_fkcc_block states it:
//   fkcc_A && fkcc_B && !inter(A, B)
// with fkcc the generated Panda hierarchy (panda/fk.hh:1335-6276) at each arm's base and inter the
// link-bounding-first sphere test between the arms (gen/panda_pair.inc).  validate_motion over
// the 14-dof configuration uses the reference rake (planning/validate.hh:23-75, resolution 32)
// with the two-register l2_norm.  Same two-phase head/tail split as the single-arm kernels.
#include "vgpu_rake.hh"

#include "gen/panda_fk.inc"
#include "gen/panda_pair.inc"

#ifndef VGPU_PAIR_WAVES_PER_EU
#define VGPU_PAIR_WAVES_PER_EU 4
#endif

namespace vgpu {

constexpr int kPairBlock = 256;
constexpr int kPairDim = 14;
constexpr int kPairRes = 32;  // robots/panda_base.hh:21

struct PairBase {
    float ax, ay, az, bx, by, bz;
};

#define PAIR_A(v) v[0], v[1], v[2], v[3], v[4], v[5], v[6]
#define PAIR_B(v) v[7], v[8], v[9], v[10], v[11], v[12], v[13]

template <class Grp, bool EXT>
__device__ __forceinline__ bool pair_fkcc(const float v[kPairDim], const EnvView& env, const PairBase& pb)
{
    if (!panda_fkcc<Grp, EXT>(PAIR_A(v), env, pb.ax, pb.ay, pb.az)) return false;
    if (!panda_fkcc<Grp, EXT>(PAIR_B(v), env, pb.bx, pb.by, pb.bz)) return false;
    return !panda_pair_inter<Grp>(PAIR_A(v), PAIR_B(v), pb.ax, pb.ay, pb.az, pb.bx, pb.by, pb.bz);
}

template <bool EXT>
__global__ __launch_bounds__(kPairBlock, VGPU_PAIR_WAVES_PER_EU) void pair_fkcc_kernel(
    const float* __restrict__ q, size_t n, EnvView env, PairBase pb, uint8_t* __restrict__ valid)
{
    const size_t i = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    if (i >= n) return;
    float v[kPairDim];
#pragma unroll
    for (int j = 0; j < kPairDim; ++j) v[j] = q[kPairDim * i + j];
    valid[i] = pair_fkcc<Grp1, EXT>(v, env, pb) ? 1 : 0;
}

template <bool EXT>
__global__ __launch_bounds__(kPairBlock, VGPU_PAIR_WAVES_PER_EU) void pair_validate_head_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, size_t n_edges, EnvView env, PairBase pb,
    uint8_t* __restrict__ ok, int32_t* __restrict__ n_blocks, uint32_t* __restrict__ cnt)
{
    const size_t tid = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    const size_t e = tid >> 3;  // one 8-lane rake group per edge
    const int lane = (int)(tid & 7);
    if (e >= n_edges) return;   // group-uniform
    const float* s = starts + kPairDim * e;
    const RakeD<kPairDim> rk = rake_setup_d<kPairDim, kPairRes>(s, goals + kPairDim * e);
    float b[kPairDim];
    rake_block_d<kPairDim>(s, rk, lane, 0, b);
    const bool valid = pair_fkcc<Grp8, EXT>(b, env, pb);
    if (lane == 0) {
        ok[e] = valid ? 1 : 0;
        if (n_blocks) n_blocks[e] = rk.n;
        cnt[e] = (valid && rk.n > 1) ? (uint32_t)(rk.n - 1) : 0u;
    }
}

template <bool EXT>
__global__ __launch_bounds__(kPairBlock, VGPU_PAIR_WAVES_PER_EU) void pair_validate_tail_kernel(
    const float* __restrict__ starts, const float* __restrict__ goals, const uint32_t* __restrict__ item_edge,
    const uint32_t* __restrict__ off, size_t n_items, EnvView env, PairBase pb, uint8_t* __restrict__ ok)
{
    const size_t tid = (size_t)blockIdx.x * kPairBlock + threadIdx.x;
    const size_t it = tid >> 3;
    const int lane = (int)(tid & 7);
    if (it >= n_items) return;
    const uint32_t e = item_edge[it];
    const int k = (int)(it - off[e]) + 1;
    const float* s = starts + kPairDim * (size_t)e;
    const RakeD<kPairDim> rk = rake_setup_d<kPairDim, kPairRes>(s, goals + kPairDim * (size_t)e);
    float b[kPairDim];
    rake_block_d<kPairDim>(s, rk, lane, k, b);
    const bool valid = pair_fkcc<Grp8, EXT>(b, env, pb);
    if (lane == 0 && !valid) ok[e] = 0;
}

}  // namespace vgpu

static bool pair_has_ext(const EnvView* env) { return env->n_hf > 0 || env->n_pc > 0; }
static unsigned pair_grid(size_t threads) { return (unsigned)((threads + vgpu::kPairBlock - 1) / vgpu::kPairBlock); }

extern "C" {

hipError_t vgpu_launch_pair_fkcc(const float* q, size_t n, const EnvView* env, const float base[6], uint8_t* valid,
                                 hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const vgpu::PairBase pb{base[0], base[1], base[2], base[3], base[4], base[5]};
    if (pair_has_ext(env))
        hipLaunchKernelGGL(vgpu::pair_fkcc_kernel<true>, dim3(pair_grid(n)), dim3(vgpu::kPairBlock), 0, st, q, n,
                           *env, pb, valid);
    else
        hipLaunchKernelGGL(vgpu::pair_fkcc_kernel<false>, dim3(pair_grid(n)), dim3(vgpu::kPairBlock), 0, st, q, n,
                           *env, pb, valid);
    return hipGetLastError();
}

hipError_t vgpu_launch_pair_validate_head(const float* starts, const float* goals, size_t n_edges, const EnvView* env,
                                          const float base[6], uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                          hipStream_t st)
{
    hipError_t err = hipMemsetAsync(cnt + n_edges, 0, sizeof(uint32_t), st);
    if (err != hipSuccess || n_edges == 0) return err;
    const vgpu::PairBase pb{base[0], base[1], base[2], base[3], base[4], base[5]};
    const unsigned grid = pair_grid(n_edges * 8);
    if (pair_has_ext(env))
        hipLaunchKernelGGL(vgpu::pair_validate_head_kernel<true>, dim3(grid), dim3(vgpu::kPairBlock), 0, st, starts,
                           goals, n_edges, *env, pb, ok, n_blocks, cnt);
    else
        hipLaunchKernelGGL(vgpu::pair_validate_head_kernel<false>, dim3(grid), dim3(vgpu::kPairBlock), 0, st, starts,
                           goals, n_edges, *env, pb, ok, n_blocks, cnt);
    return hipGetLastError();
}

hipError_t vgpu_launch_pair_validate_tail(const float* starts, const float* goals, size_t n_items, const EnvView* env,
                                          const float base[6], uint8_t* ok, const uint32_t* off,
                                          const uint32_t* item_edge, hipStream_t st)
{
    if (n_items == 0) return hipSuccess;
    const vgpu::PairBase pb{base[0], base[1], base[2], base[3], base[4], base[5]};
    const unsigned grid = pair_grid(n_items * 8);
    if (pair_has_ext(env))
        hipLaunchKernelGGL(vgpu::pair_validate_tail_kernel<true>, dim3(grid), dim3(vgpu::kPairBlock), 0, st, starts,
                           goals, item_edge, off, n_items, *env, pb, ok);
    else
        hipLaunchKernelGGL(vgpu::pair_validate_tail_kernel<false>, dim3(grid), dim3(vgpu::kPairBlock), 0, st, starts,
                           goals, item_edge, off, n_items, *env, pb, ok);
    return hipGetLastError();
}

}  // extern "C"
