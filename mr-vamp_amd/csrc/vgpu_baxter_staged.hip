// vgpu_baxter_staged.hip -- the Baxter (robots/baxter.hh: 14-dof dual arm, 388 checks of baxter/fk.hh:
// 33 link checks incl. 8 leaves + 355 self link pairs, resolution 64) through the staged pipeline
// (vgpu_staged.hh).  388 checks exceed one 64-bit check mask, so the check list runs in 7 chunks of <= 64
// (gen/baxter_fk.inc baxter_bound_mask_<k>), each a CHAINED staged pass over the same groups: the
// reference's result is an OR over checks, so the passes AND their verdicts into one flag and a group
// invalidated by an earlier chunk skips every stage of the later ones.  A chunk's bound stage evaluates
// only the frames its own checks need.
#include <utility>

#include "vgpu_rake.hh"
#include "vgpu_staged.hh"

#include "gen/baxter_fk.inc"

#ifndef VGPU_BAXTER_BOUND_WAVES
#define VGPU_BAXTER_BOUND_WAVES 5
#endif
#ifndef VGPU_BAXTER_CHILD_WAVES
#define VGPU_BAXTER_CHILD_WAVES 6
#endif

namespace vgpu {

template <int K>
struct BaxterChunkR {
    static constexpr int D = 14;
    static constexpr int kRes = 64;  // robots/baxter.hh:12
    static constexpr int kFirst = K * baxter_chunk;
    static constexpr int kChecks =
        (baxter_n_checks - kFirst) < baxter_chunk ? (baxter_n_checks - kFirst) : baxter_chunk;
    static constexpr int kWavesPerEU = VGPU_BAXTER_BOUND_WAVES;
    static constexpr int kChildWavesPerEU = VGPU_BAXTER_CHILD_WAVES;
    static constexpr unsigned kSourceKinds = 1u | 2u | 4u | 8u;  // configurations, samples, head, tail
    using Mask = uint64_t;
    static constexpr Mask kEnvChecks = baxter_env_check_bits_chunk[K];

    __device__ static __forceinline__ void sample(uint64_t k, float v[D]) { sample_d<D>(k, baxter_s_m, baxter_s_a, v); }
    __device__ static __forceinline__ void head(const float* s, const float* g, int lane, float v[D])
    {
        const RakeD<D> rk = rake_setup_d<D, kRes>(s, g);
        rake_block_d<D>(s, rk, lane, 0, v);
    }
    __device__ static __forceinline__ void tail(const float* s, const float* g, int lane, int k, float v[D])
    {
        const RakeD<D> rk = rake_setup_d<D, kRes>(s, g);
        rake_block_d<D>(s, rk, lane, k, v);
    }
    template <class Grp, bool EXT, size_t... I>
    __device__ static __forceinline__ Mask bound_(const float* v, const EnvView& env, std::index_sequence<I...>)
    {
        if constexpr (K == 0) return baxter_bound_mask_0<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
        else if constexpr (K == 1) return baxter_bound_mask_1<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
        else if constexpr (K == 2) return baxter_bound_mask_2<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
        else if constexpr (K == 3) return baxter_bound_mask_3<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
        else if constexpr (K == 4) return baxter_bound_mask_4<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
        else if constexpr (K == 5) return baxter_bound_mask_5<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
        else return baxter_bound_mask_6<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ Mask bound(const float* v, const EnvView& env, const Bases&)
    {
        return bound_<Grp, EXT>(v, env, std::make_index_sequence<D>{});
    }
    template <class Grp, bool EXT, size_t... I>
    __device__ static __forceinline__ bool children_(int c, const float* v, const EnvView& env,
                                                     std::index_sequence<I...>)
    {
        return baxter_children<Grp, EXT>(kFirst + c, v[I]..., env, 0.0f, 0.0f, 0.0f);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool children(int c, const float* v, const EnvView& env, const Bases&)
    {
        return children_<Grp, EXT>(c, v, env, std::make_index_sequence<D>{});
    }
};
static_assert(baxter_n_chunks == 7, "vgpu_api.cpp chains 7 chunks");

}  // namespace vgpu

// one chunk per object file (the Makefile compiles this TU once per VGPU_CHUNK = 0..6, in parallel)
#ifndef VGPU_CHUNK
#error "compile with -DVGPU_CHUNK=<0..6>"
#endif
#define VGPU_CAT_(a, b) a##b
#define VGPU_CAT(a, b) VGPU_CAT_(a, b)
#define VGPU_STAGED_EXPORTS_X(R, NAME) VGPU_STAGED_EXPORTS(R, NAME)  // expands NAME before the pasting
VGPU_STAGED_EXPORTS_X(vgpu::BaxterChunkR<VGPU_CHUNK>, VGPU_CAT(baxter_c, VGPU_CHUNK))
