// vgpu_ur5.hip -- UR5 (robots/ur5.hh: 6 dof, 36 spheres, 15 link checks incl. 6 leaves + 33 self
// link pairs of ur5/fk.hh:1079-3023, resolution 32) through the generic robot kernels
// (vgpu_robot.hh) and the staged pipeline (vgpu_staged.hh, 48 checks -> 64-bit masks).
#include <utility>

#include "vgpu_robot.hh"
#include "vgpu_staged.hh"

#include "gen/ur5_fk.inc"

namespace vgpu {

struct Ur5R {
    static constexpr int D = 6;
    static constexpr int kRes = 32;  // robots/ur5.hh:12
    static constexpr int kSpheres = 36;
    static constexpr int kWavesPerEU = 6;
    static constexpr int kChildWavesPerEU = 6;
    static constexpr int kChecks = ur5_n_checks;
    using Mask = ur5_mask_t;
    static constexpr Mask kEnvChecks = ur5_env_check_bits;
    static constexpr const float* s_m = ur5_s_m;
    static constexpr const float* s_a = ur5_s_a;

    template <class Grp, bool EXT, size_t... I>
    __device__ static __forceinline__ bool fkcc_(const float* v, const EnvView& env, std::index_sequence<I...>)
    {
        return ur5_fkcc<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool fkcc(const float* v, const EnvView& env)
    {
        return fkcc_<Grp, EXT>(v, env, std::make_index_sequence<D>{});
    }
    template <size_t... I>
    __device__ static __forceinline__ void fk_(const float* v, float* out, size_t ld, std::index_sequence<I...>)
    {
        ur5_sphere_fk_store(v[I]..., 0.0f, 0.0f, 0.0f, out, ld);
    }
    __device__ static __forceinline__ void sphere_fk_store(const float* v, float* out, size_t ld)
    {
        fk_(v, out, ld, std::make_index_sequence<D>{});
    }
    // staged hooks
    __device__ static __forceinline__ void sample(uint64_t k, float v[D]) { sample_d<D>(k, ur5_s_m, ur5_s_a, v); }
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
        return ur5_bound_mask<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
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
        return ur5_children<Grp, EXT>(c, v[I]..., env, 0.0f, 0.0f, 0.0f);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool children(int c, const float* v, const EnvView& env, const Bases&)
    {
        return children_<Grp, EXT>(c, v, env, std::make_index_sequence<D>{});
    }
};

}  // namespace vgpu

VGPU_ROBOT_EXPORTS(vgpu::Ur5R, ur5, true)
VGPU_STAGED_EXPORTS(vgpu::Ur5R, ur5)
