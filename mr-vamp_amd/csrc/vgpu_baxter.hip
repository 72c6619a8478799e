// vgpu_baxter.hip -- Baxter (robots/baxter.hh: 14-dof dual arm, 75 spheres, 33 link checks incl.
// 8 leaves + 355 self link pairs of baxter/fk.hh, resolution 64) through the generic robot kernels
// (vgpu_robot.hh) -- the monolithic kernels (VAMP_AMD_STAGED=0); the staged pipeline runs the 388 checks
// in 7 chained chunks (vgpu_baxter_staged.hip).
// Its validate_motion distance is the two-register FloatVector<14>::l2_norm (ref_probe "l2norm").
#include <utility>

#include "vgpu_robot.hh"

#include "gen/baxter_fk.inc"

namespace vgpu {

struct BaxterR {
    static constexpr int D = 14;
    static constexpr int kRes = 64;  // robots/baxter.hh:12
    static constexpr int kSpheres = 75;
    static constexpr int kWavesPerEU = 4;
    static constexpr const float* s_m = baxter_s_m;
    static constexpr const float* s_a = baxter_s_a;

    template <class Grp, bool EXT, size_t... I>
    __device__ static __forceinline__ bool fkcc_(const float* v, const EnvView& env, std::index_sequence<I...>)
    {
        return baxter_fkcc<Grp, EXT>(v[I]..., env, 0.0f, 0.0f, 0.0f);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool fkcc(const float* v, const EnvView& env)
    {
        return fkcc_<Grp, EXT>(v, env, std::make_index_sequence<D>{});
    }
    template <size_t... I>
    __device__ static __forceinline__ void fk_(const float* v, float* out, size_t ld, std::index_sequence<I...>)
    {
        baxter_sphere_fk_store(v[I]..., 0.0f, 0.0f, 0.0f, out, ld);
    }
    __device__ static __forceinline__ void sphere_fk_store(const float* v, float* out, size_t ld)
    {
        fk_(v, out, ld, std::make_index_sequence<D>{});
    }
};

}  // namespace vgpu

VGPU_ROBOT_EXPORTS(vgpu::BaxterR, baxter, true)  // staged: vgpu_baxter_staged.hip
