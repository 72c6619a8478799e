// vgpu_attach_ur5.hip -- UR5::fkcc_attach = ur5::interleaved_sphere_fk_attachment
// (robots/ur5.hh:43), generated from model/ur5_attach.json; kernels in vgpu_attach.hh.
#include "vgpu_attach.hh"
#include "gen/ur5_attach_fk.inc"

namespace vgpu {
struct Ur5AttR {
    static constexpr int D = 6;
    static constexpr int kRes = 32;  // robots/ur5.hh:12
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool cc(const float* v, const EnvView& env)
    {
        return ur5_attach_fkcc<Grp, EXT>(v[0], v[1], v[2], v[3], v[4], v[5], env, 0.0f, 0.0f, 0.0f);
    }
};
}  // namespace vgpu

extern "C" {
hipError_t vgpu_launch_ur5_fkcc_attach(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st)
{
    return vgpu::AttHost<vgpu::Ur5AttR>::fkcc(q, n, env, valid, st);
}
hipError_t vgpu_launch_ur5_validate_head_att(const float* starts, const float* goals, size_t n_edges,
                                               const EnvView* env, uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                               hipStream_t st)
{
    return vgpu::AttHost<vgpu::Ur5AttR>::head(starts, goals, n_edges, env, ok, n_blocks, cnt, st);
}
}
