// vcpu_panda.cpp -- Panda (PandaBase<X100, Y100, Z100>, robots/panda_base.hh:15-75) on the CPU rake:
// the generated interleaved_sphere_fk / interleaved_sphere_fk_attachment / sphere_fk restatement
// (csrc/gen/cpu/panda_*.inc, same text as the HIP kernels' csrc/gen/panda_*.inc).
#include "vcpu_robot.hh"

namespace vcpu {
namespace {
#include "../gen/cpu/panda_fk.inc"
#include "../gen/cpu/panda_attach_fk.inc"

bool fkcc(const V* q, const EnvView& env, const float* b, bool ext)
{
    return ext ? panda_fkcc<GrpBlock, true>(VCPU_Q7(q), env, b[0], b[1], b[2])
               : panda_fkcc<GrpBlock, false>(VCPU_Q7(q), env, b[0], b[1], b[2]);
}
bool fkcc_attach(const V* q, const EnvView& env, const float* b, bool ext)
{
    return ext ? panda_attach_fkcc<GrpBlock, true>(VCPU_Q7(q), env, b[0], b[1], b[2])
               : panda_attach_fkcc<GrpBlock, false>(VCPU_Q7(q), env, b[0], b[1], b[2]);
}
void sphere_fk(const V* q, const float* b, V* out) { panda_sphere_fk_store(VCPU_Q7(q), b[0], b[1], b[2], out, 1); }
}  // namespace

const RobotCpu* robot_panda()
{
    static const RobotCpu r{7, 32, 59, fkcc, fkcc_attach, sphere_fk, panda_s_m, panda_s_a, panda_d_m};  // panda_base.hh:19-23
    return &r;
}
}  // namespace vcpu
