// vcpu_ur5.cpp -- vamp::robots::UR5 (robots/ur5.hh) on the CPU rake (csrc/gen/cpu/ur5_*.inc).
#include "vcpu_robot.hh"

namespace vcpu {
namespace {
#include "../gen/cpu/ur5_fk.inc"
#include "../gen/cpu/ur5_attach_fk.inc"

bool fkcc(const V* q, const EnvView& env, const float*, bool ext)
{
    return ext ? ur5_fkcc<GrpBlock, true>(VCPU_Q6(q), env, 0.0f, 0.0f, 0.0f)
               : ur5_fkcc<GrpBlock, false>(VCPU_Q6(q), env, 0.0f, 0.0f, 0.0f);
}
bool fkcc_attach(const V* q, const EnvView& env, const float*, bool ext)
{
    return ext ? ur5_attach_fkcc<GrpBlock, true>(VCPU_Q6(q), env, 0.0f, 0.0f, 0.0f)
               : ur5_attach_fkcc<GrpBlock, false>(VCPU_Q6(q), env, 0.0f, 0.0f, 0.0f);
}
void sphere_fk(const V* q, const float*, V* out) { ur5_sphere_fk_store(VCPU_Q6(q), 0.0f, 0.0f, 0.0f, out, 1); }
}  // namespace

const RobotCpu* robot_ur5()
{
    static const RobotCpu r{6, 32, 36, fkcc, fkcc_attach, sphere_fk, ur5_s_m, ur5_s_a, ur5_d_m};
    return &r;
}
}  // namespace vcpu
