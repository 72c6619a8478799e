// vcpu_baxter.cpp -- vamp::robots::Baxter (robots/baxter.hh, 14 dof, resolution 64) on the CPU
// rake; its fkcc_attach is its plain interleaved_sphere_fk (baxter.hh:44).
#include "vcpu_robot.hh"

namespace vcpu {
namespace {
#include "../gen/cpu/baxter_fk.inc"

bool fkcc(const V* q, const EnvView& env, const float*, bool ext)
{
    return ext ? baxter_fkcc<GrpBlock, true>(VCPU_Q14(q), env, 0.0f, 0.0f, 0.0f)
               : baxter_fkcc<GrpBlock, false>(VCPU_Q14(q), env, 0.0f, 0.0f, 0.0f);
}
void sphere_fk(const V* q, const float*, V* out) { baxter_sphere_fk_store(VCPU_Q14(q), 0.0f, 0.0f, 0.0f, out, 1); }
}  // namespace

const RobotCpu* robot_baxter()
{
    static const RobotCpu r{14, 64, 75, fkcc, fkcc, sphere_fk, baxter_s_m, baxter_s_a, baxter_d_m};
    return &r;
}
}  // namespace vcpu
