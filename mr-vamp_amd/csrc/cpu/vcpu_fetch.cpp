// vcpu_fetch.cpp -- vamp::robots::Fetch (robots/fetch.hh:8-48) on the CPU rake (generated from
// model/fetch.json: csrc/gen/cpu/fetch_*.inc).
#include "vcpu_robot.hh"

namespace vcpu {
namespace {
#include "../gen/cpu/fetch_fk.inc"
#include "../gen/cpu/fetch_attach_fk.inc"

bool fkcc(const V* q, const EnvView& env, const float*, bool ext)
{
    return ext ? fetch_fkcc<GrpBlock, true>(VCPU_Q8(q), env, 0.0f, 0.0f, 0.0f)
               : fetch_fkcc<GrpBlock, false>(VCPU_Q8(q), env, 0.0f, 0.0f, 0.0f);
}
bool fkcc_attach(const V* q, const EnvView& env, const float*, bool ext)
{
    return ext ? fetch_attach_fkcc<GrpBlock, true>(VCPU_Q8(q), env, 0.0f, 0.0f, 0.0f)
               : fetch_attach_fkcc<GrpBlock, false>(VCPU_Q8(q), env, 0.0f, 0.0f, 0.0f);
}
void sphere_fk(const V* q, const float*, V* out) { fetch_sphere_fk_store(VCPU_Q8(q), 0.0f, 0.0f, 0.0f, out, 1); }
}  // namespace

const RobotCpu* robot_fetch()
{
    static const RobotCpu r{8, 32, 111, fkcc, fkcc_attach, sphere_fk, fetch_s_m, fetch_s_a, fetch_d_m};  // fetch.hh:12-14
    return &r;
}
}  // namespace vcpu
