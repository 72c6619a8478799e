// vcpu_pair.cpp -- the two-Panda composite of BASELINE configs[4] on the CPU rake: validity =
// fkcc_A && fkcc_B && no A-B sphere overlap (link-bounding pairs first), composed from the
// reference primitives exactly as oracle/vamp_oracle.c vo_pair_fkcc_block and vgpu_pair.hip.
#include "vcpu_robot.hh"

namespace vcpu {
namespace {
#include "../gen/cpu/panda_fk.inc"
#include "../gen/cpu/panda_pair.inc"

template <bool EXT>
bool fkcc_t(const V* q, const EnvView& env, const float* b)
{
    if (!panda_fkcc<GrpBlock, EXT>(VCPU_Q7(q), env, b[0], b[1], b[2])) return false;
    if (!panda_fkcc<GrpBlock, EXT>(VCPU_Q7B(q), env, b[3], b[4], b[5])) return false;
    return !panda_pair_inter<GrpBlock>(VCPU_Q7(q), VCPU_Q7B(q), b[0], b[1], b[2], b[3], b[4], b[5]);
}
bool fkcc(const V* q, const EnvView& env, const float* b, bool ext)
{
    return ext ? fkcc_t<true>(q, env, b) : fkcc_t<false>(q, env, b);
}
void sphere_fk(const V* q, const float* b, V* out)
{
    panda_sphere_fk_store(VCPU_Q7(q), b[0], b[1], b[2], out, 1);  // arm A spheres, then arm B's
    V outb[3 * 59];
    panda_sphere_fk_store(VCPU_Q7B(q), b[3], b[4], b[5], outb, 1);
    V tmp[3 * 59];
    for (int i = 0; i < 3 * 59; ++i) tmp[i] = out[i];
    for (int c = 0; c < 3; ++c)
        for (int s = 0; s < 59; ++s) {
            out[c * 118 + s] = tmp[c * 59 + s];
            out[c * 118 + 59 + s] = outb[c * 59 + s];
        }
}

// both arms' scaling, concatenated
constexpr float pair_s_m[14] = {panda_s_m[0], panda_s_m[1], panda_s_m[2], panda_s_m[3], panda_s_m[4], panda_s_m[5],
                                panda_s_m[6], panda_s_m[0], panda_s_m[1], panda_s_m[2], panda_s_m[3], panda_s_m[4],
                                panda_s_m[5], panda_s_m[6]};
constexpr float pair_s_a[14] = {panda_s_a[0], panda_s_a[1], panda_s_a[2], panda_s_a[3], panda_s_a[4], panda_s_a[5],
                                panda_s_a[6], panda_s_a[0], panda_s_a[1], panda_s_a[2], panda_s_a[3], panda_s_a[4],
                                panda_s_a[5], panda_s_a[6]};
}  // namespace

const RobotCpu* robot_panda_pair()
{
    static const RobotCpu r{14, 32, 118, fkcc, nullptr, sphere_fk, pair_s_m, pair_s_a};
    return &r;
}
}  // namespace vcpu
