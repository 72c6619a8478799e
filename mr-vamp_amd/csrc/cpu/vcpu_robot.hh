// vcpu_robot.hh -- one robot of the CPU rake: its generated block functions behind a small op
// table (one translation unit per robot, csrc/cpu/vcpu_<robot>.cpp, compiled by g++ with
// -mavx2 -mfma -ffp-contract=off: the generated straight-line code is large).
#pragma once

#include "vcpu_simd.hh"

namespace vcpu {

constexpr int kMaxDim = 16;

struct RobotCpu {
    int dim, resolution, n_spheres;
    // Robot::fkcc<8> of one rake block q[dim] (lane l = interpolant l): true = all lanes valid.
    // base: the Panda base offset(s) in metres (composite: arm A then arm B); ext: heightfields
    // or point clouds present.
    bool (*fkcc)(const V* q, const EnvView& env, const float* base, bool ext);
    // Robot::fkcc_attach<8> (the environment's attachment posed at the end effector); nullptr
    // where the robot has none
    bool (*fkcc_attach)(const V* q, const EnvView& env, const float* base, bool ext);
    // Robot::sphere_fk<8>: out[3][n_spheres] (x rows, then y, then z), world frame
    void (*sphere_fk)(const V* q, const float* base, V* out);
};

const RobotCpu* robot_panda();
const RobotCpu* robot_fetch();
const RobotCpu* robot_ur5();
const RobotCpu* robot_baxter();
const RobotCpu* robot_panda_pair();

}  // namespace vcpu

// argument lists of the generated functions
#define VCPU_Q6(q) q[0], q[1], q[2], q[3], q[4], q[5]
#define VCPU_Q7(q) q[0], q[1], q[2], q[3], q[4], q[5], q[6]
#define VCPU_Q8(q) q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]
#define VCPU_Q14(q) q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8], q[9], q[10], q[11], q[12], q[13]
#define VCPU_Q7B(q) q[7], q[8], q[9], q[10], q[11], q[12], q[13]
