// vcpu_robot.hh -- one robot of the CPU rake: its generated block functions behind a small op
// table (one translation unit per robot, csrc/cpu/vcpu_<robot>.cpp, compiled by g++ with
// -mavx2 -mfma -ffp-contract=off: the generated straight-line code is large).
#pragma once

#include "../../../include/vamp_gpu.h"
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
    // Robot::scale_configuration q * s_m + s_a (contracted to one fma per joint, ref_probe "scale")
    const float* s_m;
    const float* s_a;
    const float* d_m;  // descale_configuration (q - s_a) * d_m
};

// a bound robot (vgpu_robot -> op table + base offsets) and a host environment view (vcpu.cpp)
struct Bound {
    const RobotCpu* R = nullptr;
    float base[6] = {0, 0, 0, 0, 0, 0};
};
struct Env {
    EnvView v;
    bool ext = false, attached = false;
};
int bind(const vgpu_robot* r, Bound& b);
int view(vgpu_env* e, Env& out);
float l2_norm(const float* v, int dim);
bool validate_vector_one(const Bound& b, const Env& env, const float* start, const float* v, float distance,
                         int32_t* n, int32_t* evaluated);
bool validate_one(const Bound& b, const Env& env, const float* start, const float* goal, int32_t* n,
                  int32_t* evaluated);

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
