// vgpu_ops.hh -- the per-robot launch table the host runtime (vgpu_api.cpp) dispatches through
// for the robots built from vgpu_robot.hh (one translation unit each).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

struct EnvView;

struct RobotOps {
    int dim, resolution, n_spheres;
    bool staged;  // the robot's TU also exports the staged pipeline (<= 64 checks)
    hipError_t (*sphere_fk)(const float* q, size_t n, float* out, size_t ld, hipStream_t st);
    hipError_t (*fkcc)(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st);
    hipError_t (*sample)(uint64_t first, size_t n, float* q, hipStream_t st);
    hipError_t (*sample_fkcc)(uint64_t first, size_t n, const EnvView* env, float* q, uint8_t* valid, hipStream_t st);
    hipError_t (*validate_head)(const float* starts, const float* goals, size_t n_edges, const EnvView* env,
                                uint8_t* ok, int32_t* n_blocks, uint32_t* cnt, hipStream_t st);
    hipError_t (*validate_tail)(const float* starts, const float* goals, size_t n_items, const EnvView* env,
                                uint8_t* ok, const uint32_t* off, const uint32_t* item_edge, hipStream_t st);
    hipError_t (*tail_counts)(const float* starts, const float* goals, size_t n_edges, const uint8_t* ok,
                              int32_t* n_blocks, uint32_t* cnt, hipStream_t st);
};
