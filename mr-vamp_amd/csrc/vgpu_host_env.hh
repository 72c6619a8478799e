// vgpu_host_env.hh -- internal (not part of the C ABI): the environment's host-memory view for
// the CPU rake (csrc/cpu/vcpu.cpp).  Same blob layout and offsets as the device copy
// (vgpu_device.hh EnvView); built by vgpu_api.cpp:build_blob.
#pragma once

#include "../../include/vamp_gpu.h"

namespace vgpu {

struct HostEnvView {
    const float* obs[5];  // spheres, capsules, z-capsules, cuboids, z-cuboids (md-sorted + sentinels)
    int n[5];
    const float* hf;  // heightfield headers
    const float* pc;  // point-cloud (CAPT) headers
    const float* base;
    int n_hf, n_pc;
    const float* att;  // attachment frame + spheres
    int n_att;
    bool attached;
};

}  // namespace vgpu

// (re)builds the host blob when the environment changed; the view stays valid until the next
// change of the environment.  Thread-safe against other views / uploads of the same environment.
int vgpu_env_host_view(vgpu_env* env, vgpu::HostEnvView* view);
