#!/bin/bash
# A/B: base vs hold6 (held/streamed self-pair children, class 2 at 6 waves/EU), then PMC of base
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_ab.sh "mr-vamp_amd/vamp_amd/libvampgpu_base.so mr-vamp_amd/vamp_amd/libvampgpu_hold6.so mr-vamp_amd/vamp_amd/libvampgpu_base.so mr-vamp_amd/vamp_amd/libvampgpu_hold6.so" > gpurun_out/r03c_ab.log 2>&1 || exit 1
bash tools/pmc_r03.sh r03base mr-vamp_amd/vamp_amd/libvampgpu_base.so > gpurun_out/r03c_pmc.log 2>&1
