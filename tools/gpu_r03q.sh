#!/bin/bash
# Round-3 pass q: obstacle records staged in LDS per workgroup (VGPU_ENV_LDS variant) vs the scalar-cache scan
# (default), headline workload: kbench both ways twice, then the contract bench (with its parity) on the variant.
TAG=${1:-r03q}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for V in "" _envlds; do
    VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu$V.so timeout -k 10 200 python -u tools/kbench.py --edges 1048576 --reps 5 \
        >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  done
done
VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_envlds.so timeout -k 10 300 python -u bench.py \
    > gpurun_out/${TAG}_bench_envlds.log 2>&1 || exit 2
