#!/bin/bash
# tools/variant_staged.sh NAME "DEFS" -- A/B build of the Panda staged TU only:
# mr-vamp_amd/vamp_amd/libvampgpu_NAME.so = build/*.o with vgpu_staged.o rebuilt under DEFS
# (run `make` in mr-vamp_amd first).  Select it with VAMP_AMD_LIB=... (tools/kbench.py).
set -euo pipefail
cd "$(dirname "$0")/../mr-vamp_amd"
name=$1; defs=$2
mkdir -p build_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize $defs \
    -c csrc/vgpu_staged.hip -o build_$name/vgpu_staged.o
objs=$(ls build/*.o | grep -v '/vgpu_staged.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o vamp_amd/libvampgpu_$name.so $objs build_$name/vgpu_staged.o -lpthread
