#!/bin/bash
# tools/kres.sh <file.hip> [extra flags] -- VGPR / scratch / occupancy of the vgpu:: kernels
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function \
  -Wno-unused-variable -Rpass-analysis=kernel-resource-usage "$@" -c "$f" -o /tmp/kres.o 2>&1 |
  grep -v rocprim | grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" |
  sed -E 's/.*remark: *//; s/ \[-Rpass-analysis=kernel-resource-usage\]//' | paste - - - - | grep vgpu
