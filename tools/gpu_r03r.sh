#!/bin/bash
# Round-3 pass r: Fetch children with held self-pair centres (default) vs the chunked form (--no-hold variant),
# configs[3] vertex stage (fetch_prm), two alternating runs each.
TAG=${1:-r03r}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for V in "" _nohold; do
    echo "lib=$V" >> gpurun_out/${TAG}_ab.log
    VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu$V.so timeout -k 10 200 python -u bench.py --workload fetch_prm --no-cpu \
        >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  done
done
