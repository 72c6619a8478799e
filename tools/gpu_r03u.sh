#!/bin/bash
# Round-3 pass u: polled mid-call read-backs (variant libvampgpu_polled.so, VGPU_POLLED_READBACK=1) vs the
# default copy + stream sync, headline bench with parity, alternating; then the -m gpu suite on the variant.
TAG=${1:-r03u}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_polled.so
for rep in 1 2; do
  echo "polled" >> gpurun_out/${TAG}_ab.log
  VAMP_AMD_LIB=$P VGPU_POLLED_READBACK=1 timeout -k 10 200 python -u bench.py >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  echo "default" >> gpurun_out/${TAG}_ab.log
  timeout -k 10 200 python -u bench.py >> gpurun_out/${TAG}_ab.log 2>&1 || exit 2
done
VAMP_AMD_LIB=$P VGPU_POLLED_READBACK=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || exit 3
