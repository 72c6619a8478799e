#!/bin/bash
# round-5 pass w: the -m gpu suite on the bounds-checked build of the final kernels (libvampgpu_debug.so,
# make DEBUG=1: every VGPU_DCHECK / VGPU_DCLAMP counted, conftest.py asserts 0 violations after each test)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
VAMP_AMD_LIB=$L/libvampgpu_debug.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05w_gputest_debug.log 2>&1 || { tail -30 gpurun_out/r05w_gputest_debug.log; exit 1; }
echo "debug: $(tail -n 1 gpurun_out/r05w_gputest_debug.log)"
