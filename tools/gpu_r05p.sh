#!/bin/bash
# round-5 pass p: the -m gpu suite on the bounds-checked build of the final kernels (libvampgpu_debug.so:
# VGPU_DCHECK counters must stay 0), then A/B of finer Fetch mid-sphere clusters (fm4) on the edge stage
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
VAMP_AMD_LIB=$L/libvampgpu_debug.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05p_gputest_debug.log 2>&1 || { tail -30 gpurun_out/r05p_gputest_debug.log; exit 1; }
echo "debug: $(tail -n 1 gpurun_out/r05p_gputest_debug.log)"
FULL=1 bash tools/ab_fetch.sh r05p rel fm4
