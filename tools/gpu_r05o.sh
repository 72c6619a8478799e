#!/bin/bash
# round-5 pass o: the Fetch's children hit statistics on the final kernels (VGPU_HITSTATS variant hs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_hs.so timeout -k 10 300 python tools/hitstats.py --fetch > gpurun_out/r05o_hitstats_fetch.json 2> gpurun_out/r05o_hitstats_fetch.err || { tail -20 gpurun_out/r05o_hitstats_fetch.err; exit 1; }
echo ok
