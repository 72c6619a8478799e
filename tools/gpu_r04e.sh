#!/bin/bash
# round-4 pass e: the GPU suite on the bounds-checked build (make DEBUG=1), then A/B runs:
# Fetch 8-lane bound kernels at 4 (default) vs 5 waves/EU (variant f5) on the edge stage and the sampler;
# one staged round vs the default rounds (VAMP_AMD_ROUNDS) for the Fetch sampler and the CAPT fkcc;
# CAPT cell-grid sizes (VGPU_CAPT_GRID_CELLS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBD=$PWD/mr-vamp_amd/vamp_amd
#VAMP_AMD_LIB=$LIBD/libvampgpu_debug.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04e_gputest_debug.log 2>&1 || { tail -30 gpurun_out/r04e_gputest_debug.log; exit 1; }
#tail -2 gpurun_out/r04e_gputest_debug.log
AB=gpurun_out/r04e_ab.log
: > $AB
run() {  # tag env... -- bench args
  local tag=$1; shift
  env "$@" > /dev/null  # validate the env assignment syntax
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu $BARGS > gpurun_out/r04e_tmp.json 2>/dev/null || { echo "$tag failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04e_tmp.json')); r=d['roofline']; print('$tag', r.get('kernel_ms') or r.get('step_ms_events'), r.get('step_kernel_ms_events'), (d.get('environment_upload_ms') or {}).get('ms'))" >> $AB
}
for rep in 1 2; do
  BARGS="--workload prm_edges"
  run "edges default" VAMP_AMD_LIB=$LIBD/libvampgpu.so
  run "edges f5" VAMP_AMD_LIB=$LIBD/libvampgpu_f5.so
  BARGS="--workload fetch_prm"
  run "fetch default" VAMP_AMD_LIB=$LIBD/libvampgpu.so
  run "fetch f5" VAMP_AMD_LIB=$LIBD/libvampgpu_f5.so
  run "fetch 1round" VAMP_AMD_LIB=$LIBD/libvampgpu.so VAMP_AMD_ROUNDS=0x7fffffffffffffff
  BARGS="--workload capt"
  run "capt default" VAMP_AMD_LIB=$LIBD/libvampgpu.so
  run "capt 1round" VAMP_AMD_LIB=$LIBD/libvampgpu.so VAMP_AMD_ROUNDS=0xffffffff
  run "capt cells1M" VAMP_AMD_LIB=$LIBD/libvampgpu.so VGPU_CAPT_GRID_CELLS=1048576
  run "capt cells512k" VAMP_AMD_LIB=$LIBD/libvampgpu.so VGPU_CAPT_GRID_CELLS=524288
done
cat $AB
