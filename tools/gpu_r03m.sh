#!/bin/bash
# Round-3 pass m: EXT children occupancy A/B (7 default, 6, 8 waves/EU), CAPT tests, capt + validate
# bench lines, CAPT PMC passes of the final build.
TAG=${1:-r03m}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for V in "" _w6 _w8; do
  echo "lib=$V" >> gpurun_out/${TAG}_ab.log
  VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu$V.so timeout -k 10 120 python -u tools/kbench_capt.py >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_capt_grid.py tests/test_gpu_capt.py tests/test_pointcloud.py \
    tests/test_gpu_filter_robot.py tests/test_gpu_staged_chains.py tests/test_gpu_robots.py -q -x --timeout 200 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload capt > gpurun_out/${TAG}_bench_capt.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_validate.log 2>&1 || exit 4
bash tools/gpu_capt_pmc.sh ${TAG} || exit 5
