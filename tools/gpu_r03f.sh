#!/bin/bash
# Round-3 pass f: the CAPT cell grid -- parity tests, A/B of grid sizes (kbench_capt), configs[2] bench line.
TAG=${1:-r03f}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_capt_grid.py tests/test_gpu_capt.py tests/test_gpu_capt_build.py \
    tests/test_pointcloud.py tests/test_gpu_filter_robot.py -v -x --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
for C in default 0 131072 524288 2097152; do
  if [ $C = default ]; then unset VGPU_CAPT_GRID_CELLS; else export VGPU_CAPT_GRID_CELLS=$C; fi
  echo "cells=$C" >> gpurun_out/${TAG}_ab.log
  timeout -k 10 120 python -u tools/kbench_capt.py >> gpurun_out/${TAG}_ab.log 2>&1 || exit 2
done
unset VGPU_CAPT_GRID_CELLS
timeout -k 10 300 python -u bench.py --workload capt > gpurun_out/${TAG}_bench_capt.log 2>&1 || exit 3
