#!/bin/bash
# Round-3 pass k: deferred CAPT queries in the staged kernels -- point-cloud parity tests, the whole
# -m gpu suite, kbench_capt, the capt bench line, and the headline bench (no point cloud: unchanged path).
TAG=${1:-r03k}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_capt_grid.py tests/test_gpu_capt.py tests/test_pointcloud.py \
    tests/test_gpu_filter_robot.py tests/test_gpu_capt_build.py -v -x --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_capt_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/kbench_capt.py > gpurun_out/${TAG}_kbench_capt.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload capt > gpurun_out/${TAG}_bench_capt.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_validate.log 2>&1 || exit 5
