#!/bin/bash
# Round-3 pass o: device roadmap assembly -- roadmap GPU tests, the configs[3] edge stage at 100k and at the
# full 2.68M vertices (device assembly in the step, host assembly compared outside it).
TAG=${1:-r03o}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_roadmap.py tests/test_c_abi.py -v -x --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload prm_edges > gpurun_out/${TAG}_bench_prm_edges.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --workload prm_edges --vertices 2681709 --steps 2 --warmup 1 \
    > gpurun_out/${TAG}_bench_prm_edges_full.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_validate.log 2>&1 || exit 4
