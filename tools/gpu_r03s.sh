#!/bin/bash
# Round-3 pass s: Fetch with chunked self-pair children -- Fetch/roadmap GPU tests, fetch_prm and prm_edges lines.
TAG=${1:-r03s}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fetch.py tests/test_gpu_roadmap.py tests/test_gpu_attach.py \
    tests/test_gpu_sampling.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload fetch_prm > gpurun_out/${TAG}_bench_fetch_prm.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload prm_edges > gpurun_out/${TAG}_bench_prm_edges.log 2>&1 || exit 3
