#!/bin/bash
# Round-3 pass j: group kNN kernel v2 (uniform values in SGPRs, pipelined tile loads): tests, A/B of the
# group size, 2.7M index vs brute; then the configs[3] edge-stage bench at the max_samples default
# (100k) and at the full 4M-draw vertex count.
TAG=${1:-r03j}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_roadmap.py -v -x --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_knn_tests.log 2>&1 || exit 11
for G in 4 8 2; do
  echo "group=$G" >> gpurun_out/${TAG}_knn.log
  VAMP_AMD_KNN_GROUP=$G timeout -k 10 240 python -u tools/knn_scale.py 100000 400000 >> gpurun_out/${TAG}_knn.log 2>&1 || exit 12
done
echo "group=default 2.7M" >> gpurun_out/${TAG}_knn.log
KNN_BRUTE_MAX=3000000 timeout -k 10 300 python -u tools/knn_scale.py 2700000 >> gpurun_out/${TAG}_knn.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py --workload prm_edges > gpurun_out/${TAG}_bench_prm_edges.log 2>&1 || exit 14
timeout -k 10 600 python -u bench.py --workload prm_edges --vertices 2681709 --steps 2 --warmup 1 \
    > gpurun_out/${TAG}_bench_prm_edges_full.log 2>&1 || exit 15
