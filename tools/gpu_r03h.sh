#!/bin/bash
# Round-3 pass h: the group kNN query kernel -- roadmap GPU tests, knn_scale A/B over VAMP_AMD_KNN_GROUP
# (0 = the 64-query waves) with index == brute checks, then 2.7M vertices index vs brute.
TAG=${1:-r03h}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_roadmap.py -v -x --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_knn_tests.log 2>&1 || exit 11
for G in 4 8 2 0; do
  echo "group=$G" >> gpurun_out/${TAG}_knn.log
  VAMP_AMD_KNN_GROUP=$G timeout -k 10 240 python -u tools/knn_scale.py 100000 400000 >> gpurun_out/${TAG}_knn.log 2>&1 || exit 12
done
echo "group=4 2.7M" >> gpurun_out/${TAG}_knn.log
KNN_BRUTE_MAX=3000000 timeout -k 10 300 python -u tools/knn_scale.py 2700000 >> gpurun_out/${TAG}_knn.log 2>&1 || exit 13
