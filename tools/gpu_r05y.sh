#!/bin/bash
# round-5 pass y: the edge stage's host tables kept between calls: the roadmap / multi-rank GPU tests, then the
# edge-stage lines (tools/gpu_r05x.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_roadmap.py tests/test_multi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05y_gputest.log 2>&1 || { tail -30 gpurun_out/r05y_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05y_gputest.log
bash tools/gpu_r05x.sh
