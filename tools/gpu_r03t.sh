#!/bin/bash
# Round-3 pass t: polled read-backs (VGPU_POLLED_READBACK=1) instead of copy + stream sync -- headline bench both
# ways, alternating, then the whole -m gpu suite with polled read-backs.
TAG=${1:-r03t}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  echo "polled" >> gpurun_out/${TAG}_ab.log
  VGPU_POLLED_READBACK=1 timeout -k 10 200 python -u bench.py --no-cpu >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  echo "copy+sync" >> gpurun_out/${TAG}_ab.log
  timeout -k 10 200 python -u bench.py --no-cpu >> gpurun_out/${TAG}_ab.log 2>&1 || exit 2
done
VGPU_POLLED_READBACK=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || exit 3
