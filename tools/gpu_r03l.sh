#!/bin/bash
# Round-3 pass l: CAPT grid-size A/B with deferred queries, and the kernel trace of kbench_capt.
TAG=${1:-r03l}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in default 1048576 4194304 8388608; do
  if [ $C = default ]; then unset VGPU_CAPT_GRID_CELLS; else export VGPU_CAPT_GRID_CELLS=$C; fi
  echo "cells=$C" >> gpurun_out/${TAG}_ab.log
  timeout -k 10 120 python -u tools/kbench_capt.py >> gpurun_out/${TAG}_ab.log 2>&1 || exit 2
done
unset VGPU_CAPT_GRID_CELLS
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o capt --output-format csv \
    -- python3 tools/kbench_capt.py > gpurun_out/${TAG}_trace.log 2>&1 || exit 3
