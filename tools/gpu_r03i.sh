#!/bin/bash
# Round-3 pass i: kNN group kernel (pass h), then the CAPT profile (kernel trace + PMC) and capt bench line
# with the default cell grid.
TAG=${1:-r03i}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload capt > gpurun_out/${TAG}_bench_capt.log 2>&1 || exit 3
bash tools/gpu_capt_pmc.sh ${TAG} || exit 4
bash tools/gpu_r03h.sh ${TAG} || exit $?
