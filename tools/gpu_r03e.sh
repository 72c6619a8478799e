#!/bin/bash
# Round-3 pass e: kernel-trace stats + FETCH/WRITE passes of the contract bench (profile_round.sh),
# then the SQ/TCC PMC groups of the headline call (pmc_r03.sh).
TAG=${1:-r03}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/profile_round.sh $TAG || exit 1
bash tools/pmc_r03.sh $TAG || exit 2
