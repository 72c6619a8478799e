#!/bin/bash
# Round-3 pass p (final build): the whole -m gpu suite, then the round's rocprofv3 kernel-trace stats + FETCH/WRITE
# passes of the contract bench and the SQ/TCC PMC groups of the headline call.
TAG=${1:-r03}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_final_gputest.log 2>&1 || exit 1
bash tools/profile_round.sh $TAG || exit 2
bash tools/pmc_r03.sh $TAG || exit 3
