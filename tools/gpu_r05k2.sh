#!/bin/bash
# round-5 pass k2 (final build): the step profiles of the configs[3] edge stage at 100k and 2.68M vertices
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/prof_step.sh prm_edges prm_edges_full || exit 1
