#!/bin/bash
# End-of-round measurements on one GPU box: every bench.py workload, the headline's rocprofv3
# kernel stats + PMC traffic (tools/profile_round.sh), and the kernel stats of the PRM edge stage.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${1:-r01}
bash tools/bench_all.sh $R || exit 1
bash tools/profile_round.sh $R || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R}_prm -o prm --output-format csv -- python3 bench.py --workload prm_edges --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_${R}_prm.log 2>&1 || { echo "prm kernel-trace failed"; tail -20 gpurun_out/prof_${R}_prm.log; exit 1; }
echo measured
