#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of the contract bench, plus separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of the head kernel.  Writes gpurun_out/prof_*;
# tools/profile_collect.py turns them into profiles/<round>_*.{csv,json}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${1:-r01}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$R -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_$R.log 2>&1 || { echo "kernel-trace pass failed"; tail -20 gpurun_out/prof_$R.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "SrcHead|SrcTail|scatter_items|tail_counts|panda_validate|panda_sphere_fk" -d gpurun_out/pmc_${R}_$C -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/pmc_${R}_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 gpurun_out/pmc_${R}_$C.log; exit 1; }
done
echo done
