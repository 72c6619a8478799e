#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of one bench workload's timed steps, plus the staged passes'
# bounding statistics (VAMP_AMD_STAGED_STATS=1) of one bench step.   usage: bash tools/trace_step.sh TAG W [W ...]
# -> gpurun_out/TAG_<W>_kernel_stats.csv, gpurun_out/TAG_<W>_stats.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/trace
for W in "$@"; do
  D=gpurun_out/trace/${T}_$W
  rm -rf $D && mkdir -p $D
  timeout -k 10 300 python3 tools/pmc_drive.py prep --workload $W > $D/prep.log 2>&1 || { echo "prep $W failed"; tail -20 $D/prep.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- \
      python3 tools/pmc_drive.py run --workload $W --calls 4 > $D/trace.log 2>&1 || { echo "trace $W failed"; tail -20 $D/trace.log; exit 1; }
  cp $(find $D/trace -name "*kernel_stats.csv" | head -1) gpurun_out/${T}_${W}_kernel_stats.csv
  VAMP_AMD_STAGED_STATS=1 timeout -k 10 300 python3 tools/pmc_drive.py run --workload $W --calls 1 > gpurun_out/${T}_${W}_stats.log 2>&1 || { echo "stats $W failed"; exit 1; }
  rm -rf $D
done
echo trace done
