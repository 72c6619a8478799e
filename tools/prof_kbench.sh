#!/bin/bash
# kernel-trace stats of tools/kbench.py (development profiling).  Usage: tools/prof_kbench.sh <tag> [edges]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1
E=${2:-1048576}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_$T -o kb --output-format csv -- python3 tools/kbench.py --edges $E --reps 3 --tag $T > gpurun_out/kprof_$T.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/kprof_$T.log; exit 1; }
f=$(find gpurun_out/kprof_$T -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us avg', round(float(r['TotalDurationNs'])/1e6,2),'ms tot')
"
