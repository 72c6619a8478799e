#!/bin/bash
# Every bench.py workload once (the contract headline and BASELINE configs[2..4]), one GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${1:-r01}
for w in validate capt fetch_prm prm_edges pair rrtc; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/bench_${R}_$w.json 2> gpurun_out/bench_${R}_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/bench_${R}_$w.err; exit 1; }
  cat gpurun_out/bench_${R}_$w.json
done
