#!/bin/bash
# round-4 pass c: GPU suite on the build with per-source bound occupancy (Fetch / inter-arm head and tail)
# and the XCD-ordered kNN index, then every bench workload, then fresh profiles of the changed ones
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c_gputest.log 2>&1 || { tail -30 gpurun_out/r04c_gputest.log; exit 1; }
tail -2 gpurun_out/r04c_gputest.log
for w in validate pair fetch_prm prm_edges capt; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/bench_r04c_$w.json 2> gpurun_out/bench_r04c_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/bench_r04c_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_r04c_$w.json')); r=d['roofline']; print('$w', d['value'], d['unit'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'frac', r.get('frac'), 'exec', (r.get('executed') or {}).get('valu_issue_frac'))"
done
bash tools/prof_r04.sh pair fetch_prm prm_edges
