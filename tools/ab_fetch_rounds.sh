#!/bin/bash
# A/B of the Fetch edge stage's check rounds: VAMP_AMD_ONE_ROUND (source-kind bits; the Fetch default is the
# sampler only, 0x2) on configs[3]'s edge stage at 100k vertices, alternating, twice -> gpurun_out/ab_fetch_rounds.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab_fetch_rounds.log
for r in 1 2; do
  for k in default 0x6 0xa 0xe; do
    if [ $k = default ]; then unset VAMP_AMD_ONE_ROUND; else export VAMP_AMD_ONE_ROUND=$k; fi
    timeout -k 10 300 python bench.py --workload prm_edges --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_line.json 2>/dev/null || { echo "prm_edges $k failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_line.json')); print(json.dumps({'one_round': '$k', 'ms': d['ms_per_step'], 'validate_ms': d['phases']['validate_ms']}))" | tee -a gpurun_out/ab_fetch_rounds.log
  done
done
