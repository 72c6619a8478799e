#!/bin/bash
# A/B of the CAPT cell-grid size (VGPU_CAPT_GRID_CELLS; unset = capt_grid_plan's default, 128 cells per leaf):
# the capt bench step and its environment upload per size, alternating, twice -> gpurun_out/ab_grid.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab_grid.log
for r in 1 2; do
  for c in default 262144 524288 1048576 4194304; do
    if [ $c = default ]; then unset VGPU_CAPT_GRID_CELLS; else export VGPU_CAPT_GRID_CELLS=$c; fi
    timeout -k 10 300 python bench.py --workload capt --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_line.json 2>/dev/null || { echo "capt $c failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_line.json')); print(json.dumps({'cells': '$c', 'ms': d['ms_per_step'], 'upload_ms': d['environment_upload_ms']['ms'], 'raw_q_per_s': d['raw_queries']['queries_per_s']}))" | tee -a gpurun_out/ab_grid.log
  done
done
