#!/bin/bash
# round-4 pass f: one staged round (VAMP_AMD_ROUNDS = every check) vs the per-batch default rounds on the
# validate workloads (set B headline, set A), the Fetch edge stage and the composite; alternating, twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB=gpurun_out/r04f_ab.log
: > $AB
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-fk-leg $BARGS > gpurun_out/r04f_tmp.json 2>/dev/null || { echo "$tag failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04f_tmp.json')); r=d['roofline']; print('$tag', r.get('kernel_ms'), r.get('step_kernel_ms_events'), d['ms_per_step'])" >> $AB
}
ALL=0xffffffffffffffff
for rep in 1 2; do
  BARGS="--workload validate"; run "setB default" A=1; run "setB 1round" VAMP_AMD_ROUNDS=$ALL
  BARGS="--workload validate --edge-set A"; run "setA default" A=1; run "setA 1round" VAMP_AMD_ROUNDS=$ALL
  BARGS="--workload prm_edges"; run "edges default" A=1; run "edges 1round" VAMP_AMD_ROUNDS=$ALL
  BARGS="--workload pair"; run "pair default" A=1; run "pair 1round" VAMP_AMD_ROUNDS=$ALL
done
cat $AB
