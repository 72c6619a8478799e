#!/bin/bash
# A/B of Fetch library variants and runtime knobs on the GPU box: the Fetch GPU parity suites per variant,
# then, alternating twice, tools/kbench_robots.py --only fetch (sampler + validate) and the configs[3] edge
# stage at 100k vertices (bench.py --workload prm_edges --no-cpu); optionally the full-size edge stage once.
#   usage: bash tools/ab_fetch.sh TAG spec [spec ...]      spec = variant[:ENV=VAL[,ENV=VAL]]  ("rel" = libvampgpu.so)
#   FULL=1: also the 2.68M-vertex edge stage (one run per spec, after the alternating runs)
# -> gpurun_out/abf_TAG.log (one JSON record per measurement) and a per-(kernel, spec) summary on stdout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
L=$PWD/mr-vamp_amd/vamp_amd
mkdir -p gpurun_out
OUT=gpurun_out/abf_$T.log
: > $OUT
lib() { if [ "$1" = rel ]; then echo $L/libvampgpu.so; else echo $L/libvampgpu_$1.so; fi; }
run() {  # spec, command...
  local spec=$1; shift
  local v=${spec%%:*} envs=""
  [ "$spec" != "$v" ] && envs=${spec#*:}
  env VAMP_AMD_LIB=$(lib $v) $(echo $envs | tr ',' ' ') "$@"
}
for s in "$@"; do
  # one parity log per spec (round 5's single log was overwritten per spec, so an abort did not say whose it was)
  P=gpurun_out/abf_${T}_parity_$(echo $s | tr ':,=' '___').log
  run $s timeout -k 10 300 python -u -m pytest tests/test_gpu_fetch.py tests/test_gpu_roadmap.py -m gpu -x -v --timeout 200 --timeout-method thread > $P 2>&1 || { echo "spec $s failed: $P"; tail -30 $P; exit 1; }
  echo "$s parity: $(tail -n 1 $P)"
done
for r in 1 2; do
  for s in "$@"; do
    run $s timeout -k 10 200 python tools/kbench_robots.py --only fetch --tag $s >> $OUT 2>/dev/null || { echo "kbench $s failed"; exit 1; }
    run $s timeout -k 10 300 python bench.py --workload prm_edges --steps 10 --warmup 2 --no-cpu > gpurun_out/abf_line.json 2>gpurun_out/abf_line.err || { echo "bench $s failed"; tail -5 gpurun_out/abf_line.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abf_line.json')); p=d['phases']; print(json.dumps({'tag': '$s', 'kernel': 'prm_edges_100k', 'ms': d['ms_per_step'], 'knn': p['knn_index_ms'], 'validate': p['validate_ms']}))" >> $OUT
  done
done
if [ "$FULL" = 1 ]; then
  for s in "$@"; do
    run $s timeout -k 10 600 python bench.py --workload prm_edges --vertices 2681709 --steps 3 --warmup 1 --no-cpu > gpurun_out/abf_full.json 2>gpurun_out/abf_full.err || { echo "full $s failed"; tail -5 gpurun_out/abf_full.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abf_full.json')); p=d['phases']; print(json.dumps({'tag': '$s', 'kernel': 'prm_edges_full', 'ms': d['ms_per_step'], 'knn': p['knn_index_ms'], 'validate': p['validate_ms'], 'index_equals_brute': d['roofline']['index_equals_brute']}))" >> $OUT
  done
fi
grep -v amdgpu.ids $OUT | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["kernel"], d["tag"])].append(d["ms"] if "knn" not in d else (round(d["ms"], 2), round(d["knn"], 2), round(d["validate"], 2)))
for k, v in sorted(r.items()): print(k, v)'
