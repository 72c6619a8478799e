#!/bin/bash
# A/B of library variants on the GPU box (make -C mr-vamp_amd VARIANT=name DEFS=...): the GPU parity suites
# on every variant, then tools/kbench.py (set B, set A, fkcc, sphere_fk) and the pair / capt bench steps per
# variant, alternating, twice.   usage: bash tools/ab_variants.sh TAG name [name ...]   ("rel" = libvampgpu.so)
# -> gpurun_out/ab_TAG.log (one JSON record per measurement) and a per-(kernel, variant) summary on stdout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
L=$PWD/mr-vamp_amd/vamp_amd
lib() { if [ "$1" = rel ]; then echo $L/libvampgpu.so; else echo $L/libvampgpu_$1.so; fi; }
mkdir -p gpurun_out
OUT=gpurun_out/ab_$T.log
: > $OUT
for v in "$@"; do
  VAMP_AMD_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_staged_chains.py tests/test_gpu_pair.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_${T}_${v}_parity.log 2>&1 || { tail -30 gpurun_out/ab_${T}_${v}_parity.log; exit 1; }
  echo "$v parity: $(tail -n 1 gpurun_out/ab_${T}_${v}_parity.log)"
done
for r in 1 2; do
  for v in "$@"; do
    VAMP_AMD_LIB=$(lib $v) timeout -k 10 200 python tools/kbench.py --tag $v >> $OUT 2>/dev/null || { echo "kbench $v failed"; exit 1; }
    for w in pair capt; do
      VAMP_AMD_LIB=$(lib $v) timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_line.json 2>/dev/null || { echo "bench $w $v failed"; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab_line.json')); print(json.dumps({'tag': '$v', 'kernel': '$w', 'ms': d['ms_per_step']}))" >> $OUT
    done
  done
done
grep -v amdgpu.ids $OUT | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["kernel"], d["tag"])].append(d["ms"])
for k, v in sorted(r.items()): print(k, ["%.3f" % x for x in v])'
