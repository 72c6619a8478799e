#!/bin/bash
# round-5 pass h: the -m gpu suite on the release build (sphere pairs unpacked, arm passes back at 5 waves/EU),
# then A/B: Panda cage / set A / table_pick, CAPT, composite: rel vs old (round-5 start);
# Fetch edge stage 100k + 2.68M: rel vs fm / fm2 (mid spheres in the tails' / tails' + heads' bound stage)
# vs kd3 (three kNN tiles in flight) vs the kNN group size (8 and 2 queries per wave)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05h_gputest.log 2>&1 || { tail -30 gpurun_out/r05h_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05h_gputest.log
for v in kd3; do
  VAMP_AMD_LIB=$L/libvampgpu_$v.so timeout -k 10 200 python tools/knn_debug.py 200000 > gpurun_out/r05h_knn_debug_$v.log 2>&1 || { tail -5 gpurun_out/r05h_knn_debug_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r05h_knn_debug_$v.log | head -2
done
: > gpurun_out/r05h_panda.log
for r in 1 2; do
  for v in rel old; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    for w in "validate" "validate --edge-set A" "validate --scene table_pick" "capt" "pair"; do
      VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > gpurun_out/r05h_line.json 2>/dev/null || { echo "$w $v failed"; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r05h_line.json')); print(json.dumps({'tag': '$v', 'kernel': '$w', 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r05h_panda.log
    done
  done
done
FULL=1 bash tools/ab_fetch.sh r05h rel fm fm2 kd3 rel:VAMP_AMD_KNN_GROUP=8 rel:VAMP_AMD_KNN_GROUP=2
