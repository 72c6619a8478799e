#!/bin/bash
# round-5 pass g: the -m gpu suite on the release build (packed sphere pairs, spill-free EXT / Fetch budgets,
# coded kNN candidates), the coded kNN's lists vs brute force at 200k, then A/B:
#   Panda cage / set A / table_pick, CAPT, composite: rel vs old (round-5 start) vs np (sphere pairs unpacked)
#   Fetch edge stage 100k + 2.68M: rel vs rel with VAMP_AMD_KNN_QCODE=0 vs old
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05g_gputest.log 2>&1 || { tail -30 gpurun_out/r05g_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05g_gputest.log
timeout -k 10 200 python tools/knn_debug.py 200000 > gpurun_out/r05g_knn_debug.log 2>&1 || { tail -5 gpurun_out/r05g_knn_debug.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05g_knn_debug.log | head -3
: > gpurun_out/r05g_panda.log
for r in 1 2; do
  for v in rel old np; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    for w in "validate" "validate --edge-set A" "validate --scene table_pick" "capt" "pair"; do
      [ $v = np ] && [ "$w" = capt -o "$w" = pair ] && continue
      VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > gpurun_out/r05g_line.json 2>/dev/null || { echo "$w $v failed"; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r05g_line.json')); print(json.dumps({'tag': '$v', 'kernel': '$w', 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r05g_panda.log
    done
  done
done
FULL=1 bash tools/ab_fetch.sh r05g rel rel:VAMP_AMD_KNN_QCODE=0 old
