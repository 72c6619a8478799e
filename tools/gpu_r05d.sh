#!/bin/bash
# round-5 pass d: kNN coop mismatch debug; Panda (scan prefetch, bound occupancy) and Fetch (children occupancy,
# scan prefetch) variant A/B with the group kNN kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/knn_debug.py 200000 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05d_knn_debug.log || exit 1
L=$PWD/mr-vamp_amd/vamp_amd
for v in pf1; do
  VAMP_AMD_LIB=$L/libvampgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05d_${v}_parity.log 2>&1 || { tail -30 gpurun_out/r05d_${v}_parity.log; exit 1; }
  echo "$v parity: $(tail -n 1 gpurun_out/r05d_${v}_parity.log)"
done
: > gpurun_out/r05d_panda.log
for r in 1 2; do
  for v in rel pf1; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    VAMP_AMD_LIB=$lib timeout -k 10 200 python tools/kbench.py --tag $v >> gpurun_out/r05d_panda.log 2>/dev/null || { echo "kbench $v failed"; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r05d_panda.log | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["kernel"], d["tag"])].append(round(d["ms"], 3))
for k, v in sorted(r.items()): print(k, v)'
FULL=1 bash tools/ab_fetch.sh r05d rel:VAMP_AMD_KNN_COOP=0 fc7:VAMP_AMD_KNN_COOP=0 fc6:VAMP_AMD_KNN_COOP=0 pf2:VAMP_AMD_KNN_COOP=0
