#!/bin/bash
# round-5 pass c: the fused lead (Panda heads) and the block-cooperative kNN / Fetch children occupancy A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
VAMP_AMD_FUSE_LEAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05c_fuse_parity.log 2>&1 || { tail -30 gpurun_out/r05c_fuse_parity.log; exit 1; }
echo "fused-lead parity: $(tail -n 1 gpurun_out/r05c_fuse_parity.log)"
: > gpurun_out/r05c_panda.log
for r in 1 2; do
  for f in 0 1; do
    VAMP_AMD_FUSE_LEAD=$f timeout -k 10 200 python tools/kbench.py --tag fuse$f >> gpurun_out/r05c_panda.log 2>/dev/null || { echo "kbench fuse$f failed"; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r05c_panda.log | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["kernel"], d["tag"])].append(round(d["ms"], 3))
for k, v in sorted(r.items()): print(k, v)'
FULL=1 bash tools/ab_fetch.sh r05c rel rel:VAMP_AMD_KNN_COOP=0 rel:VAMP_AMD_KNN_COOP=8 fc7
