#!/bin/bash
# round-4 pass g: GPU suite on the current build (CAPT grids as device-only holes, per-robot rounds), then the
# host-rsqrt table in LDS (variant lut) vs the global table, tools/kbench.py, alternating twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_gputest.log 2>&1 || { tail -30 gpurun_out/r04g_gputest.log; exit 1; }
tail -2 gpurun_out/r04g_gputest.log
OUT=gpurun_out/r04g_lut_ab.log
: > $OUT
L=$PWD/mr-vamp_amd/vamp_amd
for rep in 1 2; do
  for v in default lut; do
    LIB=$L/libvampgpu.so; [ $v = lut ] && LIB=$L/libvampgpu_lut.so
    VAMP_AMD_LIB=$LIB timeout -k 10 120 python3 tools/kbench.py --edges 1048576 --reps 10 --tag $v >> $OUT 2>/dev/null || exit 1
  done
done
grep -E '"kernel": "(validate_setB|validate_setA|fkcc)"' $OUT | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["tag"], d["kernel"])].append(d["ms"])
for k, v in sorted(r.items()): print(k, ["%.3f" % x for x in v])'
