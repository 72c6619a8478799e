#!/bin/bash
# A/B of the staged pass's check rounds (VAMP_AMD_ROUNDS: comma-separated check masks, Panda) on the
# headline edges (set B), raw pairs (set A) and fkcc: tools/kbench.py per round set, alternating twice;
# plus one VAMP_AMD_STAGED_STATS pass (each staged pass's per-check bounding counts).
# usage: [SETS="default m1,m2 ..."] bash tools/rounds_ab.sh TAG  -> gpurun_out/rounds_TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/rounds_${1:-r04}.log
: > $OUT
VAMP_AMD_STAGED_STATS=1 timeout -k 10 120 python3 tools/kbench.py --edges 1048576 --reps 1 --tag stats >> $OUT 2>&1 || exit 1
# default (chosen per batch) | env, self | env, self w/o gated, gated | early env, late env, self w/o gated, gated
SETS="${SETS:-default 0x8043091f,0x7fbcf6e0 0x8043091f,0x3b9476e0,0x44208000 0x1f,0x80430900,0x3b9476e0,0x44208000}"
for rep in 1 2; do
  for s in $SETS; do
    if [ "$s" = default ]; then
      timeout -k 10 120 python3 tools/kbench.py --edges 1048576 --reps 5 --tag "default" >> $OUT 2>&1 || exit 1
    else
      VAMP_AMD_ROUNDS=$s timeout -k 10 120 python3 tools/kbench.py --edges 1048576 --reps 5 --tag "$s" >> $OUT 2>&1 || exit 1
    fi
  done
done
grep -v amdgpu.ids $OUT | grep -E '"kernel": "(validate_setB|validate_setA|fkcc)"' | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["tag"], d["kernel"])].append(d["ms"])
for k, v in sorted(r.items()): print(k, ["%.3f" % x for x in v])'
