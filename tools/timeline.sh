#!/bin/bash
# Kernel timeline of the last bench step (gaps between kernels included).  Usage: tools/timeline.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/tl_$T -o tl --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fk-leg > gpurun_out/tl_$T.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/tl_$T.log; exit 1; }
f=$(find gpurun_out/tl_$T -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# last validate step: from the last head-stage kernel back
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "SrcHead" in n and "bound" in n or "validate_head" in n]
s = idx[-1] if idx else 0
# include the step up to the next head start or end (profiling pass comes after; take step before last)
s = idx[-2] if len(idx) > 1 else s
e = idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
prev = t0
for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1e3:9.1f} us  gap {(st - prev) / 1e3:7.1f}  dur {(en - st) / 1e3:8.1f}  {r['Kernel_Name'][:80]}")
    prev = en
print("step span us", (int(rows[e]["Start_Timestamp"]) - t0) / 1e3)
PY
