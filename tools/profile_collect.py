"""Collect the round's rocprofv3 outputs (gpurun_out/) into committed profiles/ files.

    python tools/profile_collect.py r01
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

R = sys.argv[1] if len(sys.argv) > 1 else "r01"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")
os.makedirs(P, exist_ok=True)

stats = glob.glob(f"{G}/prof_{R}/**/*kernel_stats.csv", recursive=True)
if stats:
    shutil.copy(stats[0], f"{P}/{R}_bench_kernel_stats.csv")
    print("kernel stats ->", f"{P}/{R}_bench_kernel_stats.csv")
per = collections.defaultdict(lambda: collections.defaultdict(list))
step_bytes = collections.defaultdict(float)
calls = 0
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{G}/pmc_{R}_{c}/**/*counter_collection.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        byd = collections.defaultdict(float)
        name = {}
        for r in rows:
            byd[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            name[int(r["Dispatch_Id"])] = (r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vgpu::", ""),
                                           r["Grid_Size"])
        for d, v in byd.items():
            per[name[d]][c].append(v)
        # one validate_motions call = the dispatches from a head bound kernel up to the next one;
        # calls of the full-mask mode (they contain SrcTailMaskT kernels) and the FK leg are skipped
        order = sorted(byd)
        starts = [i for i, d in enumerate(order) if name[d][0].startswith("bound_kernel<") and "SrcHead" in name[d][0]]
        n_calls = 0
        for j, i0 in enumerate(starts):
            i1 = starts[j + 1] if j + 1 < len(starts) else len(order)
            seg = [order[i] for i in range(i0, i1) if "sphere_fk" not in name[order[i]][0]]
            if any("SrcTailMask" in name[d][0] or "mask_finish" in name[d][0] for d in seg):
                continue
            step_bytes[c] += sum(byd[d] for d in seg)
            n_calls += 1
        if c == "FETCH_SIZE":
            calls = n_calls
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes (tools/profile_round.sh {R}), "
                  "bench.py 2^20-edge cage workload, every validate_motions kernel; "
                  "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 "
                  "(MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a wide streaming read on gfx950; "
                  "uncalibrated for other access widths)", "kernels": {}}
for (k, grid), d in per.items():
    f = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
    w = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
    rec = {"grid": int(grid), "fetch_kb": f, "write_kb": w, "bytes_corrected": (2 * f + w) * 1024,
           "bytes_raw": (f + w) * 1024}
    out["kernels"].setdefault(k, []).append(rec)
if calls:
    out["validate_calls"] = calls
    out["step_bytes_per_call"] = (2 * step_bytes["FETCH_SIZE"] + step_bytes["WRITE_SIZE"]) * 1024 / calls
json.dump(out, open(f"{P}/traffic_{R}.json", "w"), indent=1)
print(json.dumps(out, indent=1)[:2000])
