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
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{G}/pmc_{R}_{c}/**/*counter_collection.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        byd = collections.defaultdict(float)
        name = {}
        for r in rows:
            byd[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = (r["Kernel_Name"].split("(")[0].split("::")[-1], r["Grid_Size"])
        for d, v in byd.items():
            per[name[d]][c].append(v)
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes (tools/profile_round.sh {R}), "
                  "kbench 2^20-edge cage workload; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 "
                  "(MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a wide streaming read on gfx950; "
                  "uncalibrated for other access widths)", "kernels": {}}
for (k, grid), d in per.items():
    f = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
    w = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
    rec = {"grid": int(grid), "fetch_kb": f, "write_kb": w, "bytes_corrected": (2 * f + w) * 1024,
           "bytes_raw": (f + w) * 1024}
    out["kernels"].setdefault(k, []).append(rec)
heads = [r for r in out["kernels"].get("panda_validate_head_kernel", []) if r["grid"] == 8 * (1 << 20)]
if heads:
    out["head_bytes_per_launch"] = heads[0]["bytes_corrected"]
json.dump(out, open(f"{P}/traffic_{R}.json", "w"), indent=1)
print(json.dumps(out, indent=1)[:2000])
