"""Summarise rocprofv3 --pmc CSVs per kernel (per-wave averages)."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
tot = collections.defaultdict(lambda: collections.defaultdict(float))
nd = collections.defaultdict(set)
for f in sorted(glob.glob(f"{d}/pmc*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vgpu::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        nd[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, v in tot.items():
    print(k)
    waves = v.get("SQ_WAVES", 0) / max(1, len(nd[(k, "SQ_WAVES")]))
    if v.get("SQ_ACTIVE_INST_VALU"):
        n1 = len(nd[(k, "SQ_THREAD_CYCLES_VALU")]) or 1
        n2 = len(nd[(k, "SQ_ACTIVE_INST_VALU")]) or 1
        print(f"  VALUUtilization(%)           {100 * (v['SQ_THREAD_CYCLES_VALU'] / n1) / ((v['SQ_ACTIVE_INST_VALU'] / n2) * 64):14.1f}")
    for c, x in sorted(v.items()):
        n = len(nd[(k, c)])
        per = x / n
        extra = f"  per-wave {per / waves:10.1f}" if waves and c.startswith("SQ_INSTS") else ""
        print(f"  {c:28s} {per:14.4g}{extra}")
