#!/usr/bin/env python3
"""Per-kernel averages of the CAPT counter passes (tools/gpu_capt_pmc.sh TAG -> gpurun_out/capt_TAG_pmc*/)
as the JSON bench.py's capt line reads: {"kernels": {name: {counter: per-dispatch mean, ...,
"L2_hit_rate", "VALU_insts_per_wave"}}}.

    python tools/capt_pmc_json.py TAG OUT.json
"""
import collections
import csv
import glob
import json
import sys

tag, out = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in sorted(glob.glob(f"gpurun_out/capt_{tag}_pmc*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vgpu::", "")
        vals[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
kernels = {}
for k, cs in vals.items():
    rec = {c: sum(d.values()) / len(d) for c, d in cs.items()}
    if "TCC_HIT_sum" in rec and "TCC_MISS_sum" in rec:
        rec["L2_hit_rate"] = rec["TCC_HIT_sum"] / max(1.0, rec["TCC_HIT_sum"] + rec["TCC_MISS_sum"])
    if "SQ_INSTS_VALU" in rec and rec.get("SQ_WAVES"):
        rec["VALU_insts_per_wave"] = rec["SQ_INSTS_VALU"] / rec["SQ_WAVES"]
    kernels[k] = rec
json.dump({"source": f"tools/gpu_capt_pmc.sh {tag} on MI355X: rocprofv3 --pmc, one pass per counter group, "
                     "tools/kbench_capt.py (2^20 Panda configurations fkcc vs the 10k-point CAPT, then 2^20 raw "
                     "collides_simd queries); values per dispatch, averaged over dispatches",
           "units": "FETCH_SIZE/WRITE_SIZE in KB as rocprofv3 reports them; TCC_* are L2 request counts",
           "kernels": kernels}, open(out, "w"), indent=1)
print(json.dumps(kernels, indent=1)[:1500])
