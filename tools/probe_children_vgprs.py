"""VGPRs each Fetch check's children need when compiled alone (development; tools/probe/children_vgprs.hip):
compiles the probe for gfx950 and prints, per check, the children kernel's .vgpr_count -- the data behind
the children register classes (vgpu_fetch_staged.hip kClassOf / kClassWaves).
    python tools/probe_children_vgprs.py"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import kernel_resources  # noqa: E402

out = "/tmp/children_vgprs.o"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                       "-fno-slp-vectorize", "-c", os.path.join(ROOT, "tools", "probe", "children_vgprs.hip"), "-o", out])
rows = []
for k in kernel_resources.kernels(out):
    m = re.search(r"ProbeR<(\d+)>", k["name"])
    if m and "children_kernel" in k["name"]:
        rows.append((int(m.group(1)), k["vgpr"], k["vgpr_spill"], k["scratch"]))
for c, v, s, sc in sorted(rows):
    print(f"check {c:2d}: {v:3d} VGPRs (spill {s}, scratch {sc})")
