#!/usr/bin/env python3
"""Static instruction mix of the vgpu kernels in a .hip file (development tool).

    python tools/isa_mix.py mr-vamp_amd/csrc/vgpu_kernels.hip [kernel-substring] [-- extra hipcc flags]
"""
import collections
import re
import subprocess
import sys

args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
src = args[0]
pat = args[1] if len(args) > 1 else "head_kernelILb0"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                       "-fno-slp-vectorize", "--offload-device-only", "-S", src, "-o", "/tmp/isa_mix.s"] + extra,
                      stderr=subprocess.DEVNULL)
lines = open("/tmp/isa_mix.s").read().splitlines()
starts = [i for i, l in enumerate(lines) if re.match(r"^_ZN4vgpu\w+:", l)]
for a, b in zip(starts, starts[1:] + [len(lines)]):
    name = lines[a].split(":")[0]
    if pat not in name:
        continue
    ins = [l.split()[0] for l in lines[a:b] if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]
    c = collections.Counter(ins)
    cls = collections.Counter()
    for op, n in c.items():
        k = ("valu" if op.startswith("v_") else "smem" if op.startswith("s_load") or op.startswith("s_buffer")
             else "branch" if op.startswith("s_cbranch") or op == "s_branch" else "salu" if op.startswith("s_")
             else "scratch" if op.startswith("scratch") else "vmem" if op.startswith(("global", "buffer", "flat"))
             else "other")
        cls[k] += n
    print(name[:70], dict(cls), "total", sum(c.values()))
