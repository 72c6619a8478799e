"""Save this host's _mm256_rsqrt_ps table (oracle/vamp_oracle.c vo_rsqrt_probe) with the CPU model,
so reference-DAG fixtures can be evaluated here under another host's rsqrt (tools/make_golden.py
--alt-lut).  Usage: python tools/dump_host_rsqrt.py OUT.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import oracle_py as op  # noqa: E402

op.build()
lut, kb = op.rsqrt_probe()
model = "unknown"
for line in open("/proc/cpuinfo"):
    if line.startswith("model name"):
        model = line.split(":", 1)[1].strip()
        break
np.savez_compressed(sys.argv[1], rsqrt_lut=lut, rsqrt_kbits=np.int32(kb), cpu_model=np.array(model))
print(f"{model}: kbits {kb}, {lut.size} entries -> {sys.argv[1]}")
