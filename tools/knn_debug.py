"""Development: the spatial-index kNN (VAMP_AMD_KNN_COOP / VAMP_AMD_KNN_QCODE select the kernel) vs the GPU brute force on n Halton
Fetch vertices; prints the mismatched queries.   python tools/knn_debug.py [n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mr-vamp_amd"), os.path.join(ROOT, "tests")]
from test_gpu_roadmap import knn_gpu  # noqa: E402

import oracle_py as op  # noqa: E402
import vamp_amd as vamp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
V = vamp.fetch.scale_configuration(vamp.halton(8, 1, n))
sm = op.SPACE_MEASURE["fetch"]
a = knn_gpu(vamp, V, sm, mode=2)
b = knn_gpu(vamp, V, sm, mode=1)
(an, ad, ac), (bn, bd, bc) = a, b
print("count mismatches", int((ac != bc).sum()))
bad = [i for i in range(n) if ac[i] != bc[i] or not np.array_equal(an[i, :ac[i]], bn[i, :bc[i]])]
print("list mismatches", len(bad), "first", bad[:20])
for i in bad[:5]:
    c = int(bc[i])
    sa, sb = set(an[i, :ac[i]].tolist()), set(bn[i, :c].tolist())
    print(f"query {i}: k={c} missing {sorted(sb - sa)[:8]} extra {sorted(sa - sb)[:8]}")
    for j in sorted(sb - sa)[:3]:
        print("   missing", j, "dist", float(bd[i, list(bn[i, :c]).index(j)]))
    for j in sorted(sa - sb)[:3]:
        print("   extra", j, "dist", float(ad[i, list(an[i, :ac[i]]).index(j)]))
    print("   order equal as sets:", sa == sb)
sys.exit(1 if bad else 0)
