import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "mr-vamp_amd")
import oracle_py as oracle
oracle.build()
import vamp_amd as vamp
from test_gpu_roadmap import knn_gpu
F = np.float32
n, dim = 20000, 7
rng = np.random.default_rng(21)
V = oracle.robot_scale("panda", rng.random((n, dim), dtype=F))
V[n // 2] = V[n // 3]
sm = oracle.SPACE_MEASURE["panda"]
onb, od, oc = oracle.roadmap_knn(V, sm)
gnb, gd, gc = knn_gpu(vamp, V, sm, onb.shape[1])
bad = [i for i in range(n) if not (np.array_equal(gnb[i,:oc[i]], onb[i,:oc[i]]) and np.array_equal(gd[i,:oc[i]], od[i,:oc[i]]))]
print("bad rows", len(bad), bad[:10])
for i in bad[:4]:
    c = oc[i]
    print(i, "k", c)
    print(" o", onb[i,:c].tolist()); print(" g", gnb[i,:c].tolist())
    print(" od", od[i,:c].tolist()); print(" gd", gd[i,:c].tolist())
    dd = np.nonzero(gd[i,:c] != od[i,:c])[0]
    print(" dist diffs at", dd[:10])
