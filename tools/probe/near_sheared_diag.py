"""Development probe: tests/test_gpu_near.py's sheared-cuboid scene (seed from argv), GPU vs oracle motions with
per-edge mismatch details (which edges, GPU/oracle ok and block counts)."""
import os, sys
import numpy as np
sys.path.insert(0, 'mr-vamp_amd'); sys.path.insert(0, 'tests')
import oracle_py as oracle
import vamp_amd as vamp
from test_gpu_parity import gpu_env_from_oracle
from test_gpu_near import sheared_scene
F = np.float32
oracle.build()
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 6
rng = np.random.default_rng(seed)
oenv = sheared_scene(oracle, rng)
env = gpu_env_from_oracle(vamp, oenv)
q = oracle.scale(rng.random((12000, 7), dtype=F))
for base in ((0, 0, 0), (2, 2, 0)):
    got = vamp.PandaBase(*base).fkcc_batch(q, env)
    want = oracle.fkcc_threads(oenv, q, base)
    print('fkcc', base, 'mismatch', int((got != want).sum()))
n_edges = 2000
s = oracle.scale(rng.random((n_edges, 7), dtype=F)); g = oracle.scale(rng.random((n_edges, 7), dtype=F))
g[: n_edges // 2] = s[: n_edges // 2] + (g[: n_edges // 2] - s[: n_edges // 2]) * F(0.1)
ok, n = vamp.panda_0_0.validate_batch(s, g, env)
ook, on = oracle.validate_motions(oenv, s, g, (0, 0, 0))
bad = np.nonzero((ok != ook) | (n != on))[0]
print(os.environ.get('VAMP_AMD_NEAR'), os.environ.get('VAMP_AMD_HEAD_LIST'), 'motion mismatches', len(bad), 'edges', bad[:10], 'gpu ok', ok[bad[:10]].astype(int), 'oracle ok', ook[bad[:10]].astype(int), 'n', n[bad[:10]], on[bad[:10]])
for e in bad[:3]:
    k = int(on[e]); d = (g[e] - s[e]).astype(F)
    for blk in range(k):
        pass
    # head block configs and their oracle fkcc
    pct = np.array([(l + 1) / 8 for l in range(8)], F)
    q8 = np.array([[F(np.float64(d[j]) * np.float64(pct[l]) + np.float64(s[e][j])) for j in range(7)] for l in range(8)], F)
    print(' edge', e, 'head oracle fkcc', oracle.fkcc_threads(oenv, q8, (0, 0, 0)).astype(int), 'gpu fkcc', vamp.panda_0_0.fkcc_batch(q8, env).astype(int))
# single-edge and sub-batch reruns of the first mismatching edges
if len(bad):
    sel = bad[:8]
    ok1, n1 = vamp.panda_0_0.validate_batch(s[sel], g[sel], env)
    print('subset rerun gpu ok', ok1.astype(int), 'oracle', ook[sel].astype(int))
    for e in sel[:2]:
        oke, ne = vamp.panda_0_0.validate_batch(s[e:e + 1], g[e:e + 1], env)
        print(' single edge', e, 'gpu', int(oke[0]), 'n', int(ne[0]), 'oracle', int(ook[e]))
