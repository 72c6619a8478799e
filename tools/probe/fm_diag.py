import os, sys, numpy as np
sys.path.insert(0, 'mr-vamp_amd'); sys.path.insert(0, 'tests')
import torch, vamp_amd as vamp, oracle_py as oracle
from test_gpu_parity import gpu_env_from_oracle
F = np.float32
oracle.build()
rng = np.random.default_rng(21)
oenv = oracle.sphere_cage_env()
env = gpu_env_from_oracle(vamp, oenv)
s = oracle.scale(rng.random((20000, 7), dtype=F)); g = oracle.scale(rng.random((20000, 7), dtype=F))
g[:10000] = s[:10000] + (g[:10000] - s[:10000]) * F(0.2); g[:5] = s[:5]
ok_c, n_c, blk_c, _ = vamp.panda_0_0.cpu_validate_mask(s, g, env)
dev = torch.device("cuda", 0)
ds, dg = torch.from_numpy(s).to(dev), torch.from_numpy(g).to(dev)
ok = torch.empty(len(s), dtype=torch.uint8, device=dev); nb = torch.empty(len(s), dtype=torch.int32, device=dev)
blk = torch.empty(int(n_c.sum()) + 7, dtype=torch.uint8, device=dev)
ctx = vamp.context(0)
total = vamp.panda_0_0.validate_mask_device(ds.data_ptr(), dg.data_ptr(), len(s), env, ok.data_ptr(), nb.data_ptr(), blk.data_ptr(), blk.numel(), ctx)
ctx.sync()
okg = ok.cpu().numpy().astype(bool); blkg = blk[:total].cpu().numpy().astype(bool)
off = np.concatenate([[0], np.cumsum(n_c)])
head = blkg[off[:-1]]; headc = blk_c[off[:-1]]
print(os.environ.get('VAMP_AMD_NEAR'), os.environ.get('VAMP_AMD_HEAD_LIST'), 'total', total, int(n_c.sum()), 'ok mism', int((okg != ok_c).sum()), 'blk mism', int((blkg != blk_c).sum()), 'head mism', int((head != headc).sum()), 'gpu ok', okg.mean(), 'cpu ok', ok_c.mean())
bad = np.nonzero(blkg != blk_c)[0][:10]; print('bad blocks', bad, blkg[bad], blk_c[bad])
ok_e, _ = vamp.panda_0_0.validate_batch(s, g, env); print('early-exit vs cpu mism', int((ok_e != ok_c).sum()))
