"""Development estimate (CPU, oracle sphere_fk): how often a composite arm's link spheres reach a sphere enclosing the other
arm (all links / links 0-3 / links 4-hand), per lane and per 64-lane wave -- the ceiling of a wave-level prefilter of
the 121 inter-arm bounding pairs.  Uniform configurations, bases 1 m apart."""
import sys, json, numpy as np
sys.path.insert(0,'tests'); import oracle_py as oracle
oracle.build()
m=json.load(open('model/panda.json')); sp=m['spheres']
links=sorted(set(s['link'] for s in sp), key=lambda l: min(i for i,s in enumerate(sp) if s['link']==l))
rng=np.random.default_rng(0); F=np.float32
N=64*2000
qa=oracle.scale(rng.random((N,7),dtype=F)); qb=oracle.scale(rng.random((N,7),dtype=F))
ca=np.asarray(oracle.sphere_fk(qa,(0,0,0))); cb=np.asarray(oracle.sphere_fk(qb,(100,0,0)))
r=np.array([s['radius'] for s in sp])
def link_spheres(c):
    out=[]
    for l in links:
        idx=[i for i,s in enumerate(sp) if s['link']==l]
        cc=c[:,idx]; cen=cc.mean(1); R=(np.linalg.norm(cc-cen[:,None],axis=2)+r[idx]).max(1)
        out.append((cen,R))
    return out
A=link_spheres(ca); B=link_spheres(cb)
print('links', links, 'B base x', cb[:,0,0].mean())
def encl(parts):
    cen=np.mean([p[0] for p in parts],0); R=np.max([np.linalg.norm(p[0]-cen,axis=1)+p[1] for p in parts],0); return cen,R
EB=encl(B); EBlo=encl(B[:4]); EBhi=encl(B[4:])
print('E_B radius mean', EB[1].mean(), 'lo', EBlo[1].mean(), 'hi', EBhi[1].mean())
for name,E in (('EB',EB),('EBlo',EBlo),('EBhi',EBhi)):
    hits=[]
    for i,(c,R) in enumerate(A):
        t=np.linalg.norm(c-E[0],axis=1) < R+E[1]
        wave=t.reshape(-1,64).any(1).mean()
        hits.append((round(t.mean(),3), round(wave,3)))
    print(name, hits)
# pairwise actual
pair=np.zeros((len(A),len(B)))
for i,(c,R) in enumerate(A):
    for j,(d,S) in enumerate(B):
        pair[i,j]=(np.linalg.norm(c-d,axis=1)<R+S).mean()
print('pair fire rate total', pair.sum(), 'max', pair.max())
