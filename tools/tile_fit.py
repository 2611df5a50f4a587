"""CPU model of nn_grid_wave_kernel's tiles on the C4 pair: for 64 / G consecutive slot-order queries,
the union of their complete boxes (seed = the exact NN distance) and whether it fits the wave's LDS
(cells + one per row, points ~2.2 per cell).  Scene "converged" (the model + 1e-3 noise) and "mid"
(the raw 5-degree scene), whole scene and an 8-way shard.  python tools/tile_fit.py"""
import numpy as np, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'iterative-closest-point_amd'))
import icp_amd
n=1<<20
m,p=icp_amd.synthetic_pair(n,seed=42)
lo=m.min(0); hi=m.max(0); ext=hi-lo; emax=ext.max()
vol=np.prod(np.maximum(ext,emax*1e-3)); h=np.cbrt(vol*2.0/n)
g=np.minimum(np.floor(ext/h)+1, 4096).astype(int)
inv=1.0/h
def cell(x): 
    t=(x-lo)*inv
    return np.clip(np.floor(t),0,g-1).astype(int)
from scipy.spatial import cKDTree
tree=cKDTree(m)
def morton(P):
    sc=1024.0/(hi-lo); c=np.clip(np.floor((P-lo)*sc),0,1023).astype(np.uint64)
    def spread(v):
        v=v.astype(np.uint64); r=np.zeros_like(v)
        for b in range(10): r|=((v>>np.uint64(b))&np.uint64(1))<<np.uint64(3*b)
        return r
    return spread(c[:,0])|(spread(c[:,1])<<np.uint64(1))|(spread(c[:,2])<<np.uint64(2))
for W in (1,8):
    q=p[:n//W]
    # mid-run: scene partially aligned: use model points + small noise (converged-ish) and the raw scene
    for name,Q in (('converged',m[:n//W]+np.random.default_rng(0).normal(scale=1e-3,size=(n//W,3))),('mid',q)):
        order=np.argsort(morton(Q),kind='stable'); Qs=Q[order]
        d,_=tree.query(Qs)  # seed ~ exact NN distance
        R=d
        c0=cell(Qs-R[:,None]); c1=cell(Qs+R[:,None])
        for G in (1,2,4,8):
            T=64//G; nt=len(Qs)//T
            a0=c0[:nt*T].reshape(nt,T,3).min(1); a1=c1[:nt*T].reshape(nt,T,3).max(1)
            dims=a1-a0+1; nent=dims[:,1]*dims[:,2]*(dims[:,0]+1); cells=dims.prod(1)
            for lim in ((256,512),(512,1024)):
                fit=(nent<=lim[0])&(cells*2.2<=lim[1])
                print(W,name,'G',G,'lim',lim,'fit %.3f'%fit.mean(),'mean cells %.0f'%cells.mean())
