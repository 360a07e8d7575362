"""Simulation of K2's exact pruning schedules on cfg3 pairs (CPU, oracle matches + float64 Sampson).

For a sample of pairs: every hypothesis's inlier mask, then the fraction of (hypothesis, match)
evaluations each schedule performs — natural order with the bound from earlier blocks ("model A",
the single-pass kernel) vs ordering by a PV-match preview (the ordered kernel; PV env var).
Usage: PV=64 python tests/perf/ransac_prune_sim.py"""
import os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys, numpy as np
sys.path[:0]=[os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]
import synth, oracle as O
s = synth.make_scene(50, 2048, seed=0)
pairs = synth.unordered_pairs(50)
rng = np.random.default_rng(1)
acc=np.zeros(3); tot=0
PV=int(os.environ.get("PV","64"))
for p in rng.choice(len(pairs), 5, replace=False):
    a,b = pairs[p]
    q,t,_ = O.match(s["desc"][a], s["desc"][b], 0, 1, (4,5))
    x1 = s["kps"][a][q].astype(np.float64); x2 = s["kps"][b][t].astype(np.float64)
    M=len(q); H=4096
    c1=x1.mean(0); s1=np.sqrt(2)/np.mean(np.linalg.norm(x1-c1,axis=1))
    c2=x2.mean(0); s2=np.sqrt(2)/np.mean(np.linalg.norm(x2-c2,axis=1))
    X1=(x1-c1)*s1; X2=(x2-c2)*s2
    masks=np.zeros((H,M),bool)
    h1=np.c_[X1,np.ones(M)]; h2=np.c_[X2,np.ones(M)]
    for h in range(H):
        idx=O.sample8(42,int(a),int(b),h,M)
        A=np.c_[X2[idx,0:1]*X1[idx], X2[idx,0:1], X2[idx,1:2]*X1[idx], X2[idx,1:2], X1[idx], np.ones((8,1))]
        _,_,vt=np.linalg.svd(A); F=vt[-1].reshape(3,3)
        u,sv,v=np.linalg.svd(F); F=u@np.diag([sv[0],sv[1],0])@v
        aa=h1@F.T; bb=h2@F
        r=np.sum(h2*aa,1)
        e = s2*s2*(aa[:,0]**2+aa[:,1]**2) + s1*s1*(bb[:,0]**2+bb[:,1]**2) - r*r
        masks[h]=e>0
    cnt=masks.sum(1); cum=np.cumsum(masks,1)
    chk=np.arange(64,M+64,64).clip(max=M)
    def wave_work(lanes,bound,start=0):
        for m in chk:
            if m<=start: continue
            if np.all(cum[lanes,m-1]+(M-m) < bound): return m-start
        return M-start
    def run(order, start):
        # blocks of 256 in 'order'; block bx has bound = max final count of blocks < bx (model A)
        work=0
        for bx in range(16):
            hs=order[bx*256:(bx+1)*256]
            bnd = cnt[order[:bx*256]].max() if bx>0 else 0
            for w in range(4):
                work+=64*wave_work(hs[w*64:(w+1)*64],bnd,start)
        return work
    base=run(np.arange(H),0)
    prev=cum[:,PV-1]
    order=np.argsort(-prev,kind="stable")
    sorted_work=run(order,PV)+H*PV
    acc+=[base, sorted_work, H*M]; tot+=H*M
    print(p, M, cnt.max(), round(base/(H*M),3), round(sorted_work/(H*M),3))
print("current(model A) %.3f  sorted+preview %.3f" % (acc[0]/acc[2], acc[1]/acc[2]))
