"""Ideal exact pruning of K2 (CPU simulation on cfg3 pairs): every hypothesis pruned on its own as
soon as count + remaining < the final best count (known from the start), checked every 64 (or 16)
matches, vs the wave-level ordered schedule with that same final bound.  Prints fractions of the
full (hypothesis x match) scoring work.  Usage: python tests/perf/ransac_prune_ideal.py"""
import os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]
import synth, oracle as O
s = synth.make_scene(50, 2048, seed=0)
pairs = synth.unordered_pairs(50)
rng = np.random.default_rng(1)
PV=64
tot = np.zeros(5)
for p in rng.choice(len(pairs), 4, replace=False):
    a,b = pairs[p]
    q,t,_ = O.match(s["desc"][a], s["desc"][b], 0, 1, (4,5))
    x1 = s["kps"][a][q].astype(np.float64); x2 = s["kps"][b][t].astype(np.float64)
    M=len(q); H=4096
    c1=x1.mean(0); s1=np.sqrt(2)/np.mean(np.linalg.norm(x1-c1,axis=1))
    c2=x2.mean(0); s2=np.sqrt(2)/np.mean(np.linalg.norm(x2-c2,axis=1))
    X1=(x1-c1)*s1; X2=(x2-c2)*s2
    h1=np.c_[X1,np.ones(M)]; h2=np.c_[X2,np.ones(M)]
    masks=np.zeros((H,M),bool)
    for h in range(H):
        idx=O.sample8(42,int(a),int(b),h,M)
        A=np.c_[X2[idx,0:1]*X1[idx], X2[idx,0:1], X2[idx,1:2]*X1[idx], X2[idx,1:2], X1[idx], np.ones((8,1))]
        _,_,vt=np.linalg.svd(A); F=vt[-1].reshape(3,3)
        u,sv,v=np.linalg.svd(F); F=u@np.diag([sv[0],sv[1],0])@v
        aa=h1@F.T; bb=h2@F
        r=np.sum(h2*aa,1)
        e = s2*s2*(aa[:,0]**2+aa[:,1]**2) + s1*s1*(bb[:,0]**2+bb[:,1]**2) - r*r
        masks[h]=e>0
    cnt=masks.sum(1); cum=np.cumsum(masks,1); best=cnt.max()
    # ideal per-lane: bound = final best known from start, checked every 64 matches
    chk=np.arange(64,M+64,64).clip(max=M)
    def lane_stop(h, bound, start):
        for m in chk:
            if m<=start: continue
            if cum[h,m-1]+(M-m) < bound: return m
        return M
    ideal = sum(lane_stop(h, best, PV) - PV for h in range(H)) + H*PV
    # per-wave with final bound from start (sorted by preview)
    prev=cum[:,PV-1]; order=np.argsort(-prev,kind="stable")
    wave_final = 0
    for w in range(H//64):
        hs = order[w*64:(w+1)*64]
        wave_final += 64*(max(lane_stop(h, best, PV) for h in hs) - PV)
    wave_final += H*PV
    # per-lane stop with every-16 checks
    chk16=np.arange(16,M+16,16).clip(max=M)
    def lane_stop16(h,bound,start):
        for m in chk16:
            if m<=start: continue
            if cum[h,m-1]+(M-m) < bound: return m
        return M
    ideal16 = sum(lane_stop16(h, best, PV) - PV for h in range(H)) + H*PV
    tot += [ideal, wave_final, ideal16, H*M, 0]
    print(p, M, best, "ideal-lane %.3f  wave-sorted-finalbound %.3f  ideal-lane-16 %.3f" % (ideal/(H*M), wave_final/(H*M), ideal16/(H*M)))
print("overall ideal-lane %.3f wave-sorted-final %.3f ideal16 %.3f" % (tot[0]/tot[3], tot[1]/tot[3], tot[2]/tot[3]))
