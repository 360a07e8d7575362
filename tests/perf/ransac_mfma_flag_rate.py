"""Why the certified f16-MFMA Sampson filter (SFM_RANSAC_MODE=3) cannot pay: fraction
of (hypothesis, match) evaluations whose decision a form error Delta = eps * S (S = sum |terms| of
the form, from the pair's operand maxima) leaves uncertain, |P| <= 4w(|r| + w) + ..., w = 4 Da + Dr,
on a cfg3-like pair (float64 8-point hypotheses).  The epipolar residual r cancels ~2^10 over its
terms, so eps = 2^-17 (the MFMA accumulation bound) flags ~0.1 % of evaluations (>= 1 per
1024-evaluation tile); a per-element S (one more MFMA) would cut it ~10x.  CPU only.
Usage: python tests/perf/ransac_mfma_flag_rate.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]
import synth, oracle as O
s=synth.make_scene(2,2048,seed=3)
q,t,_=O.match(s["desc"][0],s["desc"][1],0,1,(4,5))
x1=s["kps"][0][q].astype(np.float64); x2=s["kps"][1][t].astype(np.float64)
M=len(q)
def norm(x):
    c=x.mean(0); d=np.sqrt(((x-c)**2).sum(1)).mean(); sc=np.sqrt(2)/d; return (x-c)*sc, sc
n1,s1=norm(x1); n2,s2=norm(x2)
thr=1.0; k1=1/(s1*np.sqrt(thr)); k2=1/(s2*np.sqrt(thr))
X1=n1*k1; X2=n2*k2
rng=np.random.default_rng(0)
H=512
res={}
for h in range(H):
    idx=rng.choice(M,8,replace=False)
    A=np.stack([n2[idx,0]*n1[idx,0],n2[idx,0]*n1[idx,1],n2[idx,0],n2[idx,1]*n1[idx,0],n2[idx,1]*n1[idx,1],n2[idx,1],n1[idx,0],n1[idx,1],np.ones(8)],1)
    F=np.linalg.svd(A)[2][-1].reshape(3,3)
    U,S,Vt=np.linalg.svd(F); S[2]=0; F=U@np.diag(S)@Vt
    G=F.copy().ravel(); G[2]*=k1; G[5]*=k1; G[6]*=k2; G[7]*=k2; G[8]*=k1*k2
    a0=G[0]*X1[:,0]+G[1]*X1[:,1]+G[2]; a1=G[3]*X1[:,0]+G[4]*X1[:,1]+G[5]; c2=G[6]*X1[:,0]+G[7]*X1[:,1]+G[8]
    b0=G[0]*X2[:,0]+G[3]*X2[:,1]+G[6]; b1=G[1]*X2[:,0]+G[4]*X2[:,1]+G[7]
    r=X2[:,0]*a0+X2[:,1]*a1+c2; den=a0**2+a1**2+b0**2+b1**2; P=den-r**2
    Xm=np.abs(np.concatenate([X1,X2])).max()
    Sa=max(abs(G[0])*Xm+abs(G[1])*Xm+abs(G[2]),abs(G[3])*Xm+abs(G[4])*Xm+abs(G[5]),abs(G[0])*Xm+abs(G[3])*Xm+abs(G[6]),abs(G[1])*Xm+abs(G[4])*Xm+abs(G[7]))
    u=np.stack([X2[:,0]*X1[:,0],X2[:,0]*X1[:,1],X2[:,0],X2[:,1]*X1[:,0],X2[:,1]*X1[:,1],X2[:,1],X1[:,0],X1[:,1],np.ones(M)],1)
    Sr=(np.abs(G)*np.abs(u).max(0)).sum()
    Sr_elem=(np.abs(G)[None,:]*np.abs(u)).sum(1)
    for name,eps in (("2^-17",2**-17),("2^-19",2**-19),("2^-21",2**-21),("2^-23",2**-23)):
        Da=eps*Sa; Dr=eps*Sr
        c1=2*(8*Da+2*Dr); c0=4*(4*Da+Dr)**2; c2=8*2**-19
        t=c2*r*r+c1*np.abs(r)+c0
        f=np.abs(P)<=t
        Dre=eps*Sr_elem
        t2=c2*r*r+2*(8*Da+2*Dre)*np.abs(r)+4*(4*Da+Dre)**2
        f2=np.abs(P)<=t2
        d=res.setdefault(name,[0,0,0]); d[0]+=f.sum(); d[1]+=f2.sum(); d[2]+=M
print("M",M)
for k,v in res.items(): print(k,"flag frac (global S)",v[0]/v[2],"(per-elem S)",v[1]/v[2], "per 1024-eval tile", 1024*v[0]/v[2])
