import os, sys, numpy as np
sys.path[:0] = ["sfm-project_amd", "oracle"]
import torch, synth, sfmcore
s = synth.make_scene(2, 512, seed=3)
X = s["desc"][0].astype(np.int64) - 128; Y = s["desc"][1].astype(np.int64) - 128
A = (X*X).sum(1); B = (Y*Y).sum(1); dot = X @ Y.T; e = dot - (B + 1)//2
es = -np.sort(-e, axis=1)
ctx = sfmcore.context(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
os.environ["SFM_L2FR_DEBUG"] = "1"
cnt, mt, dist = ctx.match_batch(T(s["desc"]), T(s["n_kp"]), T(np.array([[0, 1]], np.int32)), ratio=(4, 5))
mt = mt.cpu().numpy()[0]; dist = dist.cpu().numpy()[0]
print("e1 ok", (mt[:512, 0] == es[:, 0]).mean(), "e2 ok", (mt[:512, 1] == es[:, 1]).mean())
bad = np.nonzero(mt[:512, 0] != es[:, 0])[0][:5]
for q in bad:
    print(q, mt[q], es[q, :3], "argmax", np.argmax(e[q]), "T", dist[q])
# tile correctness
T1 = np.array([np.argmax(e[q]) // 32 for q in range(512)])
print("tile ok", (dist[:512] == T1).mean())
print("gpu e1 as which train:", [np.nonzero(e[q] == mt[q, 0])[0][:3] for q in bad[:3]])
badall = np.nonzero(mt[:512, 0] != es[:, 0])[0]
am = np.argmax(e, axis=1)
print("bad argmax tiles", np.bincount(am[badall] // 32, minlength=16))
print("all argmax tiles", np.bincount(am // 32, minlength=16))
print("bad argmax rows mod 32", np.bincount(am[badall] % 32, minlength=32))
print("bad query ids // 32", np.bincount(badall // 32, minlength=16))
# which value did the gpu report relative to true e over rows
for q in badall[:8]:
    print(q, "true", es[q,0], am[q], "gpu", mt[q,0], "rank of gpu e1", int((e[q] > mt[q,0]).sum()))
