"""VERDICT r5 item 1 ("then"): the bench rule (L2 mutual + ratio 4/5) at cfg4's K = 4096 through
the two exact implementations — the mutual kernel (SFM_L2_PATH=mutual, the dispatcher's default
for this rule) and the forward/recovery/reverse ratio path (SFM_L2_PATH=fr) — interleaved in one
process on a cfg4 shard (the 1/8 shard rank 3 gets at N = 8: ~15.6 k pairs of the 500 x 4096
scene), with their outputs compared bit for bit on every pair.
python tests/perf/k1_mutual_ab.py  (SHARD=r/n, ROUNDS, N_IMG, K override; cfg3: N_IMG=50 K=2048
SHARD=0/1)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import match_graph
import sfmcore
import synth


def main():
    r, n = (int(x) for x in os.environ.get("SHARD", "3/8").split("/"))
    rounds = int(os.environ.get("ROUNDS", "3"))
    n_img, k = int(os.environ.get("N_IMG", "500")), int(os.environ.get("K", "4096"))
    s = synth.make_scene(n_img, k, seed=0)
    pairs = synth.unordered_pairs(n_img)
    lo, hi = match_graph.shard_range(pairs, r, n, s["n_kp"])
    pairs = pairs[lo:hi]
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, pr = T(s["desc"]), T(s["n_kp"]), T(pairs)
    ops = 2.0 * 128 * float(np.sum(s["n_kp"][pairs[:, 0]].astype(np.float64)
                                   * s["n_kp"][pairs[:, 1]]))
    outs, times = {}, {"mutual": [], "fr": []}
    for _ in range(rounds):
        for path in ("mutual", "fr"):
            os.environ["SFM_L2_PATH"] = path
            out = ctx.match_batch(desc, n_kp, pr, cross_check=sfmcore.XC_MUTUAL, ratio=(4, 5))
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            out = ctx.match_batch(desc, n_kp, pr, cross_check=sfmcore.XC_MUTUAL, ratio=(4, 5),
                                  out=out)
            ev[1].record()
            torch.cuda.synchronize()
            times[path].append(ev[0].elapsed_time(ev[1]))
            outs[path] = [t.cpu().numpy() for t in out]
    cm, mm, dm = outs["mutual"]
    cf, mf, df = outs["fr"]
    same = bool((cm == cf).all())
    if same:
        for p in range(len(pairs)):
            c = cm[p]
            same &= bool((mm[p, :c] == mf[p, :c]).all() and (dm[p, :c] == df[p, :c]).all())
    res = {"shard": f"{r}/{n}", "pairs": int(len(pairs)), "n_img": n_img, "k": k,
           "ms_mutual": times["mutual"], "ms_fr": times["fr"],
           "tops_mutual": ops / (min(times["mutual"]) * 1e-3) / 1e12,
           "tops_fr": ops / (min(times["fr"]) * 1e-3) / 1e12,
           "matches": int(cm.sum()), "bit_identical": same,
           "lib": os.path.basename(os.environ.get("SFMCORE_LIB", "libsfmcore.so"))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
