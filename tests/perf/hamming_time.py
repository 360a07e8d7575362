"""Times the reference's own matcher path (ORB 256-bit Hamming, OpenCV cross-check rule, distance
< 26: code/feature_matching.py:48-58) batched over all pairs of N_IMG synthetic ORB-like images x K
descriptors (reference default nfeatures = 500), and checks a sample against the CPU oracle.
Usage: N_IMG=50 K=500 python tests/perf/hamming_time.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]

import numpy as np
import torch

import oracle as O
import sfmcore
import synth


def main():
    n_img = int(os.environ.get("N_IMG", "50"))
    K = int(os.environ.get("K", "500"))
    s = synth.make_scene(n_img, K, seed=0, orb=True)
    pairs = synth.unordered_pairs(n_img)
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, pr = T(s["desc"]), T(s["n_kp"]), T(pairs)
    res = {}
    # key = the key-in-the-accumulator kernel (round 4 default without a ratio test),
    # mfma = the column-winner kernel (OpenCV rule: column side only; mutual: + value-only rows),
    # fused = the packed-key MFMA kernel, valu = the popcount kernel
    runs = [(f"{path}_{name}", path, xc, md) for path in ("key", "mfma", "fused", "valu")
            for name, xc, md in (("opencv_lt26", 2, 26), ("mutual", 1, -1))]
    for name, path, xc, md in runs:
        os.environ["SFM_HAMMING_VALU"] = "1" if path == "valu" else "0"
        os.environ["SFM_HAMMING_PATH"] = {"fused": "fused", "mfma": "mutual"}.get(path, "")
        kw = dict(metric=sfmcore.METRIC_HAMMING, cross_check=xc, max_dist=md)
        out = ctx.match_batch(desc, n_kp, pr, **kw)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 10
        ev[0].record()
        for _ in range(reps):
            out = ctx.match_batch(desc, n_kp, pr, out=out, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        cnt, mt, dist = (t.cpu().numpy() for t in out)
        ok = True
        for p in range(0, len(pairs), max(1, len(pairs) // 10)):
            a, b = pairs[p]
            q, t, d = O.match(s["desc"][a], s["desc"][b], 1, xc, None, md)
            ok &= bool(cnt[p] == len(q) and (mt[p, :cnt[p], 0] == q).all()
                       and (mt[p, :cnt[p], 1] == t).all() and (dist[p, :cnt[p]] == d).all())
        n_dist = float(np.sum(s["n_kp"][pairs[:, 0]].astype(np.float64) * s["n_kp"][pairs[:, 1]]))
        res[name] = {"ms": ms, "pairs": len(pairs), "distances_per_s": n_dist / (ms * 1e-3),
                     "matches": int(cnt.sum()), "parity": ok}
    print(json.dumps({"n_img": n_img, "k": K, **res}))


if __name__ == "__main__":
    main()
