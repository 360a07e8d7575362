"""Interleaved A/B of K1's mutual-rule kernels (SFM_K1_GRP=0: round 4's top-2 rows + transpose;
1: round 5's group-max rows + LDS column reduction + finalize recheck) on cfg3 (50 x 2048, 1225
pairs) and a cfg4 slice (500 x 4096 scene, PAIRS pairs): ms per launch with HIP events, and
bitwise equality of the two variants' outputs.  Usage: python tests/perf/k1_grp_ab.py [ROUNDS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]

import numpy as np
import torch

import sfmcore
import synth


def timed(ctx, desc, n_kp, pr, reps, out=None):
    out = ctx.match_batch(desc, n_kp, pr, cross_check=1, ratio=(4, 5), out=out)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        out = ctx.match_batch(desc, n_kp, pr, cross_check=1, ratio=(4, 5), out=out)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps, out


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    cases = []
    s3 = synth.make_scene(50, 2048, seed=0)
    p3 = synth.unordered_pairs(50)
    cases.append(("cfg3", T(s3["desc"]), T(s3["n_kp"]), T(p3), 10, s3["n_kp"], p3))
    n4 = int(os.environ.get("PAIRS", "8000"))
    s4 = synth.make_scene(500, 4096, seed=0)
    p4 = synth.unordered_pairs(500)
    p4 = p4[:: max(1, len(p4) // n4)][:n4]
    cases.append((f"cfg4[{len(p4)}]", T(s4["desc"]), T(s4["n_kp"]), T(p4), 3, s4["n_kp"], p4))
    for name, desc, n_kp, pr, reps, nk, pairs in cases:
        ops = 2.0 * 128 * float(np.sum(nk[pairs[:, 0]].astype(np.float64) * nk[pairs[:, 1]]))
        res = {}
        for r in range(rounds):
            for v in ("0", "1"):
                os.environ["SFM_K1_GRP"] = v
                ms, out = timed(ctx, desc, n_kp, pr, reps)
                res.setdefault(v, []).append(ms)
                if r == 0:
                    res["out" + v] = [t.cpu().numpy() for t in out]
        c0, m0, d0 = res["out0"]
        c1, m1, d1 = res["out1"]
        same = bool((c0 == c1).all()) and all(
            (m0[p, :c0[p]] == m1[p, :c1[p]]).all() and (d0[p, :c0[p]] == d1[p, :c1[p]]).all()
            for p in range(len(c0)))
        for v in ("0", "1"):
            ms = float(np.median(res[v]))
            print(f"{name} SFM_K1_GRP={v}: median {ms:.3f} ms/launch over {rounds} rounds "
                  f"{[round(x, 3) for x in res[v]]}  {ops / ms / 1e9:.0f} TOP/s  "
                  f"frac {ops / ms / 1e9 / 5033:.3f}", flush=True)
        print(f"{name}: outputs bit-identical between variants: {same}  matches={int(c1.sum())}",
              flush=True)


if __name__ == "__main__":
    main()
