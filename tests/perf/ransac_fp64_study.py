"""K2 precision study: the f32 RANSAC spec (oracle/sfm_oracle.c == the GPU
kernels, bit for bit) against an fp64 evaluation of the SAME hypotheses on every cfg3 pair.

Per pair (50 images x 2048, all 1225 pairs, mutual + ratio 4/5 matches, H = 4096, seed 42, Sampson
1 px^2): the f32 spec's per-hypothesis inlier masks come from oracle.ransac_masks; the fp64
evaluation takes the same 8-point samples, Hartley-normalises in fp64, takes the null vector of
the 8 x 9 system and the rank-2 projection by SVD (numpy, fp64) and tests the Sampson error in
pixels exactly (r^2 < thr (s2^2 |F x1|_{01}^2 + s1^2 |F^T x2|_{01}^2) in normalised coordinates).
Reported: the fraction of (hypothesis, match) decisions that differ, pairs whose winner (max
count, lowest h) or winning count differs, verified-status flips (count >= 15) and the change in
the total of verified matches.  CPU only.  Usage: python tests/perf/ransac_fp64_study.py [out.json]
"""
import json
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]

import numpy as np

H, SEED, THR, MIN_INL = 4096, 42, 1.0, 15
_scene = None


def _init():
    global _scene
    import synth
    _scene = synth.make_scene(50, 2048, seed=0)


def _hartley(xy):
    c = xy.mean(axis=0)
    mean = np.sqrt(((xy - c) ** 2).sum(axis=1)).mean()
    s = np.sqrt(2.0) / mean if mean > 0 else 1.0
    return (xy - c) * s, s


def _pair(ab):
    import oracle as O
    a, b = ab
    s = _scene
    q, t, _ = O.match(s["desc"][a], s["desc"][b], 0, O.XC_MUTUAL, (4, 5))
    M = len(q)
    out = dict(pair=[int(a), int(b)], M=M)
    if M < 8:
        return out
    xy1 = s["kps"][a][q].astype(np.float32)
    xy2 = s["kps"][b][t].astype(np.float32)
    m32, idx, ok = O.ransac_masks(xy1, xy2, H=H, seed=SEED, pa=int(a), pb=int(b), thr=THR)
    n1, s1 = _hartley(xy1.astype(np.float64))
    n2, s2 = _hartley(xy2.astype(np.float64))
    x1, y1, x2, y2 = (v[idx] for v in (n1[:, 0], n1[:, 1], n2[:, 0], n2[:, 1]))   # [H, 8]
    A = np.stack([x2 * x1, x2 * y1, x2, y2 * x1, y2 * y1, y2, x1, y1, np.ones_like(x1)], axis=2)
    _, sv, vt = np.linalg.svd(A, full_matrices=True)                          # [H, 9, 9]
    F = vt[:, -1, :].reshape(H, 3, 3)
    u, fs, fv = np.linalg.svd(F)
    fs[:, 2] = 0.0
    F = u @ (fs[:, :, None] * fv)
    ok64 = sv[:, 7] > 1e-12 * sv[:, 0]
    X1 = np.c_[n1, np.ones(M)]
    X2 = np.c_[n2, np.ones(M)]
    a_ = np.einsum("hij,mj->hmi", F, X1)        # F x1
    b_ = np.einsum("hji,mj->hmi", F, X2)        # F^T x2
    r = np.einsum("mi,hmi->hm", X2, a_)
    den = THR * (s2 ** 2 * (a_[:, :, 0] ** 2 + a_[:, :, 1] ** 2)
                 + s1 ** 2 * (b_[:, :, 0] ** 2 + b_[:, :, 1] ** 2))
    m64 = (den - r * r > 0) & ok64[:, None]
    c32 = np.where(ok, m32.sum(axis=1), -1)
    c64 = np.where(ok64, m64.sum(axis=1), -1)
    h32 = int(np.argmax(c32))                    # argmax = lowest h among the maxima
    h64 = int(np.argmax(c64))
    out.update(diff_decisions=int((m32.astype(bool) != m64).sum()), decisions=int(H * M),
               ok_diff=int((ok != ok64).sum()), h32=h32, h64=h64, c32=int(c32[h32]),
               c64=int(c64[h64]),
               winner_mask_diff=int((m32[h32].astype(bool) != m64[h64]).sum()),
               same_h_mask_diff=int((m32[h32].astype(bool) != m64[h32]).sum()),
               max_count_diff_any_h=int(np.abs(c32 - c64).max()))
    return out


def main():
    import synth
    pairs = [tuple(p) for p in synth.unordered_pairs(50)]
    t0 = time.time()
    with Pool(min(8, os.cpu_count() or 1), initializer=_init) as pool:
        res = pool.map(_pair, pairs, chunksize=8)
    res = [r for r in res if r["M"] >= 8]
    dd = sum(r["diff_decisions"] for r in res)
    nd = sum(r["decisions"] for r in res)
    v32 = sum(r["c32"] for r in res if r["c32"] >= MIN_INL)
    v64 = sum(r["c64"] for r in res if r["c64"] >= MIN_INL)
    summary = {
        "pairs": len(res), "hypotheses_per_pair": H,
        "decisions": nd, "decisions_differing": dd, "decision_diff_frac": dd / nd,
        "degenerate_flag_differs": sum(r["ok_diff"] for r in res),
        "pairs_winner_h_differs": sum(r["h32"] != r["h64"] for r in res),
        "pairs_winning_count_differs": sum(r["c32"] != r["c64"] for r in res),
        "max_winning_count_diff": max(abs(r["c32"] - r["c64"]) for r in res),
        "pairs_verified_status_flips": sum((r["c32"] >= MIN_INL) != (r["c64"] >= MIN_INL)
                                           for r in res),
        "verified_matches_f32": v32, "verified_matches_fp64": v64,
        "winner_mask_diff_total": sum(r["winner_mask_diff"] for r in res),
        "same_h_mask_diff_total": sum(r["same_h_mask_diff"] for r in res),
        "max_per_hypothesis_count_diff": max(r["max_count_diff_any_h"] for r in res),
        "wall_s": time.time() - t0,
    }
    print(json.dumps(summary, indent=1))
    if len(sys.argv) > 1:
        json.dump(dict(summary=summary, pairs=res), open(sys.argv[1], "w"))


if __name__ == "__main__":
    main()
