"""Generates the committed golden fixtures under tests/golden/ (run in this container only).

1. skimage_fixtures.npz — the oracle's matching / 8-point semantics cross-checked against an
   independent third-party implementation: scikit-image 0.18.3 (`/opt/conda/bin/python3.9`;
   skimage/feature/match.py `match_descriptors`, skimage/transform/_geometric.py
   `FundamentalMatrixTransform`).  The reference itself cannot run here (no cv2),
   so these pin the SEMANTICS (mutual cross check, lowest-index ties, Lowe ratio on unsquared
   distances, Hartley 8-point + rank 2), not the reference's outputs: parity stays "unpinned".
2. skimage_ransac_fixtures.npz — 4 noisy cfg3 pairs x 256 hypotheses: the sampled indices (the
   build's Philox sampler), scikit-image's 8-point F and Sampson decisions per hypothesis.
3. oracle_fixtures.npz — inputs and the CPU oracle's outputs (match lists, RANSAC winner, inlier
   mask, F bits) for small seeded cases; the GPU tests compare against these stored vectors.
4. skimage_xc_fixtures.npz — tie-heavy L2 and Hamming descriptor sets with scikit-image's
   nearest-neighbour tables in BOTH directions (match_descriptors(cross_check=False) on (A, B) and
   on (B, A)) and scipy's distances of those neighbours (scipy.spatial.distance.cdist).  The tests
   apply OpenCV's crossCheck update loop to these third-party tables, so the reference's own rule
   (BFMatcher(crossCheck=True), code/feature_matching.py:48) is pinned with only its loop restated.

Usage:  python tests/golden/make_golden.py      (system python 3.10; calls python3.9 for skimage)
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]

SKIMAGE_PY = "/opt/conda/bin/python3.9"

SKIMAGE_SCRIPT = r"""
import sys, numpy as np
from skimage.feature import match_descriptors
from skimage.transform import FundamentalMatrixTransform
d = np.load(sys.argv[1])
out = {}
A, B = d["l2_A"].astype(np.float64), d["l2_B"].astype(np.float64)
out["l2_mutual_r08"] = match_descriptors(A, B, metric="euclidean", cross_check=True, max_ratio=0.8)
out["l2_none_r08"] = match_descriptors(A, B, metric="euclidean", cross_check=False, max_ratio=0.8)
out["l2_mutual"] = match_descriptors(A, B, metric="euclidean", cross_check=True)
out["l2_mutual_maxd180"] = match_descriptors(A, B, metric="euclidean", cross_check=True,
                                             max_distance=180.0)
ha = np.unpackbits(d["ham_A"], axis=1).astype(bool)
hb = np.unpackbits(d["ham_B"], axis=1).astype(bool)
out["ham_mutual"] = match_descriptors(ha, hb, metric="hamming", cross_check=True)
out["ham_mutual_max26"] = match_descriptors(ha, hb, metric="hamming", cross_check=True,
                                            max_distance=25.5 / 256)
t = FundamentalMatrixTransform()
assert t.estimate(d["f_x1"], d["f_x2"])
out["F_8pt"] = t.params
np.savez(sys.argv[2], **{k: np.asarray(v) for k, v in out.items()})
"""


def skimage_fixtures():
    import synth
    s = synth.make_scene(2, 400, seed=101)
    A, B = s["desc"][0][:300], s["desc"][1][:280].copy()
    B[7] = B[9]  # exact tie among trains
    h = synth.make_scene(2, 300, seed=102, orb=True)
    # exact two-view geometry for the 8-point estimator
    g = synth.make_scene(2, 100, seed=103, noise_px=0.0, misplace_frac=0.0, inlier_frac=1.0)
    pid = g["point_ids"]
    common = np.intersect1d(pid[0][pid[0] >= 0], pid[1][pid[1] >= 0])[:8]
    i0 = [int(np.nonzero(pid[0] == c)[0][0]) for c in common]
    i1 = [int(np.nonzero(pid[1] == c)[0][0]) for c in common]
    inputs = dict(l2_A=A, l2_B=B, ham_A=h["desc"][0], ham_B=h["desc"][1],
                  f_x1=g["kps"][0][i0].astype(np.float64), f_x2=g["kps"][1][i1].astype(np.float64))
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.npz"), os.path.join(td, "out.npz")
        np.savez(fi, **inputs)
        subprocess.run([SKIMAGE_PY, "-c", SKIMAGE_SCRIPT, fi, fo], check=True,
                       stderr=subprocess.DEVNULL)
        outs = dict(np.load(fo))
    np.savez_compressed(os.path.join(HERE, "skimage_fixtures.npz"), **inputs,
                        **{"expect_" + k: v for k, v in outs.items()})
    return {k: v.shape for k, v in outs.items()}


# Per-hypothesis 8-point estimates of scikit-image's FundamentalMatrixTransform on the same
# samples the build's Philox sampler draws.  skimage normalises each 8-point sample on its own
# (RMS variant of Hartley); the build normalises once per pair (mean-distance variant, DESIGN
# 4.2).  The 8x9 null space (F before the rank-2 step) does not depend on the normalisation, but
# the rank-2 truncation does, so skimage's _center_and_normalize_points is given the build's
# pair-level transform for the estimate: the comparison is of the arithmetic (null space + rank
# 2), in the same frame.  Residuals are skimage's own Sampson distances in pixels.
SKIMAGE_RANSAC_SCRIPT = r"""
import sys, numpy as np
from skimage.transform import _geometric as g
from skimage.transform import FundamentalMatrixTransform
d = np.load(sys.argv[1]); out = {}
for i in range(int(d["n_pairs"])):
    x1 = d[f"p{i}_x1"].astype(np.float64); x2 = d[f"p{i}_x2"].astype(np.float64)
    nm = d[f"p{i}_norm"].astype(np.float64)
    mk = lambda cx, cy, s: np.array([[s, 0, -s * cx], [0, s, -s * cy], [0, 0, 1.0]])
    T = {"src": mk(*nm[:3]), "dst": mk(*nm[3:])}
    Fs, R, C = [], [], []
    orig = g._center_and_normalize_points
    for ix in d[f"p{i}_idx"]:
        seq = iter(["src", "dst"])
        def pair_frame(points, _seq=seq):
            m = T[next(_seq)]
            return m, (m @ np.row_stack([points.T, np.ones(points.shape[0])])).T[:, :2]
        g._center_and_normalize_points = pair_frame
        t = FundamentalMatrixTransform()
        assert t.estimate(x1[ix], x2[ix])
        g._center_and_normalize_points = orig
        Fs.append((t.params / np.linalg.norm(t.params)).ravel())
        R.append(t.residuals(x1, x2))
        n1 = (T["src"] @ np.row_stack([x1[ix].T, np.ones(8)])).T
        n2 = (T["dst"] @ np.row_stack([x2[ix].T, np.ones(8)])).T
        A = np.ones((8, 9)); A[:, :2] = n1[:, :2]; A[:, :3] *= n2[:, 0:1]
        A[:, 3:5] = n1[:, :2]; A[:, 3:6] *= n2[:, 1:2]; A[:, 6:8] = n1[:, :2]
        sv = np.linalg.svd(A, compute_uv=False)
        C.append(sv[-1] / sv[0])
    out[f"p{i}_F"] = np.array(Fs); out[f"p{i}_res2"] = np.array(R) ** 2; out[f"p{i}_cond"] = np.array(C)
np.savez(sys.argv[2], **out)
"""
SKIMAGE_XC_SCRIPT = r"""
import sys, numpy as np
from scipy.spatial.distance import cdist
from skimage.feature import match_descriptors
d = np.load(sys.argv[1]); out = {}
for kind in ("l2", "ham"):
    A, B = d[kind + "_A"], d[kind + "_B"]
    if kind == "l2":
        A, B, metric = A.astype(np.float64), B.astype(np.float64), "euclidean"
    else:
        A, B, metric = np.unpackbits(A, axis=1).astype(bool), np.unpackbits(B, axis=1).astype(bool), "hamming"
    for tag, X, Y in (("ab", A, B), ("ba", B, A)):
        nn = match_descriptors(X, Y, metric=metric, cross_check=False)   # (query, its NN), every query
        dd = cdist(X[nn[:, 0]], Y[nn[:, 1]], metric=metric).diagonal()
        out[f"{kind}_{tag}_nn"] = nn
        out[f"{kind}_{tag}_d"] = dd * (256 if kind == "ham" else 1)
np.savez(sys.argv[2], **out)
"""


def skimage_xc_fixtures():
    """Tie-heavy descriptor sets + scikit-image NN tables both ways (module docstring, item 4)."""
    import synth
    rng = np.random.Generator(np.random.PCG64(301))
    s = synth.make_scene(2, 400, seed=302)
    A, B = s["desc"][0][:330].copy(), s["desc"][1][:310].copy()
    B[20:25] = B[30]          # five identical trains: ties in every query's row
    A[50:54] = A[60]          # four identical queries: ties in the column direction
    A[100] = B[200]           # an exact zero distance
    pool = rng.integers(0, 256, size=(40, 32), dtype=np.uint8)     # Hamming: 40 bases, 0-2 flips
    def draw(n):
        x = pool[rng.integers(0, 40, size=n)].copy()
        for r in range(n):
            for _ in range(int(rng.integers(0, 3))):
                bit = int(rng.integers(0, 256))
                x[r, bit // 8] ^= np.uint8(1 << (bit % 8))
        return x
    inputs = dict(l2_A=A, l2_B=B, ham_A=draw(300), ham_B=draw(280))
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.npz"), os.path.join(td, "out.npz")
        np.savez(fi, **inputs)
        subprocess.run([SKIMAGE_PY, "-c", SKIMAGE_XC_SCRIPT, fi, fo], check=True,
                       stderr=subprocess.DEVNULL)
        outs = dict(np.load(fo))
    np.savez_compressed(os.path.join(HERE, "skimage_xc_fixtures.npz"), **inputs,
                        **{"sk_" + k: v for k, v in outs.items()})
    return {k: v.shape for k, v in outs.items()}


RANSAC_PAIRS = [(0, 1), (5, 6), (12, 30), (40, 41)]  # cfg3 scene (50 x 2048, seed 0)
RANSAC_H = 256
RANSAC_BAND = 1e-5  # decisions may differ only where |res^2 / thr - 1| < RANSAC_BAND


def skimage_ransac_fixtures():
    import oracle as O
    import synth
    s = synth.make_scene(50, 2048, seed=0)
    inp = {"n_pairs": np.int32(len(RANSAC_PAIRS)), "pairs": np.array(RANSAC_PAIRS, np.int32),
           "seed": np.uint64(42), "thr": np.float32(1.0), "band": np.float64(RANSAC_BAND)}
    for i, (a, b) in enumerate(RANSAC_PAIRS):
        q, t, _ = O.match(s["desc"][a], s["desc"][b], 0, 1, (4, 5))   # the bench rule's matches
        x1 = s["kps"][a][q].astype(np.float32)
        x2 = s["kps"][b][t].astype(np.float32)
        _, cx1, cy1, s1 = O.normalize(x1)
        _, cx2, cy2, s2 = O.normalize(x2)
        inp[f"p{i}_x1"], inp[f"p{i}_x2"] = x1, x2
        inp[f"p{i}_norm"] = np.array([cx1, cy1, s1, cx2, cy2, s2], np.float32)
        inp[f"p{i}_idx"] = np.stack([O.sample8(42, a, b, h, len(q)) for h in range(RANSAC_H)])
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.npz"), os.path.join(td, "out.npz")
        np.savez(fi, **inp)
        subprocess.run([SKIMAGE_PY, "-c", SKIMAGE_RANSAC_SCRIPT, fi, fo], check=True,
                       stderr=subprocess.DEVNULL)
        out = dict(np.load(fo))
    fx = dict(inp)
    for i in range(len(RANSAC_PAIRS)):
        r2 = out[f"p{i}_res2"] / 1.0
        fx[f"p{i}_expect_F"] = out[f"p{i}_F"]
        fx[f"p{i}_expect_cond"] = out[f"p{i}_cond"]
        fx[f"p{i}_expect_mask"] = np.packbits(r2 < 1.0, axis=1)
        fx[f"p{i}_band"] = np.packbits(np.abs(r2 - 1.0) < RANSAC_BAND, axis=1)
    np.savez_compressed(os.path.join(HERE, "skimage_ransac_fixtures.npz"), **fx)
    return sum(v.nbytes for v in fx.values())


def oracle_fixtures():
    import oracle as O
    import synth
    fx = {}
    # L2 matching + RANSAC on two small seeded pairs (ragged second image)
    s = synth.make_scene(3, 512, seed=201)
    n_kp = np.array([512, 437, 512], np.int32)
    fx["scene_desc"] = s["desc"]
    fx["scene_kps"] = s["kps"]
    fx["scene_n_kp"] = n_kp
    pairs = np.array([[0, 1], [1, 2], [2, 0]], np.int32)
    fx["scene_pairs"] = pairs
    meta = dict(ratio=[4, 5], cross_check=1, n_hyp=512, seed=42, thr=1.0)
    for p, (a, b) in enumerate(pairs):
        q, t, d = O.match(s["desc"][a][:n_kp[a]], s["desc"][b][:n_kp[b]], 0, 1, (4, 5))
        fx[f"pair{p}_match"] = np.stack([q, t], 1).astype(np.int32)
        fx[f"pair{p}_dist"] = d.astype(np.int32)
        r = O.ransac_f(s["kps"][a][q], s["kps"][b][t], H=512, seed=42, pa=int(a), pb=int(b),
                       thr=1.0)
        fx[f"pair{p}_count"] = np.int32(r["count"])
        fx[f"pair{p}_best_h"] = np.int32(r["best_h"])
        fx[f"pair{p}_mask"] = r["mask"]
        fx[f"pair{p}_F_bits"] = r["F"].view(np.uint32)
        fx[f"pair{p}_norm_bits"] = r["norm"].view(np.uint32)
    # the reference's own matcher: ORB Hamming, OpenCV crossCheck rule, distance < 26
    o = synth.make_scene(2, 500, seed=202, orb=True)
    fx["orb_desc"] = o["desc"]
    q, t, d = O.match(o["desc"][0], o["desc"][1], 1, 2, None, 26)
    fx["orb_match"] = np.stack([q, t], 1).astype(np.int32)
    fx["orb_dist"] = d.astype(np.int32)
    fx["meta"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "oracle_fixtures.npz"), **fx)
    return len(fx)


if __name__ == "__main__":
    print("skimage:", skimage_fixtures())
    print("skimage ransac bytes:", skimage_ransac_fixtures())
    print("oracle entries:", oracle_fixtures())
    print("skimage crossCheck tables:", skimage_xc_fixtures())
