"""CPU: pin the oracle to the committed golden fixtures (tests/golden/, made by make_golden.py).

skimage_fixtures.npz holds scikit-image 0.18.3's outputs (an independent implementation of the
same semantics: mutual cross check, lowest-index ties, ratio on unsquared distances, Hartley
8-point); oracle_fixtures.npz holds the oracle's own outputs (regression pin for the GPU tests).
"""
import json
import os

import numpy as np
import pytest

import oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def sk():
    return dict(np.load(os.path.join(G, "skimage_fixtures.npz")))


@pytest.fixture(scope="module")
def orc():
    return dict(np.load(os.path.join(G, "oracle_fixtures.npz")))


def _pairs(q, t):
    return np.stack([q, t], 1).astype(np.int64)


@pytest.mark.parametrize("key,xc,ratio,md", [("l2_mutual_r08", 1, (4, 5), -1),
                                             ("l2_none_r08", 0, (4, 5), -1),
                                             ("l2_mutual", 1, None, -1),
                                             ("l2_mutual_maxd180", 1, (4, 5), 180 * 180)])
def test_l2_semantics_vs_skimage(sk, key, xc, ratio, md):
    if key == "l2_mutual_maxd180":
        ratio = None
    q, t, _ = O.match(sk["l2_A"], sk["l2_B"], 0, xc, ratio, md)
    np.testing.assert_array_equal(_pairs(q, t), sk["expect_" + key].astype(np.int64))


@pytest.mark.parametrize("key,md", [("ham_mutual", -1), ("ham_mutual_max26", 26)])
def test_hamming_semantics_vs_skimage(sk, key, md):
    q, t, _ = O.match(sk["ham_A"], sk["ham_B"], 1, 1, None, md)
    np.testing.assert_array_equal(_pairs(q, t), sk["expect_" + key].astype(np.int64))


def test_eight_point_vs_skimage(sk):
    x1, x2 = sk["f_x1"], sk["f_x2"]
    n1, cx1, cy1, s1 = O.normalize(x1)
    n2, cx2, cy2, s2 = O.normalize(x2)
    ok, Fn = O.fit_f8(n1, n2)
    assert ok == 0
    T1 = np.array([[s1, 0, -s1 * cx1], [0, s1, -s1 * cy1], [0, 0, 1.0]])
    T2 = np.array([[s2, 0, -s2 * cx2], [0, s2, -s2 * cy2], [0, 0, 1.0]])
    F = T2.T @ Fn.astype(np.float64).reshape(3, 3) @ T1
    F /= np.linalg.norm(F)
    E = sk["expect_F_8pt"] / np.linalg.norm(sk["expect_F_8pt"])
    assert min(np.abs(F - E).max(), np.abs(F + E).max()) < 1e-4


def test_oracle_regression_pin(orc):
    meta = json.loads(bytes(orc["meta"]).decode())
    desc, kps, n_kp, pairs = orc["scene_desc"], orc["scene_kps"], orc["scene_n_kp"], orc["scene_pairs"]
    for p, (a, b) in enumerate(pairs):
        q, t, d = O.match(desc[a][:n_kp[a]], desc[b][:n_kp[b]], 0, meta["cross_check"],
                          tuple(meta["ratio"]))
        np.testing.assert_array_equal(np.stack([q, t], 1), orc[f"pair{p}_match"])
        np.testing.assert_array_equal(d, orc[f"pair{p}_dist"])
        r = O.ransac_f(kps[a][q], kps[b][t], H=meta["n_hyp"], seed=meta["seed"], pa=int(a),
                       pb=int(b), thr=meta["thr"])
        assert r["count"] == orc[f"pair{p}_count"]
        assert r["best_h"] == orc[f"pair{p}_best_h"]
        np.testing.assert_array_equal(r["mask"], orc[f"pair{p}_mask"])
        np.testing.assert_array_equal(r["F"].view(np.uint32), orc[f"pair{p}_F_bits"])
    q, t, d = O.match(orc["orb_desc"][0], orc["orb_desc"][1], 1, 2, None, 26)
    np.testing.assert_array_equal(np.stack([q, t], 1), orc["orb_match"])
    np.testing.assert_array_equal(d, orc["orb_dist"])


# ---- per-hypothesis 8-point F vs scikit-image (tests/golden/skimage_ransac_fixtures.npz) ----------
F_TOL, F_TOL_ILL, COND_MIN = 1e-4, 1e-3, 5e-3


def pixel_frame_F(Fn, norm):
    """F of the normalised frame (9 f32) -> unit-norm pixel-frame F (T2^T F T1)."""
    cx1, cy1, s1, cx2, cy2, s2 = (float(v) for v in norm)
    T1 = np.array([[s1, 0, -s1 * cx1], [0, s1, -s1 * cy1], [0, 0, 1.0]])
    T2 = np.array([[s2, 0, -s2 * cx2], [0, s2, -s2 * cy2], [0, 0, 1.0]])
    F = T2.T @ np.asarray(Fn, np.float64).reshape(3, 3) @ T1
    return F / np.linalg.norm(F)


def check_hypotheses_vs_skimage(fx, i, F_norm_frame, masks, norm):
    """Shared by the CPU (oracle) and GPU tests: every hypothesis's F within F_TOL of skimage's
    (up to sign; F_TOL_ILL where the 8x9 system's sigma_8/sigma_1 < COND_MIN), and identical
    inlier decisions except within the stated band |res^2/thr - 1| < band."""
    M = fx[f"p{i}_x1"].shape[0]
    E = fx[f"p{i}_expect_F"]
    cond = fx[f"p{i}_expect_cond"]
    err = np.array([min(np.abs(pixel_frame_F(F_norm_frame[h], norm) - E[h].reshape(3, 3)).max(),
                        np.abs(pixel_frame_F(F_norm_frame[h], norm) + E[h].reshape(3, 3)).max())
                    for h in range(E.shape[0])])
    well = cond >= COND_MIN
    assert err[well].max() < F_TOL, (i, err[well].max())
    assert err.max() < F_TOL_ILL, (i, err.max())
    exp = np.unpackbits(fx[f"p{i}_expect_mask"], axis=1)[:, :M].astype(bool)
    band = np.unpackbits(fx[f"p{i}_band"], axis=1)[:, :M].astype(bool)
    diff = (np.asarray(masks)[:, :M].astype(bool) != exp)
    assert not (diff & ~band).any(), (i, np.argwhere(diff & ~band)[:5])
    return int(well.sum()), int(diff.sum())


def test_ransac_hypotheses_vs_skimage():
    fx = dict(np.load(os.path.join(G, "skimage_ransac_fixtures.npz")))
    H = fx["p0_expect_F"].shape[0]
    for i, (a, b) in enumerate(fx["pairs"]):
        x1, x2 = fx[f"p{i}_x1"], fx[f"p{i}_x2"]
        n1, cx1, cy1, s1 = O.normalize(x1)
        n2, cx2, cy2, s2 = O.normalize(x2)
        norm = np.array([cx1, cy1, s1, cx2, cy2, s2], np.float32)
        np.testing.assert_array_equal(norm.view(np.uint32), fx[f"p{i}_norm"].view(np.uint32))
        masks, idx, ok = O.ransac_masks(x1, x2, H=H, seed=42, pa=int(a), pb=int(b), thr=1.0)
        np.testing.assert_array_equal(idx, fx[f"p{i}_idx"])
        Fn = np.stack([O.fit_f8(n1[ix], n2[ix])[1] for ix in idx])
        check_hypotheses_vs_skimage(fx, i, Fn, masks, norm)


# ---- the reference's own crossCheck rule against third-party NN tables -------
def opencv_crosscheck_from_tables(train_nn, train_d, n_query, max_d=None):
    """OpenCV's BFMatcher(crossCheck=True) update loop (code/feature_matching.py:48; batchDistance's
    per-train pass, ascending train, strict <) applied to a train -> nearest-query table computed
    by scikit-image (`train_nn` rows (train, query), `train_d` its distances).  Returns [m, 2]
    (query, train) rows in ascending query order and their distances."""
    best = np.full(n_query, np.inf)
    part = np.full(n_query, -1, np.int64)
    for (t, q), d in zip(np.asarray(train_nn), np.asarray(train_d)):
        if d < best[q]:
            best[q], part[q] = d, t
    keep = part >= 0
    if max_d is not None:
        keep &= best < max_d
    q = np.nonzero(keep)[0]
    return np.stack([q, part[q]], 1), best[q]


def xc_expectations():
    """(kind, direction, max_d) -> (descriptors X, Y, expected rows, expected integer distances)
    from tests/golden/skimage_xc_fixtures.npz: the forward (X = A) result uses the trains' table
    `ba`, the reverse (X = B) result the table `ab`."""
    sk = np.load(os.path.join(G, "skimage_xc_fixtures.npz"))
    out = {}
    for kind in ("l2", "ham"):
        A, B = sk[kind + "_A"], sk[kind + "_B"]
        for direc, X, Y, tab in (("fwd", A, B, "ba"), ("rev", B, A, "ab")):
            d = sk[f"sk_{kind}_{tab}_d"]
            dint = np.rint(d * d if kind == "l2" else d).astype(np.int64)   # d^2 resp. bits
            for md in ((None, 26) if kind == "ham" else (None, 60000)):
                rows, bd = opencv_crosscheck_from_tables(sk[f"sk_{kind}_{tab}_nn"], dint,
                                                         len(X), md)
                out[(kind, direc, md)] = (X, Y, rows, bd.astype(np.int64))
    return out


def test_oracle_opencv_rule_equals_loop_on_skimage_tables():
    """The oracle's OpenCV cross-check (oracle/sfm_oracle.c cross_check 2) equals OpenCV's update
    loop run on scikit-image's NN tables, on tie-heavy L2 and Hamming sets, both directions."""
    for (kind, direc, md), (X, Y, rows, bd) in xc_expectations().items():
        q, t, d = O.match(X, Y, metric=0 if kind == "l2" else 1, cross_check=O.XC_OPENCV,
                          max_dist=-1 if md is None else md)
        np.testing.assert_array_equal(np.stack([q, t], 1), rows, err_msg=str((kind, direc, md)))
        np.testing.assert_array_equal(np.asarray(d, np.int64), bd)


def test_skimage_xc_fixtures_are_tie_heavy():
    sk = np.load(os.path.join(G, "skimage_xc_fixtures.npz"))
    for kind in ("l2", "ham"):
        for tab in ("ab", "ba"):
            nn = sk[f"sk_{kind}_{tab}_nn"]
            # many trains share a nearest query: the loop's lowest-index / strict-< order matters
            assert len(np.unique(nn[:, 1])) < len(nn)
    ham = np.load(os.path.join(G, "skimage_xc_fixtures.npz"))["sk_ham_ab_d"]
    assert (np.diff(np.sort(ham)) == 0).mean() > 0.5
