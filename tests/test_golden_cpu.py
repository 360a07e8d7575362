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
