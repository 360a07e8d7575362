"""GPU vs the committed golden vectors (tests/golden/oracle_fixtures.npz): no oracle at run time."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def test_gpu_matches_golden_vectors(ctx):
    import torch
    f = dict(np.load(os.path.join(G, "oracle_fixtures.npz")))
    meta = json.loads(bytes(f["meta"]).decode())
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    pairs = f["scene_pairs"]
    cnt, mt, dist = ctx.match_batch(T(f["scene_desc"]), T(f["scene_n_kp"]), T(pairs),
                                    cross_check=meta["cross_check"], ratio=tuple(meta["ratio"]))
    rs = ctx.ransac_batch(T(f["scene_kps"]), T(pairs), cnt, mt, n_hyp=meta["n_hyp"],
                          seed=meta["seed"], thr=meta["thr"])
    torch.cuda.synchronize()
    cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
    rs = {k: v.cpu().numpy() for k, v in rs.items()}
    for p in range(len(pairs)):
        exp = f[f"pair{p}_match"]
        assert cnt[p] == len(exp)
        np.testing.assert_array_equal(mt[p, :cnt[p]], exp)
        np.testing.assert_array_equal(dist[p, :cnt[p]], f[f"pair{p}_dist"])
        assert rs["inl_count"][p] == f[f"pair{p}_count"]
        assert rs["best_h"][p] == f[f"pair{p}_best_h"]
        np.testing.assert_array_equal(rs["mask"][p, :cnt[p]], f[f"pair{p}_mask"])
        np.testing.assert_array_equal(rs["F"][p].view(np.uint32), f[f"pair{p}_F_bits"])
        np.testing.assert_array_equal(rs["norm"][p].view(np.uint32), f[f"pair{p}_norm_bits"])
    od = f["orb_desc"]
    c2, m2, d2 = ctx.match_batch(T(od), T(np.array([od.shape[1]] * 2, np.int32)),
                                 T(np.array([[0, 1]], np.int32)), metric=1, cross_check=2,
                                 max_dist=26)
    torch.cuda.synchronize()
    k = int(c2.cpu()[0])
    np.testing.assert_array_equal(m2.cpu().numpy()[0, :k], f["orb_match"])
    np.testing.assert_array_equal(d2.cpu().numpy()[0, :k], f["orb_dist"])


# ---- the GPU directly on scikit-image's vectors (tests/golden/skimage_fixtures.npz) -------------
SK_L2 = [("l2_mutual_r08", 1, (4, 5), -1), ("l2_none_r08", 0, (4, 5), -1), ("l2_mutual", 1, None, -1),
         ("l2_mutual_maxd180", 1, None, 180 * 180)]  # L2 max_dist on d^2: d < 180 <=> d^2 < 32400
SK_HAM = [("ham_mutual", -1), ("ham_mutual_max26", 26)]  # d < 25.5/256 of the bits <=> d < 26


def _gpu_pair(ctx, A, B, **kw):
    import torch
    k = max(A.shape[0], B.shape[0])
    desc = np.zeros((2, k, A.shape[1]), np.uint8)
    desc[0, :A.shape[0]] = A
    desc[1, :B.shape[0]] = B
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    cnt, mt, _ = ctx.match_batch(T(desc), T(np.array([A.shape[0], B.shape[0]], np.int32)),
                                 T(np.array([[0, 1]], np.int32)), **kw)
    torch.cuda.synchronize()
    n = int(cnt.cpu()[0])
    return mt.cpu().numpy()[0, :n].astype(np.int64)


@pytest.mark.parametrize("key,xc,ratio,md", SK_L2)
def test_gpu_l2_vs_skimage(ctx, key, xc, ratio, md):
    sk = np.load(os.path.join(G, "skimage_fixtures.npz"))
    got = _gpu_pair(ctx, sk["l2_A"], sk["l2_B"], metric=0, cross_check=xc, ratio=ratio,
                    max_dist=md)
    np.testing.assert_array_equal(got, sk["expect_" + key].astype(np.int64))


@pytest.mark.parametrize("key,md", SK_HAM)
def test_gpu_hamming_vs_skimage(ctx, key, md):
    sk = np.load(os.path.join(G, "skimage_fixtures.npz"))
    got = _gpu_pair(ctx, sk["ham_A"], sk["ham_B"], metric=1, cross_check=1, max_dist=md)
    np.testing.assert_array_equal(got, sk["expect_" + key].astype(np.int64))


def test_gpu_ransac_hypotheses_vs_skimage(ctx):
    """Every hypothesis of 4 noisy cfg3 pairs (256 each, the GPU's own Philox samples): F within
    1e-4 of scikit-image's FundamentalMatrixTransform (1e-3 for the ill-conditioned 8x9 systems),
    identical inlier decisions outside the stated band (test_golden_cpu.check_hypotheses_vs_skimage)."""
    import torch
    from test_golden_cpu import check_hypotheses_vs_skimage
    fx = dict(np.load(os.path.join(G, "skimage_ransac_fixtures.npz")))
    pairs = fx["pairs"].astype(np.int32)
    Ms = [fx[f"p{i}_x1"].shape[0] for i in range(len(pairs))]
    k_max = max(Ms)
    kps = np.zeros((int(pairs.max()) + 1, k_max, 2), np.float32)
    match = np.zeros((len(pairs), k_max, 2), np.int32)
    for i, (a, b) in enumerate(pairs):
        kps[a, :Ms[i]] = fx[f"p{i}_x1"]
        kps[b, :Ms[i]] = fx[f"p{i}_x2"]
        match[i, :Ms[i]] = np.arange(Ms[i])[:, None]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    H = fx["p0_expect_F"].shape[0]
    counts, norm, F, mk = ctx.ransac_counts(T(kps), T(pairs), T(np.array(Ms, np.int32)), T(match),
                                            n_hyp=H, seed=int(fx["seed"]), thr=float(fx["thr"]),
                                            hyp_F=True, hyp_mask=True)
    torch.cuda.synchronize()
    counts, norm, F, mk = (t.cpu().numpy() for t in (counts, norm, F, mk))
    for i in range(len(pairs)):
        np.testing.assert_array_equal(norm[i].view(np.uint32), fx[f"p{i}_norm"].view(np.uint32))
        ok = counts[i] >= 0  # -1: degenerate sample
        np.testing.assert_array_equal(mk[i][ok, :Ms[i]].sum(1), counts[i][ok])
        check_hypotheses_vs_skimage(fx, i, F[i], mk[i], norm[i])


def test_gpu_opencv_rule_vs_skimage_nn_tables(ctx):
    """the reference's BFMatcher(crossCheck=True) rule on the GPU against
    OpenCV's update loop applied to scikit-image's nearest-neighbour tables (both directions, tie-
    heavy L2 and Hamming, with and without the reference's `< 26` cut), through sfm_match_batch
    and through the one-tile sfm_match_batch_both."""
    import torch
    from test_golden_cpu import xc_expectations
    exp = xc_expectations()
    for (kind, direc, md), (X, Y, rows, bd) in exp.items():
        metric = 0 if kind == "l2" else 1
        mdi = -1 if md is None else md
        got = _gpu_pair(ctx, X, Y, metric=metric, cross_check=2, max_dist=mdi)
        np.testing.assert_array_equal(got, rows.astype(np.int64), err_msg=str((kind, direc, md)))
    # both orders from one tile: forward = (A, B), reverse = (B, A)
    for kind in ("l2", "ham"):
        for md in ((None, 26) if kind == "ham" else (None, 60000)):
            A, B = exp[(kind, "fwd", md)][0], exp[(kind, "fwd", md)][1]
            k = max(len(A), len(B))
            desc = np.zeros((2, k, A.shape[1]), np.uint8)
            desc[0, :len(A)], desc[1, :len(B)] = A, B
            T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
            cnt, mt, dist = ctx.match_batch_both(
                T(desc), T(np.array([len(A), len(B)], np.int32)), T(np.array([[0, 1]], np.int32)),
                metric=0 if kind == "l2" else 1, cross_check=2, max_dist=-1 if md is None else md)
            torch.cuda.synchronize()
            cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
            for slot, direc in ((0, "fwd"), (1, "rev")):
                _, _, rows, bd = exp[(kind, direc, md)]
                n = int(cnt[slot])
                np.testing.assert_array_equal(mt[slot, :n], rows, err_msg=str((kind, direc, md)))
                np.testing.assert_array_equal(dist[slot, :n], bd)
