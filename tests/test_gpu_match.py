"""GPU parity: libsfmcore matching (K1 MFMA L2, Hamming) vs the CPU oracle, bit-exact.

Calls go through the C-ABI (sfmcore.py -> libsfmcore.so).  The oracle (oracle/sfm_oracle.c) is the
checker only.  Edge cases mirror what BFMatcher sees in the reference loop (code/pipeline.py:38-47):
empty descriptor sets, a single train, ragged per-image counts, non-multiple-of-32 sizes.
"""
import numpy as np
import pytest

import oracle as O
import sfmcore
import synth

pytestmark = pytest.mark.gpu


def _gpu_match(ctx, desc, n_kp, pairs, **kw):
    import torch
    d = torch.from_numpy(np.ascontiguousarray(desc)).cuda()
    n = torch.from_numpy(np.ascontiguousarray(n_kp, np.int32)).cuda()
    pr = torch.from_numpy(np.ascontiguousarray(pairs, np.int32)).cuda()
    cnt, mt, dist = ctx.match_batch(d, n, pr, **kw)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()


def _check_pairs(ctx, desc, n_kp, pairs, metric=0, cross_check=1, ratio=None, max_dist=-1):
    cnt, mt, dist = _gpu_match(ctx, desc, n_kp, pairs, metric=metric, cross_check=cross_check,
                               ratio=ratio, max_dist=max_dist)
    for p, (a, b) in enumerate(pairs):
        q, t, d = O.match(desc[a, :n_kp[a]], desc[b, :n_kp[b]], metric=metric,
                          cross_check=cross_check, ratio=ratio, max_dist=max_dist)
        k = cnt[p]
        assert k == len(q), f"pair {p} ({a},{b}): count {k} != oracle {len(q)}"
        np.testing.assert_array_equal(mt[p, :k, 0], q)
        np.testing.assert_array_equal(mt[p, :k, 1], t)
        np.testing.assert_array_equal(dist[p, :k], d)
    return cnt


def test_l2_small_pair_mutual_ratio(ctx):
    s = synth.make_scene(2, 512, seed=3)
    cnt = _check_pairs(ctx, s["desc"], s["n_kp"], np.array([[0, 1], [1, 0]], np.int32),
                       ratio=(4, 5))
    assert cnt[0] > 100


@pytest.mark.parametrize("xc,ratio,maxd", [(0, None, -1), (1, None, -1), (2, None, -1),
                                           (1, (4, 5), -1), (0, (3, 4), -1), (1, (4, 5), 40000),
                                           (2, None, 30000)])
def test_l2_modes(ctx, xc, ratio, maxd):
    s = synth.make_scene(4, 1000, seed=5)
    pairs = synth.unordered_pairs(4)
    _check_pairs(ctx, s["desc"], s["n_kp"], pairs, cross_check=xc, ratio=ratio, max_dist=maxd)


def test_l2_batch_2048(ctx):
    s = synth.make_scene(6, 2048, seed=7)
    pairs = synth.unordered_pairs(6)
    cnt = _check_pairs(ctx, s["desc"], s["n_kp"], pairs, ratio=(4, 5))
    assert (cnt > 300).all()


def test_l2_ragged_and_edges(ctx):
    rng = np.random.default_rng(11)
    k_max = 1100
    n_img = 6
    desc = rng.integers(0, 256, size=(n_img, k_max, 128), dtype=np.uint8)
    # duplicated descriptors force exact distance ties (lowest-index rules)
    desc[1, 5] = desc[1, 7]
    desc[2, 10:20] = desc[0, 30]
    n_kp = np.array([1100, 37, 1, 0, 2, 1025], np.int32)
    pairs = np.array([[a, b] for a in range(n_img) for b in range(n_img) if a != b], np.int32)
    for xc, ratio in [(1, (4, 5)), (0, None), (2, None), (1, None)]:
        _check_pairs(ctx, desc, n_kp, pairs, cross_check=xc, ratio=ratio)
    # the ratio path (scan units: pairs of an image without descriptors join no unit), ratio only
    # and mutual + ratio through it
    import os
    os.environ["SFM_L2_PATH"] = "fr"
    try:
        for xc in (0, 1):
            _check_pairs(ctx, desc, n_kp, pairs, cross_check=xc, ratio=(4, 5))
    finally:
        os.environ.pop("SFM_L2_PATH", None)


def test_l2_extreme_values(ctx):
    # all-0 vs all-255 descriptors: the largest possible distances (exactness of the int path)
    desc = np.zeros((2, 64, 128), np.uint8)
    desc[1, :32] = 255
    desc[0, 40:] = 255
    desc[1, 50] = 0
    n_kp = np.array([64, 64], np.int32)
    for xc in (0, 1, 2):
        _check_pairs(ctx, desc, n_kp, np.array([[0, 1], [1, 0]], np.int32), cross_check=xc)


@pytest.mark.parametrize("xc,ratio,maxd", [(2, None, 26), (1, None, 26), (0, (4, 5), -1),
                                           (2, None, -1)])
def test_hamming_reference_semantics(ctx, xc, ratio, maxd):
    s = synth.make_scene(3, 500, seed=13, orb=True)
    pairs = np.array([[0, 1], [1, 0], [0, 2], [2, 1]], np.int32)
    cnt = _check_pairs(ctx, s["desc"], s["n_kp"], pairs, metric=1, cross_check=xc, ratio=ratio,
                       max_dist=maxd)
    assert cnt.sum() > 0


def test_hamming_ragged(ctx):
    rng = np.random.default_rng(2)
    desc = rng.integers(0, 256, size=(4, 300, 32), dtype=np.uint8)
    desc[1, 3] = desc[1, 4]
    n_kp = np.array([300, 1, 0, 17], np.int32)
    pairs = np.array([[a, b] for a in range(4) for b in range(4) if a != b], np.int32)
    _check_pairs(ctx, desc, n_kp, pairs, metric=1, cross_check=2, max_dist=26)
    _check_pairs(ctx, desc, n_kp, pairs, metric=1, cross_check=1)


def test_invalid_arguments_raise(ctx):
    import torch
    d = torch.zeros((2, 8, 128), dtype=torch.uint8, device="cuda")
    n = torch.full((2,), 8, dtype=torch.int32, device="cuda")
    pr = torch.tensor([[0, 1]], dtype=torch.int32, device="cuda")
    with pytest.raises(sfmcore.SfmCoreError):
        ctx.match_batch(d, n, pr, cross_check=2, ratio=(4, 5))
    with pytest.raises(sfmcore.SfmCoreError):
        ctx.match_batch(d, n, pr, metric=1)  # Hamming needs dim 32


@pytest.mark.parametrize("K", [500, 1000, 4096])
def test_hamming_mfma_and_valu_paths_agree(ctx, K):
    """The MFMA Hamming path (bits expanded to 0/1 bytes) and the VALU popcount kernel are two
    implementations of the same matcher: outputs must be identical in every mode."""
    import os
    s = synth.make_scene(3, K, seed=40 + K, orb=True)
    n_kp = s["n_kp"].copy()
    n_kp[1] = K - 37  # ragged
    pairs = np.array([[0, 1], [1, 2], [2, 0]], np.int32)
    for xc, ratio, md in ((2, None, 26), (1, None, -1), (1, (4, 5), 40), (0, None, -1)):
        outs = []
        for v in ("0", "1"):
            os.environ["SFM_HAMMING_VALU"] = v
            try:
                outs.append(_gpu_match(ctx, s["desc"], n_kp, pairs, metric=1, cross_check=xc,
                                       ratio=ratio, max_dist=md))
            finally:
                os.environ.pop("SFM_HAMMING_VALU", None)
        c0, m0, d0 = outs[0]
        for c1, m1, d1 in outs[1:]:
            np.testing.assert_array_equal(c0, c1)
            for p in range(len(pairs)):
                np.testing.assert_array_equal(m0[p, :c0[p]], m1[p, :c1[p]])
                np.testing.assert_array_equal(d0[p, :c0[p]], d1[p, :c1[p]])


def _tie_heavy(rng, n_img, k, levels):
    """Descriptors drawn from a few byte values: exact distance ties everywhere."""
    return rng.integers(0, levels, size=(n_img, k, 128)).astype(np.uint8) * (255 // max(1, levels - 1))


@pytest.mark.parametrize("ratio", [(4, 5), (1, 1), (3, 2), (65535, 1)])
@pytest.mark.parametrize("xc", [1, 0])
def test_l2_ratio_path_ties_and_ragged(ctx, xc, ratio):
    """The forward/reverse ratio path (match_l2fr.hip) and the value-only-row mutual kernel:
    exact tie handling (e1 == e2, the unit ambiguity of d2, ambiguous column winners) against the
    oracle on tie-heavy, ragged sets."""
    import os
    rng = np.random.default_rng(100 + xc)
    desc = np.concatenate([_tie_heavy(rng, 3, 600, 2), _tie_heavy(rng, 2, 600, 3),
                           rng.integers(0, 256, size=(2, 600, 128), dtype=np.uint8)])
    desc[5, 100:140] = desc[0, 7]  # many identical trains/queries across images
    desc[6, :50] = desc[5, :50]
    n_kp = np.array([600, 599, 33, 600, 1, 600, 257], np.int32)
    pairs = np.array([[a, b] for a in range(7) for b in range(7) if a != b], np.int32)
    for path in (("fr", "mutual") if xc == 1 else ("fr",)):
        os.environ["SFM_L2_PATH"] = path
        try:
            _check_pairs(ctx, desc, n_kp, pairs, cross_check=xc, ratio=ratio)
            _check_pairs(ctx, desc, n_kp, pairs, cross_check=xc, ratio=ratio, max_dist=200000)
        finally:
            os.environ.pop("SFM_L2_PATH", None)


@pytest.mark.parametrize("K", [2048, 4096])
def test_l2_ratio_path_and_fused_kernel_agree(ctx, K):
    """Both L2 implementations (fused key kernel, forward/reverse ratio path) give identical
    outputs on the SIFT-like scene at full size."""
    import os
    s = synth.make_scene(4, K, seed=60 + K)
    n_kp = s["n_kp"].copy()
    n_kp[2] = K - 101
    pairs = synth.unordered_pairs(4)
    for xc, ratio in ((1, (4, 5)), (0, (4, 5)), (1, (9, 10)), (1, None), (2, None)):
        outs = []
        for v in (("fr", "fused", "mutual") if ratio else ("mutual", "fused")):
            os.environ["SFM_L2_PATH"] = v
            try:
                outs.append(_gpu_match(ctx, s["desc"], n_kp, pairs, cross_check=xc, ratio=ratio))
            finally:
                os.environ.pop("SFM_L2_PATH", None)
        c0, m0, d0 = outs[0]
        for c1, m1, d1 in outs[1:]:
            np.testing.assert_array_equal(c0, c1)
            for p in range(len(pairs)):
                np.testing.assert_array_equal(m0[p, :c0[p]], m1[p, :c1[p]])
                np.testing.assert_array_equal(d0[p, :c0[p]], d1[p, :c1[p]])


@pytest.mark.parametrize("xc", [1, 2])
def test_hamming_column_winner_kernel(ctx, xc):
    """The column-winner kernel on Hamming (column side only for the OpenCV rule; + value-only
    rows for mutual, tie-heavy on small integer distances): identical to the oracle."""
    import os
    s = synth.make_scene(3, 700, seed=77, orb=True)
    n_kp = s["n_kp"].copy()
    n_kp[2] = 433
    pairs = np.array([[0, 1], [1, 2], [2, 0], [1, 0]], np.int32)
    os.environ["SFM_HAMMING_PATH"] = "mutual"
    try:
        _check_pairs(ctx, s["desc"], n_kp, pairs, metric=1, cross_check=xc, max_dist=26)
        _check_pairs(ctx, s["desc"], n_kp, pairs, metric=1, cross_check=xc,
                     ratio=(4, 5) if xc == 1 else None)
    finally:
        os.environ.pop("SFM_HAMMING_PATH", None)


def _both(ctx, desc, n_kp, pairs, **kw):
    import torch
    d = torch.from_numpy(np.ascontiguousarray(desc)).cuda()
    n = torch.from_numpy(np.ascontiguousarray(n_kp, np.int32)).cuda()
    pr = torch.from_numpy(np.ascontiguousarray(pairs, np.int32)).cuda()
    cnt, mt, dist = ctx.match_batch_both(d, n, pr, **kw)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()


def _assert_both_equals_two_launches(ctx, desc, n_kp, metric, xc, maxd):
    """sfm_match_batch_both on the unordered pairs == sfm_match_batch on (a, b) and on (b, a),
    bit for bit (counts, indices, distances), and both == the oracle."""
    n = len(desc)
    up = synth.unordered_pairs(n)
    cnt, mt, dist = _both(ctx, desc, n_kp, up, metric=metric, cross_check=xc, max_dist=maxd)
    P = len(up)
    for half, prs in ((0, up), (1, up[:, ::-1].copy())):
        c2, m2, d2 = _gpu_match(ctx, desc, n_kp, prs, metric=metric, cross_check=xc,
                                max_dist=maxd)
        np.testing.assert_array_equal(cnt[half * P:(half + 1) * P], c2)
        for p in range(P):
            k = c2[p]
            np.testing.assert_array_equal(mt[half * P + p, :k], m2[p, :k])
            np.testing.assert_array_equal(dist[half * P + p, :k], d2[p, :k])
    _check_pairs(ctx, desc, n_kp, np.concatenate([up, up[:, ::-1]]), metric=metric,
                 cross_check=xc, max_dist=maxd)
    return cnt


@pytest.mark.parametrize("xc,maxd", [(2, 26), (2, -1), (1, 26), (0, -1)])
def test_both_orders_hamming_reference_shape(ctx, xc, maxd):
    """ORB-like descriptors at the reference's K = 500, ragged counts (an
    empty image, a single descriptor), planted duplicates (exact ties on both sides): one tile
    per unordered pair gives both ordered results bit-identical to two launches."""
    s = synth.make_scene(6, 500, seed=29, orb=True)
    desc, n_kp = s["desc"].copy(), s["n_kp"].copy()
    n_kp[1], n_kp[3], n_kp[4] = 313, 0, 1
    desc[2, 7] = desc[2, 9]          # two identical trains
    desc[0, 40:44] = desc[5, 100]    # one train equidistant to four queries
    cnt = _assert_both_equals_two_launches(ctx, desc, n_kp, 1, xc, maxd)
    assert cnt.sum() > 0


@pytest.mark.parametrize("xc,maxd", [(2, 26), (1, -1)])
def test_both_orders_hamming_k4096(ctx, xc, maxd):
    """Both orders from one tile at the largest k_max (4096: 16 query blocks of the key kernel per
    pair, the row merges every 4 tiles, train indices past 127 / 2047 in the key's low bits),
    ragged counts and planted duplicates: bit-identical to two launches and to the oracle."""
    s = synth.make_scene(3, 4096, seed=41, orb=True)
    desc, n_kp = s["desc"].copy(), s["n_kp"].copy()
    n_kp[1] = 3001
    desc[0, 4000] = desc[0, 129]        # a duplicated train far apart in index
    desc[2, 2048:2052] = desc[1, 7]     # one row equidistant to four neighbours
    cnt = _assert_both_equals_two_launches(ctx, desc, n_kp, 1, xc, maxd)
    assert cnt.sum() > 0


@pytest.mark.parametrize("xc,maxd", [(2, -1), (1, -1), (0, -1), (2, 30000)])
def test_both_orders_l2(ctx, xc, maxd):
    s = synth.make_scene(4, 1000, seed=31)
    desc, n_kp = s["desc"].copy(), s["n_kp"].copy()
    n_kp[2] = 517
    desc[1, 3] = desc[1, 8]
    cnt = _assert_both_equals_two_launches(ctx, desc, n_kp, 0, xc, maxd)
    assert cnt.sum() > 0


def test_both_orders_rejects_ratio_and_large_k(ctx):
    import torch
    s = synth.make_scene(2, 64, seed=1)
    d = torch.from_numpy(s["desc"]).cuda()
    n = torch.from_numpy(s["n_kp"]).cuda()
    pr = torch.tensor([[0, 1]], dtype=torch.int32).cuda()
    prm = sfmcore.MatchParams(0, 1, 4, 5, -1)
    out = [torch.empty(2, dtype=torch.int32).cuda(), torch.empty((2, 64, 2), dtype=torch.int32).cuda(),
           torch.empty((2, 64), dtype=torch.int32).cuda()]
    import ctypes as C
    rc = ctx.lib.sfm_match_batch_both(ctx.handle, d.data_ptr(), n.data_ptr(), 2, 64, 128,
                                      pr.data_ptr(), 1, C.byref(prm), out[0].data_ptr(),
                                      out[1].data_ptr(), out[2].data_ptr())
    assert rc != 0 and b"ratio" in ctx.lib.sfm_last_error()


@pytest.mark.parametrize("ratio", [(4, 5), (1, 1), None])
@pytest.mark.parametrize("metric", [0, 1])
def test_mutual_rule_planted_ties_vs_oracle(ctx, ratio, metric):
    """The mutual rule's kernels against the oracle on planted cases (kept from round 5's group-
    kernel test; that kernel measured slower and left the library, its record is in
    profiles/r05/): a tie of the nearest value inside one 16-train group (trains 0/1, 8/9: same
    lane half, same tile), a tie across tiles (trains 2 and 34), the runner-up one unit away in
    the same group, ragged sizes, tie-heavy sets.  L2 with a ratio test also runs the ratio path
    (SFM_L2_PATH=fr: forward scan, MFMA recovery, reverse scan): both equal the oracle."""
    import os
    rng = np.random.default_rng(321 + metric)
    k, dim = 700, (128 if metric == 0 else 32)
    desc = rng.integers(0, 256, size=(5, k, dim), dtype=np.uint8)
    if metric == 0:
        desc[3] = _tie_heavy(rng, 1, k, 2)[0]
    else:
        desc[3] = rng.integers(0, 2, size=(k, dim), dtype=np.uint8) * 255
    desc[1, 1] = desc[1, 0]          # nearest tie inside one group
    desc[1, 9] = desc[1, 8]
    desc[1, 34] = desc[1, 2]         # nearest tie across tiles
    desc[0, :40] = desc[1, :40]      # exact nearest neighbours for those queries
    desc[1, 3] = desc[1, 0] ^ 1      # runner-up one bit / unit away, in the same group as 0
    desc[2, 100:110] = desc[0, 5]
    n_kp = np.array([k, k - 3, 65, k, 33], np.int32)
    pairs = np.array([[a, b] for a in range(5) for b in range(5) if a != b], np.int32)
    paths = ["mutual", "fr"] if (metric == 0 and ratio is not None) else ["mutual"]
    for path in paths:
        env = "SFM_L2_PATH" if metric == 0 else "SFM_HAMMING_PATH"
        os.environ[env] = path
        try:
            _check_pairs(ctx, desc, n_kp, pairs, metric=metric, cross_check=1, ratio=ratio)
        finally:
            os.environ.pop(env, None)
