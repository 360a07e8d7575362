"""GPU parity: 8-point RANSAC (K2) vs the CPU oracle at a fixed seed — identical inlier sets.

Bit-exact contract: best inlier count, winning hypothesis id, the inlier mask and the normalised
F (every f32 bit).  Also checks the per-pair shard invariance the multi-GPU path relies on:
a pair's result does not depend on which other pairs share the launch.
"""
import numpy as np
import pytest

import oracle as O
import sfmcore
import synth

pytestmark = pytest.mark.gpu


def _run(ctx, s, pairs, H=1024, seed=42, thr=1.0, ratio=(4, 5)):
    import torch
    desc = torch.from_numpy(s["desc"]).cuda()
    n_kp = torch.from_numpy(s["n_kp"]).cuda()
    kps = torch.from_numpy(s["kps"]).cuda()
    pr = torch.from_numpy(np.ascontiguousarray(pairs, np.int32)).cuda()
    cnt, mt, _ = ctx.match_batch(desc, n_kp, pr, ratio=ratio)
    out = ctx.ransac_batch(kps, pr, cnt, mt, n_hyp=H, seed=seed, thr=thr)
    torch.cuda.synchronize()
    return cnt.cpu().numpy(), mt.cpu().numpy(), {k: v.cpu().numpy() for k, v in out.items()}


def _oracle(s, a, b, q, t, H, seed, thr):
    x1 = s["kps"][a][q]
    x2 = s["kps"][b][t]
    return O.ransac_f(x1, x2, H=H, seed=seed, pa=int(a), pb=int(b), thr=thr)


@pytest.mark.parametrize("H,thr", [(256, 1.0), (1024, 1.0), (512, 4.0)])
def test_ransac_bit_exact(ctx, H, thr):
    s = synth.make_scene(5, 1024, seed=21)
    pairs = synth.unordered_pairs(5)
    cnt, mt, out = _run(ctx, s, pairs, H=H, thr=thr)
    for p, (a, b) in enumerate(pairs):
        M = cnt[p]
        r = _oracle(s, a, b, mt[p, :M, 0], mt[p, :M, 1], H, 42, thr)
        assert out["inl_count"][p] == r["count"], f"pair {p}"
        assert out["best_h"][p] == r["best_h"], f"pair {p}"
        np.testing.assert_array_equal(out["mask"][p, :M], r["mask"])
        np.testing.assert_array_equal(out["F"][p].view(np.uint32), r["F"].view(np.uint32))
        np.testing.assert_array_equal(out["norm"][p].view(np.uint32), r["norm"].view(np.uint32))


def test_ransac_hypothesis_counts_match(ctx):
    # the winner is only as good as every score: compare all hypothesis counts via best-of-one
    s = synth.make_scene(2, 2048, seed=4)
    pairs = np.array([[0, 1]], np.int32)
    cnt, mt, out = _run(ctx, s, pairs, H=256)
    M = cnt[0]
    counts = O.ransac_counts(s["kps"][0][mt[0, :M, 0]], s["kps"][1][mt[0, :M, 1]], H=256,
                             seed=42, pa=0, pb=1, thr=1.0)
    assert out["inl_count"][0] == counts.max()
    assert out["best_h"][0] == int(np.argmax(counts))


def test_ransac_few_matches_and_degenerate(ctx):
    import torch
    # pairs with < 8 tentative matches are unverified (-1); duplicated points -> degenerate samples
    rng = np.random.default_rng(0)
    k_max = 64
    kps = rng.uniform(0, 1000, size=(3, k_max, 2)).astype(np.float32)
    kps[2, :] = kps[2, 0]  # all keypoints identical
    pairs = np.array([[0, 1], [0, 2], [1, 2]], np.int32)
    count = np.array([5, 40, 0], np.int32)
    match = np.zeros((3, k_max, 2), np.int32)
    for p in range(3):
        match[p, :, 0] = np.arange(k_max)
        match[p, :, 1] = rng.permutation(k_max)
    kt = torch.from_numpy(kps).cuda()
    out = ctx.ransac_batch(kt, torch.from_numpy(pairs).cuda(), torch.from_numpy(count).cuda(),
                           torch.from_numpy(match).cuda(), n_hyp=256)
    torch.cuda.synchronize()
    ic = out["inl_count"].cpu().numpy()
    assert ic[0] == -1 and ic[2] == -1
    r = O.ransac_f(kps[0][match[1, :40, 0]], kps[2][match[1, :40, 1]], H=256, seed=42, pa=0, pb=2)
    assert ic[1] == r["count"]
    np.testing.assert_array_equal(out["mask"].cpu().numpy()[1, :40], r["mask"])


def test_ransac_shard_invariance(ctx):
    s = synth.make_scene(6, 1024, seed=8)
    pairs = synth.unordered_pairs(6)
    cnt, mt, full = _run(ctx, s, pairs, H=512)
    sub = pairs[5:11]
    cnt2, mt2, part = _run(ctx, s, sub, H=512)
    np.testing.assert_array_equal(full["inl_count"][5:11], part["inl_count"])
    np.testing.assert_array_equal(full["best_h"][5:11], part["best_h"])
    np.testing.assert_array_equal(cnt[5:11], cnt2)
    for k in range(6):
        M = cnt2[k]
        np.testing.assert_array_equal(full["mask"][5 + k, :M], part["mask"][k, :M])


def _ransac_direct(ctx, kps, count, match, pairs, H):
    import torch
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    out = ctx.ransac_batch(T(kps), T(pairs), T(count), T(match), n_hyp=H)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("M", [8, 9, 20, 63, 64, 65, 79, 80, 127, 128, 129, 130, 143, 144, 145])
def test_ransac_preview_boundaries(ctx, M):
    """Match counts around the PV-match preview (128; 64 through round 3) and the 16-match scoring
    chunks of the ordered schedule (fit + preview / ordered scoring), on a real two-view geometry with outliers."""
    s = synth.make_scene(2, 512, seed=30 + M)
    q, t, _ = O.match(s["desc"][0], s["desc"][1], 0, 1, (4, 5))
    assert len(q) >= M
    k_max = 512
    match = np.zeros((1, k_max, 2), np.int32)
    match[0, :M, 0] = q[:M]
    match[0, :M, 1] = t[:M]
    out = _ransac_direct(ctx, s["kps"], np.array([M], np.int32), match,
                         np.array([[0, 1]], np.int32), 512)
    r = O.ransac_f(s["kps"][0][q[:M]], s["kps"][1][t[:M]], H=512, seed=42, pa=0, pb=1)
    assert out["inl_count"][0] == r["count"] and out["best_h"][0] == r["best_h"]
    np.testing.assert_array_equal(out["mask"][0, :M], r["mask"])
    np.testing.assert_array_equal(out["F"][0].view(np.uint32), r["F"].view(np.uint32))


def test_ransac_schedules_agree(ctx):
    """The three K2 schedules (ordered, single-pass pruned, unpruned; SFM_RANSAC_MODE) differ only
    in which work is skipped: every output must be identical."""
    import os
    s = synth.make_scene(8, 1024, seed=12)
    pairs = synth.unordered_pairs(8)
    outs = []
    old = os.environ.get("SFM_RANSAC_MODE")
    try:
        for mode in ("0", "1", "2"):
            os.environ["SFM_RANSAC_MODE"] = mode
            outs.append(_run(ctx, s, pairs, H=1024))
    finally:
        if old is None:
            os.environ.pop("SFM_RANSAC_MODE", None)
        else:
            os.environ["SFM_RANSAC_MODE"] = old
    cnt = outs[0][0]
    for _, _, o in outs[1:]:
        for k in ("inl_count", "best_h", "F", "norm"):
            np.testing.assert_array_equal(o[k], outs[0][2][k])
        for p in range(len(pairs)):
            np.testing.assert_array_equal(o["mask"][p, :cnt[p]], outs[0][2]["mask"][p, :cnt[p]])


def test_ransac_pair_groups_agree(ctx):
    """The ordered schedule's pair groups per XCD (ransac.hip xcd_pair_block / ransac_group;
    SFM_RANSAC_GROUP) only change the block order: 465 pairs (59 per XCD, the last XCD short) with
    groups of 1, 5, 7 and 64 (one group) give identical outputs, and a sample matches the oracle."""
    import os
    s = synth.make_scene(31, 512, seed=21)
    pairs = synth.unordered_pairs(31)
    outs = []
    old = os.environ.get("SFM_RANSAC_GROUP")
    try:
        for g in ("64", "1", "5", "7"):
            os.environ["SFM_RANSAC_GROUP"] = g
            outs.append(_run(ctx, s, pairs, H=512))
    finally:
        if old is None:
            os.environ.pop("SFM_RANSAC_GROUP", None)
        else:
            os.environ["SFM_RANSAC_GROUP"] = old
    cnt, mt, ref = outs[0]
    for _, _, o in outs[1:]:
        for k in ("inl_count", "best_h", "F"):
            np.testing.assert_array_equal(o[k], ref[k])
        for p in range(len(pairs)):
            np.testing.assert_array_equal(o["mask"][p, :cnt[p]], ref["mask"][p, :cnt[p]])
    for p in range(0, len(pairs), 37):
        a, b = pairs[p]
        r = _oracle(s, a, b, mt[p, :cnt[p], 0], mt[p, :cnt[p], 1], 512, 42, 1.0)
        assert ref["inl_count"][p] == r["count"] and ref["best_h"][p] == r["best_h"]


@pytest.mark.parametrize("thr", [1.0, 4.0, 0.25])
def test_ransac_counts_every_hypothesis(ctx, thr):
    """EVERY hypothesis gets the f32 spec's count (sfm_ransac_counts: the score kernel without
    pruning), not only the winner."""
    import torch
    s = synth.make_scene(6, 1024, seed=77)
    pairs = synth.unordered_pairs(6)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    pr = T(pairs)
    cnt, mt, _ = ctx.match_batch(T(s["desc"]), T(s["n_kp"]), pr, ratio=(4, 5))
    counts, norm = ctx.ransac_counts(T(s["kps"]), pr, cnt, mt, n_hyp=512, thr=thr)
    torch.cuda.synchronize()
    counts, cnt, mt = counts.cpu().numpy(), cnt.cpu().numpy(), mt.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        M = cnt[p]
        ref = O.ransac_counts(s["kps"][a][mt[p, :M, 0]], s["kps"][b][mt[p, :M, 1]], H=512, seed=42,
                              pa=int(a), pb=int(b), thr=thr)
        np.testing.assert_array_equal(counts[p], ref, err_msg=f"pair {p} (M={M})")


def test_ransac_counts_k4096_and_tails(ctx):
    """cfg4-sized pairs (K = 4096, ~1000+ tentative matches) and match counts around the
    PV-match preview (128) and the 16-match scoring chunks: every hypothesis count equals the
    oracle's."""
    import torch
    s = synth.make_scene(3, 4096, seed=5)
    pairs = synth.unordered_pairs(3)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    pr = T(pairs)
    cnt, mt, _ = ctx.match_batch(T(s["desc"]), T(s["n_kp"]), pr, ratio=(4, 5))
    cnt_h, mt_h = cnt.cpu().numpy(), mt.cpu().numpy()
    # truncated copies of pair 0 around the preview (64 / 128) and the scoring chunks (16)
    Ms = [9, 64, 65, 79, 80, 95, 96, 97, 127, 128, 129, 144, 145, 161, 200]
    P = len(pairs) + len(Ms)
    pairs2 = np.concatenate([pairs, np.repeat(pairs[:1], len(Ms), 0)]).astype(np.int32)
    cnt2 = np.concatenate([cnt_h, np.minimum(Ms, cnt_h[0])]).astype(np.int32)
    mt2 = np.concatenate([mt_h, np.repeat(mt_h[:1], len(Ms), 0)])
    counts, _ = ctx.ransac_counts(T(s["kps"]), T(pairs2), T(cnt2), T(mt2), n_hyp=256)
    counts = counts.cpu().numpy()
    for p in range(P):
        a, b = pairs2[p]
        M = cnt2[p]
        ref = O.ransac_counts(s["kps"][a][mt2[p, :M, 0]], s["kps"][b][mt2[p, :M, 1]], H=256,
                              seed=42, pa=int(a), pb=int(b), thr=1.0)
        np.testing.assert_array_equal(counts[p], ref, err_msg=f"pair {p} (M={M})")


def test_ransac_f64_small_pairs_bit_exact(ctx):
    """fp64 mode on small / ragged pairs (fewer than 8, exactly 8, PV boundaries) vs the oracle."""
    import torch
    s = synth.make_scene(4, 700, seed=31)
    pairs = np.array([[0, 1], [1, 2], [2, 3], [0, 3]], np.int32)
    n_keep = [700, 8, 5, 129]
    cnt, mt = [], []
    k_max = 700
    match = np.zeros((len(pairs), k_max, 2), np.int32)
    for p, (a, b) in enumerate(pairs):
        q, t, _ = O.match(s["desc"][a], s["desc"][b], 0, 1, (4, 5))
        m = min(len(q), n_keep[p])
        match[p, :m] = np.c_[q[:m], t[:m]]
        cnt.append(m)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    rs = ctx.ransac_batch(T(s["kps"].astype(np.float64)), T(pairs), T(np.array(cnt, np.int32)),
                          T(match), n_hyp=512, seed=7, thr=1.0)
    torch.cuda.synchronize()
    rs = {k: v.cpu().numpy() for k, v in rs.items()}
    for p, (a, b) in enumerate(pairs):
        m = cnt[p]
        x1 = s["kps"][a][match[p, :m, 0]].astype(np.float64)
        x2 = s["kps"][b][match[p, :m, 1]].astype(np.float64)
        o = O.ransac_f(x1, x2, H=512, seed=7, pa=int(a), pb=int(b), f64=True)
        assert rs["inl_count"][p] == o["count"] and rs["best_h"][p] == o["best_h"]
        if m >= 8:
            np.testing.assert_array_equal(rs["mask"][p, :m], o["mask"])
            assert rs["F"][p].view(np.uint64).tolist() == o["F"].view(np.uint64).tolist()
            assert rs["norm"][p].view(np.uint64).tolist() == o["norm"].view(np.uint64).tolist()


def test_ransac_stats_identity(ctx):
    """K2's `executed` counter is issued lane-slots, and it satisfies an exact
    identity with the per-wave counts read back separately (sfm_ransac_wave_stops):
    executed = sum over pairs with M >= 8 of H min(PV, M) + 64 sum_w stop_w + M;
    algorithmic = H sum M; H min(PV, M) + M <= executed <= H M + M per batch.  Pairs with M < 8
    and M <= PV (no wave scores past the preview) are in the batch."""
    import torch
    PV, H = 128, 1024
    s = synth.make_scene(7, 2048, seed=5)
    pairs = synth.unordered_pairs(7)
    desc = torch.from_numpy(s["desc"]).cuda()
    kps = torch.from_numpy(s["kps"]).cuda()
    pr = torch.from_numpy(np.ascontiguousarray(pairs, np.int32)).cuda()
    cnt, mt, _ = ctx.match_batch(desc, torch.from_numpy(s["n_kp"]).cuda(), pr, ratio=(4, 5))
    cnt[0], cnt[1], cnt[2] = 5, 100, 128          # M < 8, M < PV, M == PV
    ctx.ransac_stats(enable=True, read=True)      # reset
    out = ctx.ransac_batch(kps, pr, cnt, mt, n_hyp=H, seed=42, thr=1.0)
    stops = ctx.ransac_wave_stops(len(pairs), H).astype(np.int64)
    ex, al, npairs = ctx.ransac_stats(enable=False, read=True)
    M = cnt.cpu().numpy().astype(np.int64)
    sel = M >= 8
    assert sel.sum() == npairs == len(pairs) - 1
    assert al == H * M[sel].sum()
    assert (stops[sel] <= np.maximum(M[sel] - PV, 0)[:, None]).all()
    assert (stops[1:3] == 0).all()
    exp = (H * np.minimum(PV, M[sel]) + 64 * stops[sel].sum(1) + M[sel]).sum()
    assert ex == exp
    assert (H * np.minimum(PV, M[sel]) + M[sel]).sum() <= ex <= (H * M[sel] + M[sel]).sum()
    # the counters do not change the results (mask entries past M are not written)
    ref = ctx.ransac_batch(kps, pr, cnt, mt, n_hyp=H, seed=42, thr=1.0)
    for k in ("inl_count", "best_h"):
        assert torch.equal(out[k], ref[k])
    for p in range(len(pairs)):
        assert torch.equal(out["mask"][p, :M[p]], ref["mask"][p, :M[p]])
    # any later workspace user invalidates the counted batch's wave words, and the
    # read-back then fails cleanly (no stale or freed device memory is read)
    ctx.ransac_stats(enable=True, read=True)
    ctx.ransac_batch(kps, pr, cnt, mt, n_hyp=H, seed=42, thr=1.0)
    ctx.match_batch(desc, torch.from_numpy(s["n_kp"]).cuda(), pr, ratio=(4, 5))
    ctx.ransac_stats(enable=False, read=True)
    with pytest.raises(sfmcore.SfmCoreError):
        ctx.ransac_wave_stops(len(pairs), H)
