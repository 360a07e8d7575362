"""GPU parity of the reference-facing host layer (drop-in modules) and of the sizes the benchmark
configs use: K = 4096 (cfg4), the full 4096-hypothesis RANSAC (cfg3), the batched pair-graph
builder, and the BA J^TJ build through reconstruction.py (single rank of the sharded path).
Everything is checked against the CPU oracle (test infrastructure)."""
import numpy as np
import pytest

import feature_matching as fm
import geometric_verification as gv
import match_graph
import oracle as O
import reconstruction
import sfmcore
import synth

pytestmark = pytest.mark.gpu


def _ref_reference_semantics(d1, d2):
    """code/feature_matching.py:48-58 on the oracle: OpenCV cross-check rule, stable sort by
    distance, prefix with distance < 26."""
    q, t, d = O.match(d1, d2, metric=1, cross_check=O.XC_OPENCV, ratio=None, max_dist=-1)
    order = np.argsort(d, kind="stable")
    out = []
    for i in order:
        if d[i] >= 26:
            break
        out.append((int(q[i]), int(t[i]), float(d[i])))
    return out


def test_match_descriptors_reference_semantics():
    s = synth.make_scene(2, 500, seed=11, orb=True)
    d1, d2 = s["desc"][0][:480], s["desc"][1][:500]
    got = fm.match_descriptors(d1, d2)  # defaults = the reference's matcher
    want = _ref_reference_semantics(d1, d2)
    assert len(want) > 50
    assert [(m.queryIdx, m.trainIdx, m.distance) for m in got] == want
    assert all(m.imgIdx == 0 for m in got)


def test_match_descriptors_l2_ratio():
    s = synth.make_scene(2, 700, seed=12)
    got = fm.match_descriptors(s["desc"][0], s["desc"][1], norm="l2", cross_check="mutual",
                               max_distance=None, ratio=0.8, sort=False)
    q, t, d = O.match(s["desc"][0], s["desc"][1], 0, 1, (4, 5))
    assert [(m.queryIdx, m.trainIdx) for m in got] == list(zip(q.tolist(), t.tolist()))
    np.testing.assert_array_equal([m.distance for m in got],
                                  np.sqrt(d).astype(np.float32).astype(np.float64))


def test_l2_k4096_cfg4_size(ctx):
    import torch
    s = synth.make_scene(3, 4096, seed=13)
    pairs = np.array([[0, 1], [2, 0]], np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    cnt, mt, dist = ctx.match_batch(T(s["desc"]), T(s["n_kp"]), T(pairs), ratio=(4, 5))
    torch.cuda.synchronize()
    cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        q, t, d = O.match(s["desc"][a], s["desc"][b], 0, 1, (4, 5))
        assert cnt[p] == len(q) > 500
        np.testing.assert_array_equal(mt[p, :cnt[p], 0], q)
        np.testing.assert_array_equal(mt[p, :cnt[p], 1], t)
        np.testing.assert_array_equal(dist[p, :cnt[p]], d)


def test_verify_pair_full_4096_hypotheses():
    s = synth.make_scene(2, 2048, seed=14)
    q, t, _ = O.match(s["desc"][0], s["desc"][1], 0, 1, (4, 5))
    r = gv.verify_pair(s["kps"][0], s["kps"][1], np.c_[q, t], pair=(0, 1), n_hyp=4096)
    o = O.ransac_f(s["kps"][0][q], s["kps"][1][t], H=4096, seed=42, pa=0, pb=1)
    assert r["count"] == o["count"] and r["best_h"] == o["best_h"] and r["verified"]
    np.testing.assert_array_equal(r["inliers"], np.nonzero(o["mask"])[0])
    np.testing.assert_allclose(r["F"], gv.denormalize_F(o["F"], o["norm"]), rtol=0, atol=1e-6)


def test_verify_pairs_on_reference_pair_objects():
    class Pair:  # code/pipeline.py:6-9
        def __init__(self, i, j, matches):
            self.img_inx_1, self.img_inx_2, self.matches = i, j, matches

    s = synth.make_scene(3, 1024, seed=15)
    prs = []
    for i, j in ((0, 1), (1, 2)):
        ms = fm.match_descriptors(s["desc"][i], s["desc"][j], norm="l2", cross_check="mutual",
                                  max_distance=None, ratio=(4, 5), sort=False)
        prs.append(Pair(i, j, ms))
    n_before = [len(p.matches) for p in prs]
    out = gv.verify_pairs(prs, s["kps"], n_hyp=1024)
    assert len(out) == 2
    for p, nb in zip(out, n_before):
        mt = np.array([[m.queryIdx, m.trainIdx] for m in p.matches])
        assert 15 <= len(mt) < nb and p.F.shape == (3, 3)


def test_graph_builder_matches_oracle():
    import torch
    s = synth.make_scene(6, 1024, seed=16)
    pairs = synth.unordered_pairs(6)
    gb = match_graph.GraphBuilder(s["desc"], s["kps"], s["n_kp"], ratio=(4, 5), n_hyp=512)
    pt = torch.from_numpy(pairs).cuda()
    count, match, dist, rs = gb.run(pt)
    rows = gb.graph_rows(0, count, match, rs).cpu().numpy()
    want = []
    for p, (a, b) in enumerate(pairs):
        q, t, _ = O.match(s["desc"][a], s["desc"][b], 0, 1, (4, 5))
        r = O.ransac_f(s["kps"][a][q], s["kps"][b][t], H=512, seed=42, pa=int(a), pb=int(b))
        if r["count"] >= 15:
            want += [(p, int(q[i]), int(t[i])) for i in np.nonzero(r["mask"])[0]]
    np.testing.assert_array_equal(rows, np.array(want, np.int32).reshape(-1, 3))


def test_build_jtj_and_sharded_single_rank():
    pr = synth.make_ba_problem(9, 300, obs_per_pt=4, seed=17)
    o = O.ba_jtj(pr["cams"], pr["pp"], pr["pts"], pr["cam_idx"], pr["pt_idx"], pr["uv"],
                 loss_s=1.5)
    g = reconstruction.build_jtj(pr["cams"], pr["pp"], pr["pts"], pr["cam_idx"], pr["pt_idx"],
                                 pr["uv"], loss_s=1.5)
    np.testing.assert_allclose(g["U"], o["U"], rtol=1e-10, atol=1e-8)
    assert np.abs(g["res"] - o["res"]).max() < 1e-4
    sh = reconstruction.build_jtj_sharded(pr["cams"], pr["pp"], pr["pts"], pr["cam_idx"],
                                          pr["pt_idx"], pr["uv"], 0, 1, loss_s=1.5)
    assert sh["pt_range"] == (0, 300)
    np.testing.assert_array_equal(sh["U"].cpu().numpy(), g["U"])
    # shuffled observation order goes through the regrouping path of build_jtj
    perm = np.random.default_rng(0).permutation(len(pr["pt_idx"]))
    g2 = reconstruction.build_jtj(pr["cams"], pr["pp"], pr["pts"], pr["cam_idx"][perm],
                                  pr["pt_idx"][perm], pr["uv"][perm], loss_s=1.5)
    np.testing.assert_array_equal(g2["res"], g["res"][perm])
    np.testing.assert_allclose(g2["U"], g["U"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("P,K", [(1, 16), (37, 300), (2500, 64)])
def test_graph_rows_compaction(ctx, P, K):
    """sfm_graph_offsets / sfm_graph_rows against a numpy restatement on random masks: scan over
    more than one 1024-pair tile, unverified / empty pairs, ragged match counts."""
    import torch
    rng = np.random.default_rng(P)
    count = rng.integers(0, K + 1, P).astype(np.int32)
    match = rng.integers(0, 5000, (P, K, 2)).astype(np.int32)
    mask = (rng.random((P, K)) < 0.4).astype(np.uint8)
    mask[:, :][np.arange(K)[None, :] >= count[:, None]] = 1  # stale entries beyond count
    inl = np.array([mask[p, :count[p]].sum() for p in range(P)], np.int32)
    inl[rng.random(P) < 0.2] = -1
    want = [(7 + p, *match[p, m]) for p in range(P) if inl[p] >= 15
            for m in range(count[p]) if mask[p, m]]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    rows = ctx.graph_rows(7, T(count), T(match), T(inl), T(mask), 15).cpu().numpy()
    np.testing.assert_array_equal(rows, np.array(want, np.int32).reshape(-1, 3))


def test_graph_packed_roundtrip_on_device():
    """Device path of the bench step: graph_rows + offsets -> pack_rows -> all_gather_graph
    (world 1) reproduces the rows."""
    import torch
    s = synth.make_scene(5, 1024, seed=18)
    pairs = synth.unordered_pairs(5)
    gb = match_graph.GraphBuilder(s["desc"], s["kps"], s["n_kp"], ratio=(4, 5), n_hyp=512)
    count, match, dist, rs = gb.run(torch.from_numpy(pairs).cuda())
    rows, offs = gb.graph_rows(0, count, match, rs, return_offsets=True)
    c, pk = match_graph.pack_rows(rows, offs)
    g = match_graph.all_gather_graph(c, pk, [(0, len(pairs))])
    np.testing.assert_array_equal(g.cpu().numpy(), rows.cpu().numpy())
    assert int(offs[-1]) == rows.shape[0] > 0
    # the kernel-written exchange form (sfm_graph_rows_packed) is the same packing, same offsets
    pk2, offs2 = gb.graph_rows(0, count, match, rs, return_offsets=True, packed=True)
    np.testing.assert_array_equal(offs2.cpu().numpy(), offs.cpu().numpy())
    np.testing.assert_array_equal(pk2.cpu().numpy(), pk.cpu().numpy())
    c2 = (offs2[1:] - offs2[:-1]).to(torch.int32)
    g2 = match_graph.all_gather_graph(c2, pk2, [(0, len(pairs))])
    np.testing.assert_array_equal(g2.cpu().numpy(), rows.cpu().numpy())


def test_graph_expand_kernel_multi_rank_layout():
    """sfm_graph_expand on a gathered multi-rank layout (padded per-rank slots, ragged shards, an
    empty shard, empty pairs, indices >= 32768 in both halves of the packed word) equals the
    host expansion of the same buffers, and a non-zero first pair index carries through."""
    import torch
    rng = np.random.default_rng(7)
    ranges = [(3, 40), (40, 40), (40, 95), (95, 101)]
    world = len(ranges)
    maxp = max(hi - lo for lo, hi in ranges)
    call = np.zeros((world, maxp), np.int32)
    tot = []
    for r, (lo, hi) in enumerate(ranges):
        c = rng.integers(0, 200, hi - lo).astype(np.int32)
        c[rng.random(hi - lo) < 0.2] = 0
        call[r, :hi - lo] = c
        tot.append(int(c.sum()))
    maxn = max(max(tot), 1)
    rall = np.full((world, maxn), -7, np.int32)  # padding must never be read
    for r in range(world):
        q = rng.integers(0, 65536, tot[r]).astype(np.uint32)
        t = rng.integers(0, 65536, tot[r]).astype(np.uint32)
        rall[r, :tot[r]] = ((q << 16) | t).view(np.int32)
    want = match_graph.expand_gathered(torch.from_numpy(call), torch.from_numpy(rall), tot,
                                       ranges, maxn)
    got = match_graph.expand_gathered(torch.from_numpy(call).cuda(),
                                      torch.from_numpy(rall).cuda(), tot, ranges, maxn)
    assert got.shape == (sum(tot), 3)
    np.testing.assert_array_equal(got.cpu().numpy(), want.numpy())
    assert int(got[0, 0]) == 3 and int(got[:, 1].max()) >= 32768


def test_match_all_pairs_equals_reference_loop():
    """Batched all-pairs entry == the reference's per-ordered-pair loop (code/pipeline.py:38-47)
    over match_descriptors, including the drop of empty results."""
    s = synth.make_scene(4, 300, seed=19, orb=True)
    des = [s["desc"][i][: 300 - 25 * i] for i in range(4)]
    des.append(np.zeros((0, 32), np.uint8))  # an image without keypoints
    got = fm.match_all_pairs(des)
    want = []
    for i in range(len(des)):
        for j in range(len(des)):
            if i != j:
                m = fm.match_descriptors(des[i], des[j])
                if m:
                    want.append((i, j, [(x.queryIdx, x.trainIdx, x.distance) for x in m]))
    assert [(p.img_inx_1, p.img_inx_2, [(x.queryIdx, x.trainIdx, x.distance) for x in p.matches])
            for p in got] == want
    assert all(p.img_inx_1 != 4 and p.img_inx_2 != 4 for p in got)


def test_verify_pairs_batched_equals_per_pair_on_ordered_list():
    """The reference's ordered N(N-1) Pair list (code/pipeline.py:36-47, match_all_pairs
    ordered=True) verified in ONE ransac_batch launch equals verify_pair on each pair."""
    import copy
    s = synth.make_scene(5, 1024, seed=17)
    prs = fm.match_all_pairs([s["desc"][i] for i in range(5)], norm="l2", cross_check="mutual",
                             max_distance=None, ratio=(4, 5), ordered=True, sort=False)
    assert len(prs) == 20
    ref = [gv.verify_pair(s["kps"][p.img_inx_1], s["kps"][p.img_inx_2], p.matches,
                          pair=(p.img_inx_1, p.img_inx_2), n_hyp=1024) for p in prs]
    calls = []
    orig = sfmcore.Context.ransac_batch

    def counted(self, *a, **k):
        calls.append(1)
        return orig(self, *a, **k)

    sfmcore.Context.ransac_batch = counted
    try:
        before = copy.deepcopy(prs)
        out = gv.verify_pairs(prs, s["kps"], n_hyp=1024)
    finally:
        sfmcore.Context.ransac_batch = orig
    assert len(calls) == 1
    exp = [(b, r) for b, r in zip(before, ref) if r["verified"]]
    assert len(out) == len(exp) > 0
    for o, (b, r) in zip(out, exp):
        assert (o.img_inx_1, o.img_inx_2) == (b.img_inx_1, b.img_inx_2)
        assert [(m.queryIdx, m.trainIdx) for m in o.matches] == \
            [(b.matches[i].queryIdx, b.matches[i].trainIdx) for i in r["inliers"]]
        np.testing.assert_array_equal(o.F, r["F"])


def test_verify_pairs_chunked_equals_one_batch():
    """verify_pairs works in fixed-size chunks (constant memory for the ordered
    N(N-1) list); the RNG is keyed by image ids, so chunking changes nothing."""
    import copy
    s = synth.make_scene(5, 1024, seed=17)
    prs = fm.match_all_pairs([s["desc"][i] for i in range(5)], norm="l2", cross_check="mutual",
                             max_distance=None, ratio=(4, 5), ordered=True, sort=False)
    one = gv.verify_pairs(copy.deepcopy(prs), s["kps"], n_hyp=1024)
    chunked = gv.verify_pairs(copy.deepcopy(prs), s["kps"], n_hyp=1024, chunk=3)
    assert len(one) == len(chunked) > 0
    for a, b in zip(one, chunked):
        assert (a.img_inx_1, a.img_inx_2) == (b.img_inx_1, b.img_inx_2)
        assert [(m.queryIdx, m.trainIdx) for m in a.matches] == \
            [(m.queryIdx, m.trainIdx) for m in b.matches]
        np.testing.assert_array_equal(a.F, b.F)
