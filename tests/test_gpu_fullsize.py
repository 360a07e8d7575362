"""GPU parity at the benchmark's full launch sizes (VERDICT r1 "next" item 1), against the CPU
oracle (test infrastructure):

* cfg3 (BASELINE configs[2]): the full 1225-pair launch (XCD-mapped pair ordering, grid padding,
  H = 4096) through match_graph.GraphBuilder — every pair's count, match indices, d^2, inlier
  count, winner, mask and F bits, and the verified graph rows;
* cfg4 (configs[3]) per-GPU shard: one contiguous 1/8 shard of the 500-image x 4096 scene's
  124 750 pairs in one launch, a stride sample of it checked the same way;
* cfg5 (configs[4]) BA J^TJ at 500 cameras x 100 k points x 5 observations;
* k_max above 4096: the Hamming VALU path (ragged 5000) under both cross-check rules with
  `< 26`, then RANSAC on its matches;
* one context driven from two torch streams (the workspace hand-off in sfm_ctx_set_stream);
* the RCCL (`nccl`) branches of the graph all-gather and the camera-block all-reduce, in a
  world-size-1 group on the device.

Reference semantics: code/feature_matching.py:48-58 (matcher), code/pipeline.py:38-47 (pair
loop); RANSAC / BA follow the build's spec.
"""
import os
import socket

import numpy as np
import pytest

import match_graph
import oracle as O
import reconstruction
import sfmcore
import synth

pytestmark = pytest.mark.gpu

H = 4096


def _check_pairs(scene, pairs, idx, res, min_inl=15):
    """Full per-pair comparison of GPU results `res` (numpy, rows `idx` of the launch) against
    the oracle on pairs[idx]."""
    sample = np.ascontiguousarray(pairs[idx])
    _, nm, ni, full = O.match_verify_batch(scene["desc"], scene["kps"], sample, ratio=(4, 5),
                                           H=H, seed=42, thr=1.0, min_inl=min_inl, full=True)
    cnt, mt, dist = res["count"][idx], res["match"][idx], res["dist"][idx]
    inl, bh, mask, F = res["inl_count"][idx], res["best_h"][idx], res["mask"][idx], res["F"][idx]
    np.testing.assert_array_equal(cnt, nm)
    n_checked = 0
    for p in range(len(sample)):
        m = nm[p]
        np.testing.assert_array_equal(mt[p, :m], full["match"][p, :m], err_msg=f"pair {p}")
        np.testing.assert_array_equal(dist[p, :m], full["dist"][p, :m], err_msg=f"pair {p}")
        if m < 8:
            assert inl[p] == -1
            continue
        assert inl[p] == ni[p] and bh[p] == full["best_h"][p], f"pair {p}"
        np.testing.assert_array_equal(mask[p, :m], full["mask"][p, :m], err_msg=f"pair {p}")
        assert F[p].view(np.uint32).tolist() == full["F"][p].view(np.uint32).tolist()
        n_checked += 1
    return nm, ni, full, n_checked


def _run_builder(gb, pairs_np, base=0):
    import torch
    pt = torch.from_numpy(np.ascontiguousarray(pairs_np)).cuda()
    count, match, dist, rs = gb.run(pt)
    rows = gb.graph_rows(base, count, match, rs)
    torch.cuda.synchronize()
    res = dict(count=count.cpu().numpy(), match=match.cpu().numpy(), dist=dist.cpu().numpy(),
               **{k: v.cpu().numpy() for k, v in rs.items()})
    return res, rows.cpu().numpy()


def _expected_rows(gpair, nm, ni, full, min_inl=15):
    out = []
    for p in range(len(gpair)):
        if ni[p] >= min_inl:
            mm = full["mask"][p, :nm[p]].astype(bool)
            q = full["match"][p, :nm[p]][mm]
            out.append(np.column_stack([np.full(len(q), gpair[p], np.int32), q]))
    return np.concatenate(out) if out else np.zeros((0, 3), np.int32)


def test_cfg3_full_launch_every_pair():
    scene = synth.make_scene(50, 2048, seed=0)
    pairs = synth.unordered_pairs(50)
    gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"], ratio=(4, 5),
                                  n_hyp=H, seed=42, thr=1.0, min_inliers=15)
    res, rows = _run_builder(gb, pairs)
    idx = np.arange(len(pairs))
    nm, ni, full, n = _check_pairs(scene, pairs, idx, res)
    assert n == len(pairs)                     # every pair has >= 8 tentative matches
    np.testing.assert_array_equal(rows, _expected_rows(idx, nm, ni, full))
    assert rows.shape[0] > 500_000              # the bench's ~554 k verified matches


def test_cfg2_ratio_rule_every_pair(ctx):
    """BASELINE configs[1] (cfg2) at full size, its own rule: all 1225 pairs of 50 x 2048 128-D,
    L2 with the fused ratio test 4/5 and no cross check — the dispatcher's ratio path (forward
    MFMA scan, MFMA recovery, exact slow path, compaction). Every pair's count, (query, train)
    indices and d^2 equal the oracle's (oracle_match, the rule of code/feature_matching.py:48-58
    without crossCheck plus the exact ratio test), bit for bit."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    scene = synth.make_scene(50, 2048, seed=0)
    pairs = synth.unordered_pairs(50)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    cnt, mt, dist = ctx.match_batch(T(scene["desc"]), T(scene["n_kp"]), T(pairs), cross_check=0,
                                    ratio=(4, 5))
    torch.cuda.synchronize()
    cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
    d = scene["desc"]
    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:   # ctypes releases the GIL
        ref = list(ex.map(lambda ab: O.match(d[ab[0]], d[ab[1]], 0, 0, (4, 5)), pairs))
    for p, (q, t, dd) in enumerate(ref):
        assert cnt[p] == len(q), f"pair {p}"
        np.testing.assert_array_equal(mt[p, :cnt[p], 0], q, err_msg=f"pair {p}")
        np.testing.assert_array_equal(mt[p, :cnt[p], 1], t, err_msg=f"pair {p}")
        np.testing.assert_array_equal(dist[p, :cnt[p]], dd, err_msg=f"pair {p}")
    assert cnt.sum() > 1_000_000                # 1 170 943 tentative matches (k1_cfg2_time.py)


def test_cfg4_shard_sample():
    scene = synth.make_scene(500, 4096, seed=0)
    pairs = synth.unordered_pairs(500)
    assert len(pairs) == 124_750
    lo, hi = match_graph.shard_range(pairs, 3, 8, scene["n_kp"])
    assert 15_000 < hi - lo < 16_000
    gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"], ratio=(4, 5),
                                  n_hyp=H, seed=42, thr=1.0, min_inliers=15)
    res, rows = _run_builder(gb, pairs[lo:hi], base=lo)
    idx = np.arange(0, hi - lo, (hi - lo) // 96)[:96]
    nm, ni, full, n = _check_pairs(scene, pairs[lo:hi], idx, res)
    assert n == len(idx) and nm.min() > 500
    got = rows[np.isin(rows[:, 0], lo + idx)]
    np.testing.assert_array_equal(got, _expected_rows(lo + idx, nm, ni, full))


def test_ba_jtj_cfg5_size(ctx):
    import torch
    prob = synth.make_ba_problem(500, 100_000, obs_per_pt=5, seed=5)
    nc, npt = prob["cams"].shape[0], prob["pts"].shape[0]
    pt_ptr, _ = sfmcore.csr_by(prob["pt_idx"], npt)
    cam_ptr, cam_obs = sfmcore.csr_by(prob["cam_idx"], nc)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    for loss_s in (0.0, 2.0):
        g = ctx.ba_jtj(T(prob["cams"]), T(prob["pp"]), T(prob["pts"]), T(prob["cam_idx"]),
                       T(prob["pt_idx"]), T(prob["uv"]), T(pt_ptr), T(cam_ptr), T(cam_obs),
                       loss_s=loss_s)
        torch.cuda.synchronize()
        g = {k: v.cpu().numpy() for k, v in g.items()}
        o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                     prob["uv"], loss_s=loss_s)
        np.testing.assert_allclose(g["res"], o["res"], rtol=0, atol=1e-4)   # north_star: 1e-4 px
        for k in ("U", "V", "W", "gc", "gp"):
            scale = np.abs(o[k]).max()
            np.testing.assert_allclose(g[k], o[k], rtol=1e-9, atol=1e-11 * scale, err_msg=k)
        assert abs(g["cost"][0] - o["cost"]) <= 1e-9 * abs(o["cost"])


@pytest.mark.parametrize("xc", [O.XC_OPENCV, O.XC_MUTUAL])
def test_hamming_k5000_valu_path_then_ransac(ctx, xc):
    import torch
    s = synth.make_scene(3, 5000, seed=21, orb=True)
    n_kp = np.array([5000, 4731, 4977], np.int32)            # ragged
    pairs = np.array([[0, 1], [2, 0], [1, 2]], np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    cnt, mt, dist = ctx.match_batch(T(s["desc"]), T(n_kp), T(pairs), metric=1, cross_check=xc,
                                    max_dist=26)
    rs = ctx.ransac_batch(T(s["kps"]), T(pairs), cnt, mt, n_hyp=1024, seed=42, thr=1.0)
    torch.cuda.synchronize()
    cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        q, t, d = O.match(s["desc"][a][:n_kp[a]], s["desc"][b][:n_kp[b]], metric=1,
                          cross_check=xc, max_dist=26)
        assert cnt[p] == len(q) > 100
        np.testing.assert_array_equal(mt[p, :cnt[p], 0], q)
        np.testing.assert_array_equal(mt[p, :cnt[p], 1], t)
        np.testing.assert_array_equal(dist[p, :cnt[p]], d)
        r = O.ransac_f(s["kps"][a][q], s["kps"][b][t], H=1024, seed=42, pa=int(a), pb=int(b))
        assert int(rs["inl_count"][p]) == r["count"] and int(rs["best_h"][p]) == r["best_h"]
        np.testing.assert_array_equal(rs["mask"][p, :cnt[p]].cpu().numpy(), r["mask"])


def test_one_context_two_streams():
    """Match on stream A, RANSAC on stream B, through ONE context (shared workspace), while
    stream A immediately launches another match that reuses the workspace: the hand-off in
    sfm_ctx_set_stream must order them.  Result == the serial result."""
    import torch
    ctx = sfmcore.context(0)
    s = synth.make_scene(12, 2048, seed=31)
    pairs = synth.unordered_pairs(12)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, kps, pt = T(s["desc"]), T(s["n_kp"]), T(s["kps"]), T(pairs)
    cnt, mt, _ = ctx.match_batch(desc, n_kp, pt, ratio=(4, 5))
    ref = ctx.ransac_batch(kps, pt, cnt, mt, n_hyp=4096)
    torch.cuda.synchronize()
    valid = torch.arange(2048, device="cuda")[None, :] < cnt[:, None]   # mask is defined < count
    ref = {k: v.clone() for k, v in ref.items()}
    ref["mask"] *= valid
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(sa):
            c2, m2, _ = ctx.match_batch(desc, n_kp, pt, ratio=(4, 5))
            ev = torch.cuda.Event()
            ev.record(sa)
        with torch.cuda.stream(sb):
            sb.wait_event(ev)
            r2 = ctx.ransac_batch(kps, pt, c2, m2, n_hyp=4096)
        with torch.cuda.stream(sa):  # no stream dependency on sb: only the workspace is shared
            _ = ctx.match_batch(desc, n_kp, pt, ratio=(4, 5),
                                out=(torch.empty_like(c2), torch.empty_like(m2),
                                     torch.empty((pt.shape[0], 2048), dtype=torch.int32,
                                                 device="cuda")))
        torch.cuda.synchronize()
        assert torch.equal(c2, cnt)
        r2["mask"] *= valid
        for k in ("inl_count", "best_h", "mask", "F"):
            assert torch.equal(r2[k], ref[k]), k


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_rccl_world1_graph_allgather_and_camera_allreduce():
    """The `nccl` (RCCL) branches of match_graph._gather / all_gather_rows / all_gather_graph and
    reconstruction.allreduce_camera_blocks, on device tensors in a world-size-1 group."""
    import torch
    import torch.distributed as dist
    assert not dist.is_initialized()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        scene = synth.make_scene(8, 1024, seed=41)
        pairs = synth.unordered_pairs(8)
        gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"], n_hyp=1024)
        pt = torch.from_numpy(pairs).cuda()
        count, match, _, rs = gb.run(pt)
        rows, offs = gb.graph_rows(0, count, match, rs, return_offsets=True)
        counts, packed = match_graph.pack_rows(rows, offs)
        g = match_graph.all_gather_graph(counts, packed, [(0, len(pairs))])
        assert g.is_cuda and torch.equal(g, rows) and rows.shape[0] > 1000
        t = torch.arange(37, dtype=torch.int32, device="cuda")
        assert torch.equal(match_graph._gather(t, 1, None)[0], t)
        assert torch.equal(match_graph.all_gather_rows(rows), rows)
        U = torch.randn(5, 8, 8, dtype=torch.float64, device="cuda")
        gc = torch.randn(5, 8, dtype=torch.float64, device="cuda")
        cost = torch.tensor([3.5], dtype=torch.float64, device="cuda")
        U0, gc0 = U.clone(), gc.clone()
        reconstruction.allreduce_camera_blocks(U, gc, cost)
        torch.cuda.synchronize()
        assert torch.equal(U, U0) and torch.equal(gc, gc0) and float(cost) == 3.5
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k,xc,ratio", [(8192, O.XC_MUTUAL, (4, 5)), (6000, O.XC_OPENCV, None),
                                        (5000, O.XC_MUTUAL, None)])
def test_l2_above_4096_cross_check_then_ransac(ctx, k, xc, ratio):
    """L2 k_max above 4096 (COLMAP-style 8192 SIFT): the column-winner kernel with its column
    state past 64 KB of LDS, ragged sizes, then RANSAC on the matches; vs the oracle."""
    import torch
    s = synth.make_scene(3, k, seed=23)
    n_kp = np.array([k, k - 371, k - 13], np.int32)
    pairs = np.array([[0, 1], [2, 0], [1, 2]], np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    cnt, mt, dist = ctx.match_batch(T(s["desc"]), T(n_kp), T(pairs), cross_check=xc, ratio=ratio)
    rs = ctx.ransac_batch(T(s["kps"]), T(pairs), cnt, mt, n_hyp=1024, seed=42, thr=1.0)
    torch.cuda.synchronize()
    cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        q, t, d = O.match(s["desc"][a][:n_kp[a]], s["desc"][b][:n_kp[b]], 0, xc, ratio)
        assert cnt[p] == len(q) > 1000
        np.testing.assert_array_equal(mt[p, :cnt[p], 0], q)
        np.testing.assert_array_equal(mt[p, :cnt[p], 1], t)
        np.testing.assert_array_equal(dist[p, :cnt[p]], d)
        r = O.ransac_f(s["kps"][a][q], s["kps"][b][t], H=1024, seed=42, pa=int(a), pb=int(b))
        assert int(rs["inl_count"][p]) == r["count"] and int(rs["best_h"][p]) == r["best_h"]
        np.testing.assert_array_equal(rs["mask"][p, :cnt[p]].cpu().numpy(), r["mask"])


def test_l2_above_4096_without_cross_check_refused(ctx):
    import torch
    d = torch.zeros((2, 5000, 128), dtype=torch.uint8, device="cuda")
    n = torch.full((2,), 5000, dtype=torch.int32, device="cuda")
    pr = torch.tensor([[0, 1]], dtype=torch.int32, device="cuda")
    with pytest.raises(sfmcore.SfmCoreError, match="cross-check"):
        ctx.match_batch(d, n, pr, cross_check=sfmcore.XC_NONE, ratio=(4, 5))


def _check_f64(scene, pairs, count, match, rs64, idx):
    """fp64 K2 (sfm_ransac_f_batch_f64) vs the oracle's *_f64 restatement, bit for bit."""
    sample = np.ascontiguousarray(pairs[idx])
    _, nm, ni, full = O.match_verify_batch(scene["desc"], scene["kps"].astype(np.float64),
                                           sample, ratio=(4, 5), H=H, seed=42, thr=1.0,
                                           min_inl=15, full=True, f64=True)
    inl, bh = rs64["inl_count"][idx], rs64["best_h"][idx]
    mask, F = rs64["mask"][idx], rs64["F"][idx]
    np.testing.assert_array_equal(count[idx], nm)
    for p in range(len(sample)):
        m = nm[p]
        np.testing.assert_array_equal(match[idx[p], :m], full["match"][p, :m])
        if m < 8:
            assert inl[p] == -1
            continue
        assert inl[p] == ni[p] and bh[p] == full["best_h"][p], f"pair {p}"
        np.testing.assert_array_equal(mask[p, :m], full["mask"][p, :m], err_msg=f"pair {p}")
        assert F[p].view(np.uint64).tolist() == full["F"][p].view(np.uint64).tolist(), p
    return ni


@pytest.mark.parametrize("cfg", ["cfg3", "cfg4_shard"])
def test_ransac_f64_mode_full_size(cfg):
    """fp64 verification mode: equal to the fp64 oracle bit for bit on all
    1225 cfg3 pairs and on a 96-pair sample of a cfg4 shard (K1 from the same launch)."""
    import torch
    n_img, k = (50, 2048) if cfg == "cfg3" else (500, 4096)
    scene = synth.make_scene(n_img, k, seed=0)
    pairs = synth.unordered_pairs(n_img)
    if cfg != "cfg3":
        lo, hi = match_graph.shard_range(pairs, 3, 8, scene["n_kp"])
        pairs = pairs[lo:hi]
    gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"], ratio=(4, 5),
                                  n_hyp=H, seed=42, thr=1.0, min_inliers=15)
    pt = torch.from_numpy(np.ascontiguousarray(pairs)).cuda()
    count, match, _ = gb.match(pt)
    kps64 = gb.kps.double().contiguous()
    rs = gb.ctx.ransac_batch(kps64, pt, count, match, n_hyp=H, seed=42, thr=1.0, min_inliers=15)
    rs32 = gb.verify(pt, count, match)
    torch.cuda.synchronize()
    rs = {k: v.cpu().numpy() for k, v in rs.items()}
    rs32 = {k: v.cpu().numpy() for k, v in rs32.items()}
    assert rs["F"].dtype == np.float64 and rs["norm"].dtype == np.float64
    idx = np.arange(len(pairs)) if cfg == "cfg3" else np.arange(0, len(pairs), len(pairs) // 96)[:96]
    _check_f64(scene, pairs, count.cpu().numpy(), match.cpu().numpy(), rs, idx)
    # f32 vs f64 specs: the verified sets differ only marginally
    diff = int((rs["inl_count"] != rs32["inl_count"]).sum())
    assert diff <= max(5, len(pairs) // 50), diff
