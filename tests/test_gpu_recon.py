"""GPU parity: feature tracks (sfm_tracks) and multi-view triangulation (sfm_triangulate) vs the
CPU restatement oracle/recon.py, and the matching → tracks → triangulation → bundle-adjustment
chain on a synthetic scene.

Tracks: exact (same tracks, same order, same nodes).  Triangulation: fp64, points within 1e-9 of
the scene scale (eigenvector by Jacobi on the GPU vs LAPACK eigh), statuses exact.
"""
import numpy as np
import pytest

import match_graph
import recon
import reconstruction as R
import synth

pytestmark = pytest.mark.gpu


def _random_graph(rng, n_img, k, n_rows):
    n_kp = rng.integers(k // 2, k, size=n_img).astype(np.int32)
    pairs = np.array([(a, b) for a in range(n_img) for b in range(a + 1, n_img)], np.int32)
    p = rng.integers(0, len(pairs), size=n_rows)
    q = rng.integers(0, n_kp[pairs[p, 0]])
    t = rng.integers(0, n_kp[pairs[p, 1]])
    return n_kp, pairs, np.stack([p, q, t], 1).astype(np.int32)


def _check_tracks(n_kp, pairs, rows, min_len):
    ptr, ti, tk = (t.cpu().numpy() for t in match_graph.build_tracks(rows, pairs, n_kp, min_len))
    base = np.r_[0, np.cumsum(n_kp)].astype(np.int32)
    optr, oti, otk = recon.tracks(base, pairs, rows, min_len)
    np.testing.assert_array_equal(ptr, optr)
    np.testing.assert_array_equal(ti, oti)
    np.testing.assert_array_equal(tk, otk)
    return ptr


@pytest.mark.parametrize("seed,n_img,k,n_rows,min_len", [
    (0, 6, 40, 300, 2), (1, 12, 200, 3000, 2), (2, 12, 200, 3000, 3), (3, 30, 500, 40000, 2)])
def test_tracks_match_oracle(seed, n_img, k, n_rows, min_len):
    rng = np.random.default_rng(seed)
    _check_tracks(*_random_graph(rng, n_img, k, n_rows), min_len)


def test_tracks_long_chain_and_empty():
    n_img = 300                                     # one 300-image chain: many hook rounds
    n_kp = np.full(n_img, 4, np.int32)
    pairs = np.array([(a, a + 1) for a in range(n_img - 1)], np.int32)
    rows = np.array([(p, 1, 1) for p in range(n_img - 1)][::-1], np.int32)
    ptr = _check_tracks(n_kp, pairs, rows, 2)
    assert len(ptr) == 2 and ptr[1] == n_img
    ptr, _, _ = match_graph.build_tracks(np.zeros((0, 3), np.int32), pairs, n_kp, 2)
    assert ptr.cpu().numpy().tolist() == [0]


def test_tracks_from_verified_graph():
    import torch
    scene = synth.make_scene(8, 512, seed=5)
    pairs = synth.unordered_pairs(8)
    gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"])
    count, match, _, rs = gb.run(torch.from_numpy(pairs).cuda())
    rows = gb.graph_rows(0, count, match, rs).cpu().numpy()
    ptr = _check_tracks(scene["n_kp"], pairs, rows, 2)
    assert len(ptr) > 100


def _noisy_problem(seed, n_cam=10, n_pt=400, k=4):
    prob = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=k, seed=seed, noise_px=0.5, perturb=0.0)
    ptr = np.r_[0, np.cumsum(np.bincount(prob["pt_idx"], minlength=n_pt))].astype(np.int32)
    return prob, ptr


def _gpu_triangulate(prob, ptr, cam_idx=None, uv=None):
    import torch
    ctx = R.sfmcore.context(0)
    T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).cuda()
    pts, st = ctx.triangulate(T(prob["cams"], np.float64), T(prob["pp"], np.float64),
                              T(ptr, np.int32),
                              T(prob["cam_idx"] if cam_idx is None else cam_idx, np.int32),
                              T(prob["uv"] if uv is None else uv, np.float64))
    return pts.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("seed", [0, 1])
def test_triangulate_matches_oracle(seed):
    prob, ptr = _noisy_problem(seed)
    g, gs = _gpu_triangulate(prob, ptr)
    o, os_ = recon.triangulate(prob["cams"], prob["pp"], ptr, prob["cam_idx"], prob["uv"])
    np.testing.assert_array_equal(gs[:, 3], os_[:, 3])
    np.testing.assert_allclose(g, o, rtol=0, atol=1e-9 * np.abs(o).max())
    np.testing.assert_allclose(gs[:, :3], os_[:, :3], rtol=1e-8, atol=1e-9)


def test_triangulate_status_codes():
    prob, ptr = _noisy_problem(2, n_pt=20)
    keep = np.r_[0, np.arange(4, len(prob["cam_idx"]))]
    ptr2 = np.r_[0, 1, ptr[2:] - 3].astype(np.int32)
    g, gs = _gpu_triangulate(prob, ptr2, prob["cam_idx"][keep], prob["uv"][keep])
    assert gs[0, 3] == 1 and np.all(gs[1:, 3] == 0)


def test_scene_to_bundle_adjustment():
    """matches -> verified graph -> tracks -> triangulation (true cameras, perturbed) -> LM."""
    import torch
    scene = synth.make_scene(8, 512, seed=6, k1_range=0.03)
    pairs = synth.unordered_pairs(8)
    gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"])
    count, match, _, rs = gb.run(torch.from_numpy(pairs).cuda())
    rows = gb.graph_rows(0, count, match, rs)
    ptr, ti, tk = match_graph.build_tracks(rows, pairs, scene["n_kp"], 3)
    cam_idx, pt_idx, uv = match_graph.tracks_to_observations(ptr, ti, tk, gb.kps)
    rng = np.random.default_rng(0)
    cams = scene["cams"].copy()
    cams[:, :6] += rng.normal(0, 1e-3, size=(8, 6))
    ctx = R.sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    pts, st = ctx.triangulate(T(cams), T(scene["pp"]), ptr, cam_idx, uv)
    ok = (st[:, 3] == 0) & (st[:, 0] < 8.0)          # drop tracks with a misplaced keypoint
    okn = ok.cpu().numpy()
    assert okn.mean() > 0.5
    # keep the good tracks' observations (point-major, renumbered)
    ptr_n, cam_n, uv_n = ptr.cpu().numpy(), cam_idx.cpu().numpy(), uv.cpu().numpy()
    sel = np.repeat(okn, np.diff(ptr_n))
    new_id = np.cumsum(okn) - 1
    pt_new = np.repeat(new_id, np.diff(ptr_n))[sel]
    p0 = pts.cpu().numpy()[okn]
    err0 = R.reprojection_errors(cams, scene["pp"], p0, cam_n[sel], pt_new, uv_n[sel])
    c2, p2, hist = R.bundle_adjust(cams, scene["pp"], p0, cam_n[sel], pt_new, uv_n[sel],
                                   loss_s=2.0, max_iter=30)
    assert any(h[2] for h in hist)
    err = R.reprojection_errors(c2, scene["pp"], p2, cam_n[sel], pt_new, uv_n[sel])
    assert np.median(err) < np.median(err0) and np.median(err) < 1.0   # px (noise 0.5 px)
