"""CPU: the reference-facing host modules (drop-ins for code/feature_matching.py,
code/geometric_verification.py, code/3d_reconstruction.py) — names, records, argument handling,
and that nothing falls back to a CPU implementation when no GPU is present."""
import importlib

import numpy as np
import pytest

import feature_matching as fm
import geometric_verification as gv
import match_graph
import oracle as O
import reconstruction
import sfmcore
import synth


def test_star_export_names_of_reference_module():
    # code/pipeline.py:14,15,19,41 use os, cv2, np and extract_and_match from the star import
    for name in ("os", "np", "cv2", "extract_and_match", "extract_and_match_draw", "read_img"):
        assert hasattr(fm, name), name
    ns = {}
    exec("from feature_matching import *", ns)
    assert "extract_and_match" in ns and "np" in ns and "os" in ns


def test_3d_reconstruction_module_loads_under_reference_name():
    m = importlib.import_module("3d_reconstruction")
    assert hasattr(m, "build_jtj") and hasattr(m, "reprojection_errors")


def test_extract_and_match_needs_the_gpu_not_cv2():
    """Extraction and matching run on the GPU (no cv2 needed); without a device the product
    path fails loudly — there is no CPU fallback.  Image I/O and drawing still need cv2."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_gpu_orb.py")
    with pytest.raises(sfmcore.SfmCoreError, match="no CPU fallback"):
        fm.extract_and_match(np.zeros((8, 8), np.uint8), np.zeros((8, 8), np.uint8))
    if fm.cv2 is None:
        with pytest.raises(ImportError, match="OpenCV"):
            fm.read_img("x.png")


def test_dmatch_record():
    a = fm.DMatch(3, 7, 0, 12.0)
    assert (a.queryIdx, a.trainIdx, a.imgIdx, a.distance) == (3, 7, 0, 12.0)
    assert a == fm.DMatch(3, 7, 0, 12) and a != fm.DMatch(3, 8, 0, 12)
    assert "queryIdx=3" in repr(a)
    # the reference sorts with key=lambda x: x.distance (code/feature_matching.py:52), stably
    ms = [fm.DMatch(i, i, 0, d) for i, d in enumerate([5, 3, 5, 1])]
    assert [m.queryIdx for m in sorted(ms, key=lambda x: x.distance)] == [3, 1, 0, 2]


def test_empty_descriptor_sets_return_empty_list_without_device():
    # cv2 raises on None descriptors; the drop-in returns [] so pipeline.py drops the pair (:42)
    assert fm.match_descriptors(None, np.zeros((4, 32), np.uint8)) == []
    assert fm.match_descriptors(np.zeros((0, 32), np.uint8), np.zeros((4, 32), np.uint8)) == []


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    d = np.random.default_rng(0).integers(0, 256, (16, 32), dtype=np.uint8)
    with pytest.raises(sfmcore.SfmCoreError, match="no CPU fallback"):
        fm.match_descriptors(d, d)
    with pytest.raises(sfmcore.SfmCoreError):
        gv.verify_pair(np.zeros((8, 2)), np.zeros((8, 2)), np.zeros((8, 2), np.int32))
    with pytest.raises(sfmcore.SfmCoreError):
        match_graph.GraphBuilder(np.zeros((2, 8, 128), np.uint8), np.zeros((2, 8, 2), np.float32))


def test_ratio_fraction():
    assert fm._ratio_fraction(0.8) == (4, 5)
    assert fm._ratio_fraction(0.75) == (3, 4)
    n, d = fm._ratio_fraction(0.7)
    assert n / d == pytest.approx(0.7)


def test_denormalize_F_matches_pixel_epipolar_constraint():
    s = synth.make_scene(2, 256, seed=5)
    q, t, _ = O.match(s["desc"][0], s["desc"][1], 0, 1, (4, 5))
    x1, x2 = s["kps"][0][q], s["kps"][1][t]
    r = O.ransac_f(x1, x2, H=256, seed=42, pa=0, pb=1)
    assert r["count"] >= 15
    F = gv.denormalize_F(r["F"], r["norm"])
    assert np.linalg.norm(F) == pytest.approx(1.0)
    assert np.linalg.matrix_rank(F, tol=1e-6) == 2
    inl = r["mask"].astype(bool)
    h1 = np.c_[x1[inl], np.ones(inl.sum())].astype(np.float64)
    h2 = np.c_[x2[inl], np.ones(inl.sum())].astype(np.float64)
    a = h1 @ F.T
    b = h2 @ F
    alg = np.sum(h2 * a, axis=1)
    samp = alg ** 2 / (a[:, 0] ** 2 + a[:, 1] ** 2 + b[:, 0] ** 2 + b[:, 1] ** 2)
    assert np.median(samp) < 1.0


def test_rows_to_pairs_groups_by_pair():
    pairs = synth.unordered_pairs(4)
    rows = np.array([[2, 5, 6], [0, 1, 1], [2, 7, 8], [0, 3, 4]], np.int32)
    g = match_graph.rows_to_pairs(rows, pairs)
    assert [(a, b) for a, b, _ in g] == [tuple(pairs[0]), tuple(pairs[2])]
    np.testing.assert_array_equal(g[0][2], [[1, 1], [3, 4]])
    np.testing.assert_array_equal(g[1][2], [[5, 6], [7, 8]])
    assert match_graph.rows_to_pairs(np.zeros((0, 3), np.int32), pairs) == []


def test_csr_by_is_stable_grouping():
    idx = np.array([2, 0, 2, 1, 0], np.int32)
    ptr, order = sfmcore.csr_by(idx, 4)
    np.testing.assert_array_equal(ptr, [0, 2, 3, 5, 5])
    np.testing.assert_array_equal(order, [1, 4, 3, 0, 2])


def test_build_jtj_sharded_rejects_unsorted_observations():
    with pytest.raises(ValueError):
        reconstruction.build_jtj_sharded(np.zeros((1, 8)), np.zeros((1, 2)), np.zeros((2, 3)),
                                         [0, 0], [1, 0], np.zeros((2, 2)), 0, 1)


def test_graph_npz_roundtrip(tmp_path):
    pairs = synth.unordered_pairs(4)
    rows = np.array([[0, 1, 2], [0, 3, 4], [4, 5, 6]], np.int32)
    f = str(tmp_path / "g.npz")
    match_graph.save_graph(f, pairs, rows, n_kp=[10, 11, 12, 13], meta={"seed": 42})
    g = match_graph.load_graph(f)
    np.testing.assert_array_equal(g["rows"], rows)
    np.testing.assert_array_equal(g["pairs"], pairs)
    assert g["meta"] == {"seed": 42} and g["n_kp"].tolist() == [10, 11, 12, 13]
    assert [(a, b) for a, b, _ in g["pair_matches"]] == [tuple(pairs[0]), tuple(pairs[4])]


def test_pair_record_and_pipeline_entry_need_the_gpu():
    import torch
    p = fm.Pair(1, 2, [fm.DMatch(0, 1, 0, 3.0)])
    assert (p.img_inx_1, p.img_inx_2, len(p.matches)) == (1, 2, 1)
    k = fm.KeyPoint(3.0, 4.0, 31.0, 90.0, 1.5, 2)
    assert k.pt == (3.0, 4.0) and k.octave == 2 and k.class_id == -1
    if not torch.cuda.is_available():
        with pytest.raises(sfmcore.SfmCoreError):
            fm.pipeline_pair_matches([np.zeros((8, 8), np.uint8)] * 2)


def test_draw_matches_numpy():
    """numpy drawMatches (the cv2-free debug path): canvas layout, circles and line pixels in the
    match colour, single points not drawn."""
    import numpy as np
    import feature_matching as fm
    g1 = np.full((40, 50), 10, np.uint8)
    g2 = np.full((60, 30), 200, np.uint8)
    kp1 = [fm.KeyPoint(10, 20, 31), fm.KeyPoint(40, 5, 31)]
    kp2 = [fm.KeyPoint(5, 50, 31), fm.KeyPoint(20, 10, 31)]
    img = fm.draw_matches(g1, kp1, g2, kp2, [fm.DMatch(0, 1, 0, 3.0)])
    assert img.shape == (60, 80, 3) and img.dtype == np.uint8
    assert (img[50:, :50] == 0).all()                     # below image 1: empty
    col = img[20, 13]                                     # ring point (r = 3) right of kp1[0]
    assert not (col == 10).all()
    assert (img[10, 50 + 23] == col).all()                # ring of kp2[1] (shifted by w1 = 50)
    assert (img[15, 41] == col).all()                     # on the line (10,20) -> (70,10)
    assert (img[5, 43] == 10).all() and (img[50, 58] == 200).all()  # unmatched points not drawn


def test_csr_by_device_equals_host_csr():
    """BAProblem builds its CSR indices with torch's stable sort (sfmcore.csr_by_device); the
    result is the host csr_by's, bit for bit (run here on CPU tensors)."""
    import torch
    rng = np.random.default_rng(4)
    for n, m in ((7, 0), (1, 5), (500, 20000), (3, 1000)):
        idx = rng.integers(0, n, m).astype(np.int32)
        ptr, order = sfmcore.csr_by(idx, n)
        dptr, dorder = sfmcore.csr_by_device(torch.from_numpy(idx), n)
        np.testing.assert_array_equal(dptr.numpy(), ptr)
        np.testing.assert_array_equal(dorder.numpy(), order)
        # the point CSR of a point-major problem (ascending index: a searchsorted)
        sidx = np.sort(idx)
        np.testing.assert_array_equal(
            sfmcore.csr_ptr_device(torch.from_numpy(sidx), n, ascending=True).numpy(), ptr)


@pytest.mark.parametrize("kw,digest", [
    (dict(n_img=5, n_kp=300, seed=3), "0fa28c8d2d4c31a4"),
    (dict(n_img=4, n_kp=256, seed=13, orb=True), "3651d5334fb017ee"),
    (dict(n_img=6, n_kp=200, seed=21, k1_range=0.02), "1c3760a59af7cc39"),
])
def test_default_scenes_unchanged(kw, digest):
    """Round 4 added local visibility to synth.make_scene (window / grid / track_len) from a
    separate random stream: scenes without a window keep every descriptor and point id (the
    fixtures and the committed bench checksums depend on them)."""
    import hashlib
    s = synth.make_scene(**kw)
    h = hashlib.sha256(np.ascontiguousarray(s["desc"]).tobytes()
                       + np.ascontiguousarray(s["point_ids"]).tobytes()).hexdigest()[:16]
    assert h == digest


def test_grid_scene_local_visibility():
    """cfg5's scene shape: views on a sphere-cap grid, each point observed by ~track_len of the
    3 x 3 views around its home cell, and only those."""
    n_az, n_el = 8, 4
    s = synth.make_scene(32, 400, seed=5, window=1, grid=(n_az, n_el, 60.0, 20.0), track_len=5)
    pid = s["point_ids"]
    cnt = np.bincount(pid[pid >= 0].ravel(), minlength=len(s["pts"]))
    assert abs(cnt[cnt > 0].mean() - 5.0) < 0.6
    cell = np.stack([np.arange(32) // n_el, np.arange(32) % n_el], 1)
    for p in np.nonzero(cnt >= 2)[0][:200]:
        views = np.nonzero((pid == p).any(1))[0]
        span = cell[views].max(0) - cell[views].min(0)
        assert (span <= 2).all()          # all observers within one 3 x 3 window
    c = synth.camera_centres(s["cams"])
    d01 = np.linalg.norm(c[1] - c[0])     # elevation neighbours: 20/4 = 5 degrees at radius 8
    assert abs(d01 - 2 * 8 * np.sin(np.deg2rad(2.5))) < 1e-9


def _track_arrays(rng, n_tr=400, n_img=20):
    lens = rng.integers(1, 7, n_tr)
    tptr = np.r_[0, np.cumsum(lens)].astype(np.int64)
    obs_track = np.repeat(np.arange(n_tr), lens)
    timg = rng.integers(0, n_img, len(obs_track)).astype(np.int64)
    return tptr, obs_track, timg


def test_track_obs_equals_host_gather():
    """incremental.track_obs (the device-side observation selection of the triangulation step)
    equals the host CSR gather it replaced, on CPU tensors."""
    import torch
    import incremental
    rng = np.random.default_rng(3)
    tptr, obs_track, timg = _track_arrays(rng)
    n_tr = len(tptr) - 1
    for trial in range(4):
        tracks = np.sort(rng.choice(n_tr, size=int(rng.integers(1, n_tr)), replace=False))
        imgs = rng.choice(20, size=int(rng.integers(1, 20)), replace=False)
        in_img = np.zeros(20, bool)
        in_img[imgs] = True
        lens = tptr[tracks + 1] - tptr[tracks]
        start = np.r_[0, np.cumsum(lens)[:-1]]
        o_ref = np.arange(int(lens.sum())) + np.repeat(tptr[tracks] - start, lens)
        keep = in_img[timg[o_ref]]
        o_ref = o_ref[keep]
        per = np.bincount(np.repeat(np.arange(len(tracks)), lens)[keep], minlength=len(tracks))
        ptr_ref = np.r_[0, np.cumsum(per)].astype(np.int32)
        o, ptr = incremental.track_obs(torch.from_numpy(obs_track), torch.from_numpy(timg), n_tr,
                                       torch.from_numpy(tracks), torch.from_numpy(in_img))
        np.testing.assert_array_equal(o.numpy(), o_ref)
        np.testing.assert_array_equal(ptr.numpy(), ptr_ref)
        assert ptr.dtype == torch.int32


def test_registration_obs_equals_host_selection():
    """incremental.registration_obs equals the host selection it replaced (observations of
    triangulated tracks in unregistered images, grouped by image, images with >= min_corr)."""
    import torch
    import incremental
    rng = np.random.default_rng(4)
    tptr, obs_track, timg = _track_arrays(rng, n_tr=3000)
    for trial in range(4):
        has_point = rng.random(len(tptr) - 1) < 0.6
        registered = rng.random(20) < 0.4
        obs_sel = np.nonzero(has_point[obs_track] & ~registered[timg])[0]
        obs_sel = obs_sel[np.argsort(timg[obs_sel], kind="stable")]
        img_u, img_n = np.unique(timg[obs_sel], return_counts=True)
        thr = int(np.median(img_n)) + 1            # some candidate images kept, some not
        keep = img_n >= thr
        assert keep.any() and not keep.all()
        sel, ids, cptr = incremental.registration_obs(
            torch.from_numpy(obs_track), torch.from_numpy(timg), torch.from_numpy(has_point),
            torch.from_numpy(registered), min_corr=thr)
        np.testing.assert_array_equal(ids, img_u[keep])
        np.testing.assert_array_equal(cptr, np.r_[0, np.cumsum(img_n[keep])])
        np.testing.assert_array_equal(sel.numpy(), obs_sel[np.repeat(keep, img_n)])
        assert ids.dtype == np.int32 and cptr.dtype == np.int32


def test_point_mean_equals_host_bincount():
    """incremental.point_mean (device-side reprojection filter of the bundle adjustments) gives
    numpy.bincount(pt_idx, err) / max(count, 1) bit for bit on runs of observations."""
    import torch
    import incremental
    rng = np.random.default_rng(5)
    lens = rng.integers(1, 12, 3000)
    pt_idx = np.repeat(np.arange(len(lens)), lens)
    err = rng.gamma(1.0, 1.5, len(pt_idx)) * np.exp(rng.normal(0, 3, len(pt_idx)))
    ref = np.bincount(pt_idx, err, minlength=len(lens)) / np.maximum(
        np.bincount(pt_idx, minlength=len(lens)), 1)
    first = np.ones(len(pt_idx), bool)
    first[1:] = pt_idx[1:] != pt_idx[:-1]
    got = incremental.point_mean(torch.from_numpy(err), torch.from_numpy(first)).numpy()
    np.testing.assert_array_equal(got.view(np.uint64), ref.view(np.uint64))


def test_orb_cache_extracts_each_distinct_image_once(monkeypatch):
    """extract_and_match's content-keyed ORB cache (the reference loop calls it 2 (N-1) times per
    image): one extraction per distinct image content, duplicates inside a call extracted once,
    an in-place change is a new key, LRU-bounded, read-only cached arrays."""
    calls = []

    def fake_orb(images, device=0, **kw):
        calls.append(len(images))
        return [(np.full((3, 6), float(im.sum()), np.float32),
                 np.full((3, 32), int(im.sum()) % 251, np.uint8)) for im in images]

    monkeypatch.setattr(fm, "_orb_gpu", fake_orb)
    monkeypatch.setattr(fm, "_orb_cache", None)
    monkeypatch.setattr(fm, "ORB_CACHE_SIZE", 3)
    rng = np.random.default_rng(0)
    a, b, c, d = (rng.integers(0, 255, (40, 60), dtype=np.uint8) for _ in range(4))
    r1 = fm._orb_cached([a, b])
    assert calls == [2]
    r2 = fm._orb_cached([b, a, a])
    assert calls == [2] and r2[1][1] is r1[0][1] and r2[0][1] is r1[1][1]
    assert not r1[0][1].flags.writeable
    a2 = a.copy()
    a2[0, 0] ^= 1                                   # same shape, different content
    fm._orb_cached([a2, a2])
    assert calls == [2, 1]
    fm._orb_cached([c, d])                          # 5 distinct keys > 3: the oldest go
    assert calls == [2, 1, 2] and len(fm._orb_cache) == 3
    fm._orb_cached([b])                             # evicted (least recently used)
    assert calls == [2, 1, 2, 1]
    monkeypatch.setattr(fm, "ORB_CACHE_SIZE", 0)
    fm._orb_cached([c])
    assert calls == [2, 1, 2, 1, 1]


def test_verify_pairs_rejects_non_positive_chunk():
    """chunk <= 0 raises (it used to give empty slices: no verified pair, silently)."""
    import geometric_verification as gv
    for c in (0, -3):
        with pytest.raises(ValueError, match="chunk must be >= 1"):
            gv.verify_pairs([object()], [np.zeros((1, 2))], chunk=c)


def test_image_key_without_xxhash(monkeypatch):
    """the ORB cache key falls back to blake2b-128 when xxhash is not importable; equal
    images give equal keys, a changed pixel a different key."""
    import builtins
    import feature_matching as fm
    real = builtins.__import__

    def no_xxhash(name, *a, **k):
        if name == "xxhash":
            raise ImportError("no xxhash")
        return real(name, *a, **k)
    monkeypatch.setattr(builtins, "__import__", no_xxhash)
    im = np.arange(64, dtype=np.uint8).reshape(8, 8)
    k1, k2 = fm._image_key(im), fm._image_key(im.copy())
    im2 = im.copy()
    im2[3, 3] ^= 1
    assert k1 == k2 and k1[1].startswith("b2:") and fm._image_key(im2) != k1


def test_shard_cuts_device_equals_shard_points():
    """the sharded BA's cuts come from the device (torch ops; run here on CPU
    tensors) and equal reconstruction.shard_points of the host CSR for every rank, including
    empty points, one heavy point and more ranks than points."""
    import torch
    rng = np.random.default_rng(5)
    for n_pt, n_obs in ((1000, 5000), (7, 40), (3, 2), (50, 0)):
        pt = np.sort(rng.integers(0, n_pt, n_obs)).astype(np.int32)
        if n_obs > 10:
            pt[n_obs // 3: n_obs // 2] = pt[n_obs // 3]       # a heavy point
        ptr, _ = sfmcore.csr_by(pt, n_pt)
        for world in (1, 2, 3, 4, 8):
            cuts, ocuts = reconstruction.shard_cuts_device(torch.from_numpy(pt), n_pt, world)
            exp = [reconstruction.shard_points(ptr, r, world) for r in range(world)]
            assert [(cuts[r], cuts[r + 1]) for r in range(world)] == exp
            assert ocuts == [int(ptr[c]) for c in cuts]


def test_track_observations_equal_host_build():
    """incremental.track_observations (the driver's device build of the track observation arrays)
    gives the host numpy build it replaced — np.repeat of the track ids, np.take of the keypoint
    rows as f64 — element for element (CPU tensors here), for f32 and f64 keypoints."""
    import torch
    import incremental
    rng = np.random.default_rng(9)
    n_img, K = 7, 50
    lens = rng.integers(2, 6, 40)
    ptr = np.r_[0, np.cumsum(lens)].astype(np.int32)
    img = rng.integers(0, n_img, ptr[-1]).astype(np.int32)
    kp = rng.integers(0, K, ptr[-1]).astype(np.int32)
    for dt in (np.float32, np.float64):
        kps = (rng.random((n_img, K, 2)) * 1000).astype(dt)
        otr, oimg, oxy = incremental.track_observations(torch.from_numpy(ptr), torch.from_numpy(img),
                                                        torch.from_numpy(kp), torch.from_numpy(kps))
        np.testing.assert_array_equal(otr.numpy(), np.repeat(np.arange(len(lens)), lens))
        np.testing.assert_array_equal(oimg.numpy(), img.astype(np.int64))
        ref = np.take(kps.reshape(-1, 2), img.astype(np.int64) * K + kp, axis=0).astype(np.float64)
        np.testing.assert_array_equal(oxy.numpy(), ref)
        assert oxy.dtype == torch.float64


def test_reconstruction_host_views_are_read_only_copies():
    """The driver keeps points / flags on the device (Reconstruction.pts_d / has_d); .points and
    .has_point are host copies that refuse writes (a write to a copy would be lost)."""
    import torch
    import incremental
    rec = incremental.Reconstruction(3)
    assert rec.points is None and rec.has_point is None
    rec.pts_d = torch.arange(12, dtype=torch.float64).reshape(4, 3)
    rec.has_d = torch.tensor([True, False, True, False])
    np.testing.assert_array_equal(rec.points, np.arange(12.0).reshape(4, 3))
    np.testing.assert_array_equal(rec.has_point, [True, False, True, False])
    with pytest.raises(ValueError):
        rec.points[0, 0] = 1.0
    with pytest.raises(ValueError):
        rec.has_point[1] = True
