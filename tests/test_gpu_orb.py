"""GPU parity: ORB extraction (csrc/orb.hip, sfm_orb_batch) vs the CPU restatement
oracle/sfm_oracle_orb.c — bit-exact keypoints (positions, size, octave, Harris response) and
descriptors; angles (output only, atan2 in fp64 on both sides) within 1e-3 degrees.

Reference: code/feature_matching.py:42-45 (cv2.ORB_create + detectAndCompute).  Parity against
OpenCV itself is unpinned (no cv2 here); the spec is in the oracle's header."""
import numpy as np
import pytest

import oracle as O
import synth

pytestmark = pytest.mark.gpu


def _gpu_orb(ctx, imgs, **kw):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(imgs)).cuda()
    kp, desc, cnt = ctx.orb_batch(t, **kw)
    torch.cuda.synchronize()
    return kp.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()


def _check(img, kp, desc, n, **kw):
    okp, odesc, _ = O.orb(img, **{{"n_features": "nfeat", "n_levels": "nlevels",
                                    "scale_factor": "scale", "fast_threshold": "fast_thr"}[k]: v
                                   for k, v in kw.items()})
    assert n == len(okp)
    np.testing.assert_array_equal(kp[:n, [0, 1, 2, 4, 5]], okp[:, [0, 1, 2, 4, 5]])
    np.testing.assert_allclose(kp[:n, 3], okp[:, 3], rtol=0, atol=1e-3)
    np.testing.assert_array_equal(desc[:n], odesc)
    return n


def test_orb_batch_matches_oracle(ctx):
    imgs = np.stack([synth.make_image(480, 640, seed=s) for s in range(4)])
    kp, desc, cnt = _gpu_orb(ctx, imgs)
    for i in range(len(imgs)):
        assert _check(imgs[i], kp[i], desc[i], cnt[i]) == 500


def test_orb_full_hd_and_parameters(ctx):
    img = synth.make_image(1080, 1920, seed=7)[None]
    kp, desc, cnt = _gpu_orb(ctx, img)
    _check(img[0], kp[0], desc[0], cnt[0])
    kw = dict(n_features=1000, n_levels=5, scale_factor=1.5, fast_threshold=10)
    kp, desc, cnt = _gpu_orb(ctx, img, **kw)
    assert _check(img[0], kp[0], desc[0], cnt[0], **kw) > 900


@pytest.mark.parametrize("hw", [(257, 331), (719, 1283)])
def test_orb_odd_sizes(ctx, hw):
    """Widths and heights that are no multiple of the 64 x 32 tiles or the 64-B level pitch, two
    images per batch."""
    imgs = np.stack([synth.make_image(*hw, seed=s) for s in (21, 22)])
    kp, desc, cnt = _gpu_orb(ctx, imgs)
    for i in range(len(imgs)):
        assert _check(imgs[i], kp[i], desc[i], cnt[i]) > 0


@pytest.mark.parametrize("hw", [(100, 80), (61, 70), (40, 40)])
def test_orb_small_images(ctx, hw):
    """Levels without room inside the 31-pixel border detect nothing (fewer keypoints or 0)."""
    img = synth.make_image(*hw, seed=3, n_shapes=10)[None]
    kp, desc, cnt = _gpu_orb(ctx, img)
    _check(img[0], kp[0], desc[0], cnt[0])


def test_orb_flat_image_has_no_keypoints(ctx):
    img = np.full((1, 200, 300), 128, np.uint8)
    _, _, cnt = _gpu_orb(ctx, img)
    assert cnt[0] == 0


def test_orb_rotation_invariance(ctx):
    """rBRIEF with intensity-centroid orientation: the same corners found in a 90-degree rotated
    image carry nearly the same descriptors (a property check, not parity)."""
    import feature_matching as fm
    img = synth.make_image(480, 480, seed=11)
    rot = np.ascontiguousarray(np.rot90(img))
    kp, desc, cnt = _gpu_orb(ctx, np.stack([img, rot]))
    d0, d1 = desc[0, :cnt[0]], desc[1, :cnt[1]]
    ms = fm.match_descriptors(d0, d1, cross_check=True, max_distance=40)
    good = 0
    for m in ms:  # rot90 (counter-clockwise): (x, y) -> (y, W - 1 - x)
        x, y = kp[0, m.queryIdx, :2]
        xr, yr = kp[1, m.trainIdx, :2]
        good += abs(xr - y) < 2.5 and abs(yr - (479 - x)) < 2.5
    assert good > 150 and good > 0.8 * len(ms)


def test_extract_and_match_on_gpu_without_cv2():
    """The reference entry point code/feature_matching.py:41 end to end on the GPU: ORB on both
    images, BF Hamming + crossCheck, stable sort, `distance < 26`; image 2 is image 1 shifted, so
    every kept match must be the shift."""
    import feature_matching as fm
    img = synth.make_image(480, 640, seed=5)
    sh = np.zeros_like(img)
    sh[:, :-17] = img[:, 17:]
    sh[:, -17:] = img[:, -17:]
    ms = fm.extract_and_match(img, sh)
    assert len(ms) > 100
    assert all(a.distance <= b.distance for a, b in zip(ms, ms[1:]))
    assert all(m.distance < 26 for m in ms)
    kp1, _ = fm.detect_and_compute(img)
    kp2, _ = fm.detect_and_compute(sh)
    ok = sum(abs(kp1[m.queryIdx].pt[0] - 17 - kp2[m.trainIdx].pt[0]) < 1.5
             and abs(kp1[m.queryIdx].pt[1] - kp2[m.trainIdx].pt[1]) < 1.5 for m in ms)
    assert ok > 0.85 * len(ms)   # the rest: repeated texture and the replicated right margin


def test_extract_and_match_cache_is_transparent(monkeypatch):
    """The content-keyed ORB cache of extract_and_match returns what fresh extractions give: the
    same matches cached and uncached, and an image changed in place is re-extracted."""
    import feature_matching as fm
    img = synth.make_image(480, 640, seed=6)
    sh = np.zeros_like(img)
    sh[:, :-11] = img[:, 11:]
    monkeypatch.setattr(fm, "_orb_cache", None)
    first = fm.extract_and_match(img, sh)
    again = fm.extract_and_match(img, sh)            # both images from the cache
    back = fm.extract_and_match(sh, img)
    monkeypatch.setattr(fm, "ORB_CACHE_SIZE", 0)
    assert first == again == fm.extract_and_match(img, sh) and len(first) > 100
    assert back == fm.extract_and_match(sh, img)
    monkeypatch.setattr(fm, "ORB_CACHE_SIZE", 1024)
    sh[100:200, 100:300] = 255 - sh[100:200, 100:300]  # in place: a new cache key
    cached = fm.extract_and_match(img, sh)
    monkeypatch.setattr(fm, "ORB_CACHE_SIZE", 0)
    assert cached == fm.extract_and_match(img, sh) and cached != first


def test_extract_and_match_draw_without_cv2(monkeypatch):
    """The reference's debug entry (code/feature_matching.py:15-37) on the GPU with the numpy
    drawMatches: the same matches as extract_and_match, and the drawing shown (headless)."""
    import feature_matching as fm
    shown = []
    import matplotlib.pyplot as plt
    monkeypatch.setattr(plt, "show", lambda *a, **k: shown.append(True))
    img = synth.make_image(480, 640, seed=5)
    sh = np.zeros_like(img)
    sh[:, :-17] = img[:, 17:]
    ms = fm.extract_and_match_draw(img, sh)
    assert ms == fm.extract_and_match(img, sh) and len(ms) > 100
    assert shown


def test_orb_dense_texture_beyond_32768_survivors(ctx):
    """a heavily textured image whose level 0 has far more than 32768 NMS survivors
    (uniform noise: a strict 3x3 maximum every few pixels, ~10^5 at 1080p).  Every survivor enters
    the FAST top-2n_l selection (no per-level cap), so the keypoints cover the whole image instead
    of the upper rows; GPU == oracle (uncapped too)."""
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (1, 1080, 1920), dtype=np.uint8)
    kp, desc, cnt = _gpu_orb(ctx, img)
    n = _check(img[0], kp[0], desc[0], cnt[0])
    assert n == 500
    lvl0 = kp[0, :n][kp[0, :n, 5] == 0]
    assert len(lvl0) > 50
    # a 32768 cap in raster order would end around row 31 + 32768 / (~0.1 x 1858) ~ 200
    assert lvl0[:, 1].max() > 0.8 * 1080 and lvl0[:, 1].min() < 0.2 * 1080
