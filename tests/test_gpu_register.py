"""GPU parity: next-view registration (sfm_register_batch) vs oracle/sfm_oracle_reg.c.

RANSAC part bit-identical: the winning hypothesis (4h + root), its inlier count and mask.
Refined pose: within 1e-9 (rotation matrix entries) / 1e-9 relative (t) of the numpy
Gauss-Newton restatement (oracle/recon.py reg_refine).  Batch-composition invariance: an image
registered alone or inside a batch gives identical results.
"""
import numpy as np
import pytest

import oracle as O
import recon
import sfmcore

pytestmark = pytest.mark.gpu


def _image(rng, n, outlier_frac=0.4, k1=0.02):
    from scipy.spatial.transform import Rotation
    R = Rotation.random(random_state=int(rng.integers(1 << 30))).as_matrix()
    X = rng.uniform(-2, 2, size=(n, 3))
    t = rng.normal(size=3)
    t = t + np.array([0, 0, 8 - (X @ R.T + t)[:, 2].min()])
    intr = np.array([1000.0, k1, 960.0, 540.0])
    P = X @ R.T + t
    q = P[:, :2] / P[:, 2:]
    xy = intr[0] * (1 + intr[1] * (q * q).sum(1, keepdims=True)) * q + intr[2:]
    xy += rng.normal(0, 0.5, size=xy.shape)
    out = rng.random(n) < outlier_frac
    xy[out] = rng.uniform([0, 0], [1920, 1080], size=(int(out.sum()), 2))
    return dict(R=R, t=t, X=X, xy=xy, intr=intr)


def _gpu(images, ids, n_hyp=512, thr=3.0, refine=True):
    import torch
    ptr = np.r_[0, np.cumsum([len(im["xy"]) for im in images])].astype(np.int32)
    cat = lambda k: np.concatenate([im[k] for im in images]) if images else np.zeros((0, 3))
    T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).cuda()
    cams, cnt, key, mask = sfmcore.context(0).register_batch(
        T(ptr, np.int32), T(cat("xy"), np.float64), T(cat("X"), np.float64),
        T(np.stack([im["intr"] for im in images]), np.float64), T(ids, np.int32), n_hyp=n_hyp,
        thr=thr, seed=42, refine=refine)
    return cams.cpu().numpy(), cnt.cpu().numpy(), key.cpu().numpy(), mask.cpu().numpy(), ptr


def test_register_matches_oracle_bitwise():
    rng = np.random.default_rng(0)
    # sizes around the scoring kernel's correspondence slices (REG_SPLIT 4): 3 and 5 leave empty
    # or one-correspondence slices, 1000 is many per slice
    images = [_image(rng, n) for n in (300, 50, 1000, 7, 3, 5)]
    ids = np.array([3, 11, 5, 8, 2, 9], np.int32)
    cams, cnt, key, mask, ptr = _gpu(images, ids)
    for i, im in enumerate(images):
        o = O.reg_ransac(im["xy"], im["X"], im["intr"], img=int(ids[i]), n_hyp=512, seed=42,
                         thr=3.0)
        assert cnt[i] == o["count"] and key[i] == o["key"]
        np.testing.assert_array_equal(mask[ptr[i]:ptr[i + 1]], o["mask"])
        Rr, tr = recon.reg_refine(o["R"], o["t"], im["xy"], im["X"], im["intr"], o["mask"])
        np.testing.assert_allclose(recon._rotmat(cams[i, :3]), Rr, atol=1e-9)
        np.testing.assert_allclose(cams[i, 3:6], tr, rtol=1e-9, atol=1e-9)
        np.testing.assert_array_equal(cams[i, 6:], im["intr"][:2])
        if len(im["xy"]) >= 50:                      # accurate pose after refinement
            np.testing.assert_allclose(Rr, im["R"], atol=2e-3)


def test_register_failures_and_batch_invariance():
    rng = np.random.default_rng(1)
    good = _image(rng, 200)
    tiny = _image(rng, 2)
    cams, cnt, key, mask, _ = _gpu([tiny, good], np.array([0, 1], np.int32))
    assert cnt[0] == -1 and key[0] == -1 and np.all(cams[0] == 0)
    cams1, cnt1, key1, mask1, _ = _gpu([good], np.array([1], np.int32))
    assert cnt1[0] == cnt[1] and key1[0] == key[1]
    np.testing.assert_array_equal(cams1[0], cams[1])
    np.testing.assert_array_equal(mask1, mask[2:])
