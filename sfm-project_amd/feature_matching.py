"""Drop-in for the reference's code/feature_matching.py (Justin-Huber/SfM-project).

`pipeline.py` star-imports this module (code/pipeline.py:2) and uses `os`, `np`, `cv2`
(code/pipeline.py:14,15,19) and `extract_and_match` (code/pipeline.py:41).  The module keeps those
names and signatures; the matching arithmetic — cv2.BFMatcher(NORM_HAMMING, crossCheck=True).match
at code/feature_matching.py:48-50 — runs in libsfmcore's HIP kernels instead of OpenCV.

Feature EXTRACTION (ORB, code/feature_matching.py:42-45) is out of the hot-path scope and still
needs OpenCV; this container has no cv2, so `extract_and_match` raises ImportError there while the
descriptor-level entry `match_descriptors` works on any uint8 descriptor arrays.
"""
from __future__ import annotations

import os  # noqa: F401  (re-exported: code/pipeline.py:14 uses os.listdir/os.path)

import numpy as np

try:  # re-exported: code/pipeline.py:15 calls cv2.imread
    import cv2  # type: ignore
except Exception:  # cv2 is not installed in this image
    cv2 = None

import sfmcore

# reference constants: code/feature_matching.py:29,55 (`distance < 26`), :22,48 (crossCheck=True)
REFERENCE_MAX_HAMMING = 26


class DMatch:
    """cv2.DMatch-compatible record (queryIdx, trainIdx, imgIdx, distance)."""

    __slots__ = ("queryIdx", "trainIdx", "imgIdx", "distance")

    def __init__(self, queryIdx: int, trainIdx: int, imgIdx: int = 0, distance: float = 0.0):
        self.queryIdx = int(queryIdx)
        self.trainIdx = int(trainIdx)
        self.imgIdx = int(imgIdx)
        self.distance = float(distance)

    def __repr__(self):
        return (f"<DMatch queryIdx={self.queryIdx} trainIdx={self.trainIdx} "
                f"imgIdx={self.imgIdx} distance={self.distance:g}>")

    def __eq__(self, other):
        return (isinstance(other, DMatch) and self.queryIdx == other.queryIdx
                and self.trainIdx == other.trainIdx and self.imgIdx == other.imgIdx
                and self.distance == other.distance)


def _require_cv2(what: str):
    if cv2 is None:
        raise ImportError(f"{what} needs OpenCV (cv2), which is not installed; use "
                          "match_descriptors() on precomputed descriptors")


def read_img(path):
    """code/feature_matching.py:9-11: grayscale read."""
    _require_cv2("read_img")
    return cv2.imread(path, 0)


def match_descriptors(des1, des2, norm: str = "hamming", cross_check: bool | str = True,
                      max_distance=REFERENCE_MAX_HAMMING, ratio=None, sort: bool = True,
                      device: int = 0):
    """BF-match two descriptor sets on the GPU; returns a list of DMatch.

    norm='hamming': u8 [K,32] ORB descriptors, distance = Hamming bits (the reference matcher).
    norm='l2':      u8 [K,128] SIFT-like descriptors, distance = Euclidean (sqrt of exact d^2).
    cross_check:    True / 'opencv' -> OpenCV BFMatcher(crossCheck=True) rule (the reference's);
                    'mutual' -> strict mutual nearest neighbours; False -> none.
    max_distance:   keep distance < max_distance (reference: 26 Hamming bits); None: no cut.
    ratio:          Lowe ratio as a float or (num, den); not combinable with the OpenCV rule.
    sort:           stable sort by distance (code/feature_matching.py:52).
    """
    import torch
    if des1 is None or des2 is None or len(des1) == 0 or len(des2) == 0:
        return []
    metric = sfmcore.METRIC_HAMMING if norm == "hamming" else sfmcore.METRIC_L2
    xc = {True: sfmcore.XC_OPENCV, "opencv": sfmcore.XC_OPENCV, "mutual": sfmcore.XC_MUTUAL,
          False: sfmcore.XC_NONE, None: sfmcore.XC_NONE}[cross_check]
    if ratio is not None and not isinstance(ratio, tuple):
        ratio = _ratio_fraction(float(ratio))
    if max_distance is None:
        md = -1
    elif metric == sfmcore.METRIC_L2:
        md = int(np.ceil(float(max_distance) ** 2))  # integer d^2: d < m  <=>  d^2 < ceil(m^2)
    else:
        md = int(np.ceil(float(max_distance)))
    d1 = np.ascontiguousarray(des1, np.uint8)
    d2 = np.ascontiguousarray(des2, np.uint8)
    k_max = max(d1.shape[0], d2.shape[0])
    desc = np.zeros((2, k_max, d1.shape[1]), np.uint8)
    desc[0, :d1.shape[0]] = d1
    desc[1, :d2.shape[0]] = d2
    ctx = sfmcore.context(device)
    dev = torch.device("cuda", device)
    cnt, mt, dist = ctx.match_batch(torch.from_numpy(desc).to(dev),
                                    torch.tensor([d1.shape[0], d2.shape[0]], dtype=torch.int32,
                                                 device=dev),
                                    torch.tensor([[0, 1]], dtype=torch.int32, device=dev),
                                    metric=metric, cross_check=xc, ratio=ratio, max_dist=md)
    k = int(cnt.cpu()[0])
    mt = mt[0, :k].cpu().numpy()
    dist = dist[0, :k].cpu().numpy().astype(np.float64)
    if metric == sfmcore.METRIC_L2:
        dist = np.sqrt(dist).astype(np.float32).astype(np.float64)
    out = [DMatch(q, t, 0, d) for (q, t), d in zip(mt.tolist(), dist.tolist())]
    if sort:
        out = sorted(out, key=lambda x: x.distance)
    return out


def _ratio_fraction(r: float):
    from fractions import Fraction
    f = Fraction(r).limit_denominator(1000)
    return (f.numerator, f.denominator)


def extract_and_match(gray1, gray2):
    """code/feature_matching.py:41-60: ORB on both images, BF Hamming + crossCheck, sorted,
    prefix with distance < 26.  Matching runs on the GPU; extraction needs cv2."""
    _require_cv2("extract_and_match")
    orb = cv2.ORB_create()
    kp1, des1 = orb.detectAndCompute(gray1, None)
    kp2, des2 = orb.detectAndCompute(gray2, None)
    return match_descriptors(des1, des2, "hamming", True, REFERENCE_MAX_HAMMING)


def extract_and_match_draw(gray1, gray2):
    """code/feature_matching.py:15-37: as extract_and_match, then draws the matches."""
    _require_cv2("extract_and_match_draw")
    import matplotlib.pyplot as plt
    orb = cv2.ORB_create()
    kp1, des1 = orb.detectAndCompute(gray1, None)
    kp2, des2 = orb.detectAndCompute(gray2, None)
    cropped = match_descriptors(des1, des2, "hamming", True, REFERENCE_MAX_HAMMING)
    cvm = [cv2.DMatch(m.queryIdx, m.trainIdx, m.imgIdx, m.distance) for m in cropped]
    img = cv2.drawMatches(gray1, kp1, gray2, kp2, cvm, None,
                          flags=cv2.DrawMatchesFlags_NOT_DRAW_SINGLE_POINTS)
    plt.imshow(img), plt.show()
    return cropped
