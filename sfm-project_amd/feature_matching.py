"""Drop-in for the reference's code/feature_matching.py (Justin-Huber/SfM-project).

`pipeline.py` star-imports this module (code/pipeline.py:2) and uses `os`, `np`, `cv2`
(code/pipeline.py:14,15,19) and `extract_and_match` (code/pipeline.py:41).  The module keeps those
names and signatures; the arithmetic runs in libsfmcore's HIP kernels instead of OpenCV:
  * ORB extraction — cv2.ORB_create() + detectAndCompute at code/feature_matching.py:42-45 —
    is `sfm_orb_batch` (csrc/orb.hip; the build's integer-exact ORB spec, oracle/sfm_oracle_orb.c;
    parity against OpenCV itself unpinned), batched over images and done ONCE per image by
    `extract_all` / `pipeline_pair_matches` instead of 2 x N(N-1) times;
  * matching — cv2.BFMatcher(NORM_HAMMING, crossCheck=True).match at :48-50 — is
    `sfm_match_batch`.
Only image I/O and drawing (`read_img`, `extract_and_match_draw`) still need cv2.
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
        raise ImportError(f"{what} needs OpenCV (cv2) for image I/O / drawing, which is not "
                          "installed; extraction and matching run without it")


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
    md = _max_dist(metric, max_distance)
    d1 = np.ascontiguousarray(des1, np.uint8)
    d2 = np.ascontiguousarray(des2, np.uint8)
    k_max = max(d1.shape[0], d2.shape[0])
    desc = np.zeros((2, k_max, d1.shape[1]), np.uint8)
    desc[0, :d1.shape[0]] = d1
    desc[1, :d2.shape[0]] = d2
    ctx = sfmcore.context(device)
    dev = torch.device("cuda", device)
    # one host -> device copy (descriptors, counts, the pair) and one device -> host copy back
    head = np.zeros(64, np.int32)                 # 256 B: the descriptors stay 256-B aligned
    head[:4] = (d1.shape[0], d2.shape[0], 0, 1)   # n_kp of both, then the pair (0, 1)
    up = torch.from_numpy(np.concatenate([head.view(np.uint8), desc.reshape(-1)])).to(dev)
    meta = up[:256].view(torch.int32)
    cnt, mt, dist = ctx.match_batch(up[256:].view(desc.shape), meta[:2], meta[2:4].view(1, 2),
                                    metric=metric, cross_check=xc, ratio=ratio, max_dist=md)
    back = torch.cat([cnt[:1], mt[0].reshape(-1), dist[0]]).cpu().numpy()
    k = int(back[0])
    mt = back[1:1 + 2 * k_max].reshape(k_max, 2)[:k]
    dist = back[1 + 2 * k_max:1 + 3 * k_max][:k].astype(np.float64)
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


class Pair:
    """code/pipeline.py:6-9 record: img_inx_1, img_inx_2, matches."""

    def __init__(self, img_inx_1=None, img_inx_2=None, matches=None):
        self.img_inx_1 = img_inx_1
        self.img_inx_2 = img_inx_2
        self.matches = matches


def match_all_pairs(descriptors, norm: str = "hamming", cross_check=True,
                    max_distance=REFERENCE_MAX_HAMMING, ratio=None, ordered: bool = True,
                    sort: bool = True, device: int = 0, keypoint_counts=None):
    """The pair loop of code/pipeline.py:36-47 in one batched GPU call.

    descriptors: list of u8 [K_i, 32] (ORB) or [K_i, 128] (SIFT-like) arrays, one per image (None
    or empty for an image without keypoints).  For every ordered pair i != j (ordered=True, the
    reference's enumeration) or every i < j (ordered=False) the matches of
    match_descriptors(des_i, des_j, ...) are computed; pairs with no match are dropped, exactly
    as `if match:` at code/pipeline.py:42.  Returns a list of Pair(i, j, [DMatch]) in the
    reference's (i, j) order.  Ordered lists without a ratio test compute each unordered pair's
    distances once and read both orders from them (sfm_match_batch_both, bit-identical to
    matching (i, j) and (j, i) separately)."""
    import torch
    n = len(descriptors)
    dim = 32 if norm == "hamming" else 128
    ks = [0 if d is None else len(d) for d in descriptors]
    k_max = max(ks + [1])
    desc = np.zeros((n, k_max, dim), np.uint8)
    for i, d in enumerate(descriptors):
        if ks[i]:
            desc[i, :ks[i]] = np.asarray(d, np.uint8)
    metric = sfmcore.METRIC_HAMMING if norm == "hamming" else sfmcore.METRIC_L2
    xc = {True: sfmcore.XC_OPENCV, "opencv": sfmcore.XC_OPENCV, "mutual": sfmcore.XC_MUTUAL,
          False: sfmcore.XC_NONE, None: sfmcore.XC_NONE}[cross_check]
    if ratio is not None and not isinstance(ratio, tuple):
        ratio = _ratio_fraction(float(ratio))
    md = _max_dist(metric, max_distance)
    dev = torch.device("cuda", device)
    ctx = sfmcore.context(device)
    desc_t = torch.from_numpy(desc).to(dev)
    ks_t = torch.tensor(ks, dtype=torch.int32, device=dev)
    upper = np.stack(np.triu_indices(n, 1), axis=1).astype(np.int32).reshape(-1, 2)
    if ordered and ratio is None and k_max <= 4096 and len(upper):
        # one distance tile serves (i, j) and (j, i) (sfm_match_batch_both): the reference's
        # ordered enumeration at the cost of the unordered one
        cnt, mt, dist = ctx.match_batch_both(desc_t, ks_t, torch.from_numpy(upper).to(dev),
                                             metric=metric, cross_check=xc, max_dist=md)
        cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
        # slot of ordered (i, j): its unordered pair u = (min, max); forward if i < j
        slot = np.zeros((n, n), np.int64)
        u = np.arange(len(upper))
        slot[upper[:, 0], upper[:, 1]] = u
        slot[upper[:, 1], upper[:, 0]] = len(upper) + u
        pairs = np.array([(i, j) for i in range(n) for j in range(n) if i != j],
                         np.int32).reshape(-1, 2)
        sel = slot[pairs[:, 0], pairs[:, 1]]
        cnt, mt, dist = cnt[sel], mt[sel], dist[sel]
    else:
        pairs = np.array([(i, j) for i in range(n) for j in range(n)
                          if (i != j if ordered else i < j)], np.int32).reshape(-1, 2)
        if len(pairs) == 0:
            return []
        cnt, mt, dist = ctx.match_batch(desc_t, ks_t, torch.from_numpy(pairs).to(dev),
                                        metric=metric, cross_check=xc, ratio=ratio, max_dist=md)
        cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
    out = []
    for p, (i, j) in enumerate(pairs.tolist()):
        k = int(cnt[p])
        if k == 0:
            continue
        d = dist[p, :k].astype(np.float64)
        if metric == sfmcore.METRIC_L2:
            d = np.sqrt(d).astype(np.float32).astype(np.float64)
        ms = [DMatch(q, t, 0, dd) for (q, t), dd in zip(mt[p, :k].tolist(), d.tolist())]
        if sort:
            ms = sorted(ms, key=lambda x: x.distance)
        out.append(Pair(i, j, ms))
    return out


class KeyPoint:
    """cv2.KeyPoint-compatible record (pt, size, angle, response, octave, class_id)."""

    __slots__ = ("pt", "size", "angle", "response", "octave", "class_id")

    def __init__(self, x, y, size, angle=-1.0, response=0.0, octave=0, class_id=-1):
        self.pt = (float(x), float(y))
        self.size = float(size)
        self.angle = float(angle)
        self.response = float(response)
        self.octave = int(octave)
        self.class_id = int(class_id)

    def __repr__(self):
        return (f"<KeyPoint pt=({self.pt[0]:g}, {self.pt[1]:g}) size={self.size:g} "
                f"angle={self.angle:.2f} octave={self.octave}>")


ORB_DEFAULTS = dict(n_features=500, n_levels=8, scale_factor=1.2, fast_threshold=20)


def _orb_gpu(images, device=0, **kw):
    """GPU ORB over a list of grayscale u8 images; images of one size share one launch.
    Returns per image (kp [n,6] f32, desc [n,32] u8) numpy arrays."""
    import torch
    prm = dict(ORB_DEFAULTS, **kw)
    ctx = sfmcore.context(device)
    dev = torch.device("cuda", device)
    out = [None] * len(images)
    groups = {}
    for i, im in enumerate(images):
        groups.setdefault(np.asarray(im).shape, []).append(i)
    for shape, idx in groups.items():
        if len(shape) != 2:
            raise ValueError(f"ORB needs 2-D grayscale images, got shape {shape}")
        batch = torch.from_numpy(np.ascontiguousarray(
            np.stack([np.asarray(images[i], np.uint8) for i in idx]))).to(dev)
        kp, desc, cnt = ctx.orb_batch(batch, **prm)
        kp, desc, cnt = kp.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
        for j, i in enumerate(idx):
            out[i] = (kp[j, :cnt[j]], desc[j, :cnt[j]])
    return out


# The reference's loop (code/pipeline.py:38-41) calls extract_and_match on every ordered pair, i.e.
# 2 (N - 1) times per image; the drop-in extracts each distinct image once.  Entries are keyed by
# the image's content (shape + xxh3-128 of its bytes), so an image changed in place is a new key;
# LRU-bounded at ORB_CACHE_SIZE images (0 = no cache).  ORB is deterministic: a hit returns the
# arrays a fresh extraction would (read-only views).
ORB_CACHE_SIZE = 1024
_orb_cache = None


def _image_key(im):
    """(shape, 128-bit digest of the bytes): xxh3-128 when xxhash is importable, else hashlib's
    blake2b-128 (slower, same role; xxhash is an optional dependency of the drop-in)."""
    a = np.ascontiguousarray(np.asarray(im, np.uint8))
    try:
        import xxhash
    except ImportError:
        import hashlib
        return a.shape, "b2:" + hashlib.blake2b(a.data, digest_size=16).hexdigest()
    return a.shape, xxhash.xxh3_128_hexdigest(a.data)


def _orb_cached(images, device=0):
    """_orb_gpu with the default ORB parameters through the content-keyed LRU cache: the missing
    images are extracted in one batch."""
    global _orb_cache
    from collections import OrderedDict
    if ORB_CACHE_SIZE <= 0:
        return _orb_gpu(images, device)
    if _orb_cache is None:
        _orb_cache = OrderedDict()
    keys = [(device,) + _image_key(im) for im in images]
    miss = [i for i, k in enumerate(keys) if k not in _orb_cache]
    first = {}
    for i in miss:
        first.setdefault(keys[i], i)
    if first:
        fresh = _orb_gpu([images[i] for i in first.values()], device)
        for k, (kp, desc) in zip(first, fresh):
            kp.setflags(write=False)
            desc.setflags(write=False)
            _orb_cache[k] = (kp, desc)
    out = []
    for k in keys:
        _orb_cache.move_to_end(k)
        out.append(_orb_cache[k])
    while len(_orb_cache) > ORB_CACHE_SIZE:
        _orb_cache.popitem(last=False)
    return out


def _keypoints(kp):
    return [KeyPoint(k[0], k[1], k[2], k[3], k[4], int(k[5])) for k in kp]


def detect_and_compute(gray, nfeatures: int = 500, device: int = 0):
    """orb.detectAndCompute(gray, None) (code/feature_matching.py:44) on the GPU: returns
    ([KeyPoint], descriptors u8 [n,32] or None when nothing is found, as OpenCV)."""
    kp, desc = _orb_gpu([gray], device, n_features=nfeatures)[0]
    return _keypoints(kp), (desc if len(desc) else None)


def extract_all(images, nfeatures: int = 500, device: int = 0):
    """ORB once per image, batched on the GPU (the reference extracts 2 x N(N-1) times,
    code/pipeline.py:38-41 -> code/feature_matching.py:42-45): returns (keypoints, descriptors)
    lists."""
    res = _orb_gpu(list(images), device, n_features=nfeatures)
    return ([_keypoints(k) for k, _ in res], [d if len(d) else None for _, d in res])


def pipeline_pair_matches(images):
    """Drop-in for the whole loop of code/pipeline.py:36-47: ORB once per image, then every
    ordered pair matched with the reference's matcher (Hamming, crossCheck, distance < 26) in one
    batched GPU call.  Returns the reference's pair_matches list."""
    _, des = extract_all(images)
    return match_all_pairs(des)


def _max_dist(metric, max_distance):
    if max_distance is None:
        return -1
    if metric == sfmcore.METRIC_L2:
        return int(np.ceil(float(max_distance) ** 2))  # integer d^2: d < m  <=>  d^2 < ceil(m^2)
    return int(np.ceil(float(max_distance)))


def extract_and_match(gray1, gray2):
    """code/feature_matching.py:41-60: ORB on both images, BF Hamming + crossCheck, sorted,
    prefix with distance < 26 — extraction and matching on the GPU.  Each distinct image is
    extracted once across calls (content-keyed cache, ORB_CACHE_SIZE)."""
    (_, des1), (_, des2) = _orb_cached([gray1, gray2])
    return match_descriptors(des1, des2, "hamming", True, REFERENCE_MAX_HAMMING)


_RING3 = None


def _ring3():
    """Offsets of a radius-3 circle outline (midpoint rule), as cv2.circle draws it."""
    global _RING3
    if _RING3 is None:
        pts = set()
        x, y, d = 0, 3, 1 - 3
        while x <= y:
            for sx, sy in ((x, y), (y, x)):
                for a, b in ((sx, sy), (-sx, sy), (sx, -sy), (-sx, -sy)):
                    pts.add((a, b))
            if d < 0:
                d += 2 * x + 3
            else:
                d += 2 * (x - y) + 5
                y -= 1
            x += 1
        _RING3 = np.array(sorted(pts), np.int64)
    return _RING3


def draw_matches(gray1, kp1, gray2, kp2, matches, seed: int = 0):
    """numpy restatement of cv2.drawMatches(..., flags=NOT_DRAW_SINGLE_POINTS) for the debug path
    of code/feature_matching.py:34-35: the two images side by side (RGB), each match a random
    colour, a radius-3 circle at both keypoints and a 1-pixel line between them.  Returns
    uint8 [max(h1, h2), w1 + w2, 3]."""
    g1, g2 = np.asarray(gray1, np.uint8), np.asarray(gray2, np.uint8)
    h1, w1 = g1.shape[:2]
    h2, w2 = g2.shape[:2]
    out = np.zeros((max(h1, h2), w1 + w2, 3), np.uint8)
    out[:h1, :w1] = g1[..., None] if g1.ndim == 2 else g1
    out[:h2, w1:] = g2[..., None] if g2.ndim == 2 else g2
    H, W = out.shape[:2]
    rng = np.random.default_rng(seed)
    ring = _ring3()

    def put(xs, ys, col):
        ok = (xs >= 0) & (xs < W) & (ys >= 0) & (ys < H)
        out[ys[ok], xs[ok]] = col

    for m in matches:
        col = rng.integers(0, 256, 3, dtype=np.uint8)
        x1, y1 = (int(round(v)) for v in kp1[m.queryIdx].pt)
        x2, y2 = (int(round(v)) for v in kp2[m.trainIdx].pt)
        x2 += w1
        n = max(abs(x2 - x1), abs(y2 - y1)) + 1
        t = np.linspace(0.0, 1.0, n)
        put(np.rint(x1 + (x2 - x1) * t).astype(np.int64), np.rint(y1 + (y2 - y1) * t).astype(np.int64),
            col)
        for cx, cy in ((x1, y1), (x2, y2)):
            put(cx + ring[:, 0], cy + ring[:, 1], col)
    return out


def extract_and_match_draw(gray1, gray2):
    """code/feature_matching.py:15-37: as extract_and_match, then draws the matches
    (cv2.drawMatches when cv2 is present, else the numpy draw_matches) and shows them with
    matplotlib (a no-op on a headless backend).  Returns the cropped matches."""
    kp1, des1 = detect_and_compute(gray1)
    kp2, des2 = detect_and_compute(gray2)
    cropped = match_descriptors(des1, des2, "hamming", True, REFERENCE_MAX_HAMMING)
    if cv2 is not None:
        ck1 = [cv2.KeyPoint(k.pt[0], k.pt[1], k.size, k.angle, k.response, k.octave) for k in kp1]
        ck2 = [cv2.KeyPoint(k.pt[0], k.pt[1], k.size, k.angle, k.response, k.octave) for k in kp2]
        cvm = [cv2.DMatch(m.queryIdx, m.trainIdx, m.imgIdx, m.distance) for m in cropped]
        img = cv2.drawMatches(gray1, ck1, gray2, ck2, cvm, None,
                              flags=cv2.DrawMatchesFlags_NOT_DRAW_SINGLE_POINTS)
    else:
        img = draw_matches(gray1, kp1, gray2, kp2, cropped)
    try:
        import matplotlib.pyplot as plt
    except ImportError:  # drawing is a debug aid only
        plt = None
    if plt is not None:
        plt.imshow(img), plt.show()
    return cropped
