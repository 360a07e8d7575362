"""Seeded synthetic SfM scenes: cameras, 3D points, keypoints and descriptors.

The reference reads real photos (`code/pipeline.py:25`, `dataset/Bicycle/images`) and extracts ORB
features with OpenCV (`code/feature_matching.py:42-45`).  Neither the dataset nor `cv2` exists here,
so every benchmark and parity test starts at the descriptor level from this generator
(SURVEY.md §8d "Concrete synthetic inputs").

Scene model
-----------
* 3D points uniform in the box [-2, 2]^3 around the origin.
* Cameras on a 120-degree arc of radius 8 around the y axis, all looking at the origin;
  pinhole f = 1000 px, 1920x1080, principal point at the image centre, optional radial k1.
* Each image observes a random subset of the points (projection + N(0, noise_px) pixel noise) and is
  topped up to exactly K keypoints with uniform random outlier keypoints.  A `misplace_frac` share of
  the observed points is put at a random position while keeping the point's descriptor (repeated
  texture), so tentative matches contain geometric outliers for RANSAC to reject.  Keypoints are
  shuffled.
* SIFT-like descriptors: per point a base |N(0,1)|^128, L2-normalised, clipped at 0.2,
  renormalised, scaled to 512 and rounded into [0, 255].  Each view adds N(0, desc_noise), rounds
  and clips.  Outliers get independent bases.
* ORB-like descriptors: per point a random 256-bit base; each view flips every bit with p = 0.05.

Everything is drawn from numpy's PCG64 with the given seed, so scenes are reproducible on every
machine (the GPU box regenerates them from the seed instead of shipping data).
"""
from __future__ import annotations

import numpy as np

WIDTH, HEIGHT, FOCAL = 1920, 1080, 1000.0


def _look_at(center: np.ndarray) -> np.ndarray:
    """World->camera rotation for a camera at `center` looking at the origin (y up)."""
    z = -center / np.linalg.norm(center)
    up = np.array([0.0, 1.0, 0.0])
    x = np.cross(up, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z])  # rows = camera axes


def rotmat_to_angle_axis(R: np.ndarray) -> np.ndarray:
    cos = np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)
    theta = np.arccos(cos)
    if theta < 1e-12:
        return np.zeros(3)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return w * (theta / (2.0 * np.sin(theta)))


def angle_axis_to_rotmat(r: np.ndarray) -> np.ndarray:
    theta = np.linalg.norm(r)
    if theta < 1e-12:
        return np.eye(3)
    k = r / theta
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(theta) * K + (1 - np.cos(theta)) * K @ K


def project(R, t, f, k1, cx, cy, X):
    """Pinhole + one radial term; returns (N, 2) pixels and camera-frame depth."""
    P = X @ R.T + t
    p = P[:, :2] / P[:, 2:3]
    d = 1.0 + k1 * np.sum(p * p, axis=1, keepdims=True)
    return f * d * p + np.array([cx, cy]), P[:, 2]


def _sift_bases(rng, n):
    b = np.abs(rng.standard_normal((n, 128)))
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    b = np.minimum(b, 0.2)
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    return b * 512.0


def make_scene(n_img: int, n_kp: int, seed: int = 0, n_pts: int | None = None,
               inlier_frac: float = 0.7, noise_px: float = 0.5, desc_noise: float = 6.0,
               k1_range: float = 0.0, orb: bool = False, arc_deg: float = 120.0,
               misplace_frac: float = 0.25, window: int | None = None, grid=None,
               track_len: float | None = None) -> dict:
    """Build a scene; returns a dict of numpy arrays (see module docstring).

    window: if set, every 3-D point has a home cell among the camera positions (uniform, drawn from
    a separate stream so scenes without a window are unchanged) and only cameras within `window`
    cells of it can observe it: local overlap, as in a real image collection, instead of every
    camera seeing the whole point cloud.
    grid: (n_az, n_el, az_deg, el_deg) puts the cameras on a sphere-cap grid (azimuth-major, the
    first n_img of n_az x n_el positions, all looking at the origin) instead of the arc; the
    window is then 2-D.  Neighbouring views are az_deg / n_az and el_deg / n_el apart, which gives
    the triangulation angles an arc of 500 views (0.24 degrees apart) cannot.
    track_len: mean observations per point with a window (default: every camera of the window);
    n_pts then defaults to n_img * n_in / track_len and each camera observes a random n_in of its
    candidate points."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n_in = int(round(inlier_frac * n_kp))
    wcams = None
    if window is not None:
        wcams = (2 * window + 1) ** (2 if grid is not None else 1)
        track_len = float(wcams if track_len is None else track_len)
    if n_pts is None:
        n_pts = (max(int(1.5 * n_in), 16) if window is None
                 else max(int(np.ceil(n_img * n_in / track_len)), 16))
    if grid is not None:
        n_az, n_el, az_deg, el_deg = grid
        if n_az * n_el < n_img:
            raise ValueError("make_scene: grid has fewer positions than images")
        cell = np.stack([np.arange(n_img) // n_el, np.arange(n_img) % n_el], 1)
    else:
        n_az, n_el = n_img, 1
        cell = np.stack([np.arange(n_img), np.zeros(n_img, np.int64)], 1)
    home_key = None
    if window is not None:
        hr = np.random.Generator(np.random.PCG64([seed, 0x5EC]))
        ha = np.clip(np.rint(hr.uniform(-0.5, n_az - 0.5, size=n_pts)), 0, n_az - 1).astype(np.int64)
        he = (np.clip(np.rint(hr.uniform(-0.5, n_el - 0.5, size=n_pts)), 0, n_el - 1).astype(np.int64)
              if grid is not None else np.zeros(n_pts, np.int64))
        home_key = ha * n_el + he
        by_home = np.argsort(home_key, kind="stable")
        hs = home_key[by_home]
    pts = rng.uniform(-2.0, 2.0, size=(n_pts, 3))
    cx, cy = WIDTH / 2.0, HEIGHT / 2.0

    cams = np.zeros((n_img, 8))          # angle-axis(3), t(3), f, k1
    pp = np.tile(np.array([cx, cy]), (n_img, 1))
    Rs = []
    for i in range(n_img):
        if grid is not None:
            az = np.deg2rad(-az_deg / 2 + az_deg * (cell[i, 0] + 0.5) / n_az)
            el = np.deg2rad(-el_deg / 2 + el_deg * (cell[i, 1] + 0.5) / n_el)
            C = 8.0 * np.array([np.sin(az) * np.cos(el), np.sin(el), np.cos(az) * np.cos(el)])
        else:
            ang = np.deg2rad(-arc_deg / 2 + arc_deg * (i + 0.5) / n_img)
            C = 8.0 * np.array([np.sin(ang), 0.15 * np.cos(3 * ang), np.cos(ang)])
        R = _look_at(C)
        t = -R @ C
        Rs.append(R)
        cams[i, :3] = rotmat_to_angle_axis(R)
        cams[i, 3:6] = t
        cams[i, 6] = FOCAL
        cams[i, 7] = rng.uniform(-k1_range, k1_range) if k1_range > 0 else 0.0

    def candidates(i):
        """points whose home cell is within `window` cells of camera i's (sorted indices)"""
        out = []
        for da in range(-window, window + 1):
            a = cell[i, 0] + da
            if a < 0 or a >= n_az:
                continue
            lo_e = max(cell[i, 1] - window, 0) if grid is not None else 0
            hi_e = min(cell[i, 1] + window, n_el - 1) if grid is not None else 0
            out.append(by_home[np.searchsorted(hs, a * n_el + lo_e):
                               np.searchsorted(hs, a * n_el + hi_e, side="right")])
        return np.sort(np.concatenate(out))

    if orb:
        pbase = rng.integers(0, 256, size=(n_pts, 32), dtype=np.uint8)
    else:
        pbase = _sift_bases(rng, n_pts)

    kps = np.zeros((n_img, n_kp, 2), np.float32)
    desc = np.zeros((n_img, n_kp, 32 if orb else 128), np.uint8)
    pid = np.full((n_img, n_kp), -1, np.int32)
    for i in range(n_img):
        cand = candidates(i) if home_key is not None else slice(None)
        uv, z = project(Rs[i], cams[i, 3:6], cams[i, 6], cams[i, 7], cx, cy, pts[cand])
        vis_m = (z > 0) & (uv[:, 0] >= 0) & (uv[:, 0] < WIDTH) & (uv[:, 1] >= 0) & (uv[:, 1] < HEIGHT)
        vis = np.nonzero(vis_m)[0]
        if home_key is not None:
            vis, uv = cand[vis], uv[vis]
            uv_full = np.empty((n_pts, 2))
            uv_full[vis] = uv
            uv = uv_full
        sel = rng.choice(vis, size=min(n_in, vis.size), replace=False)
        n_out = n_kp - sel.size
        xy_in = uv[sel] + rng.normal(0.0, noise_px, size=(sel.size, 2))
        # repeated-texture confusers: the descriptor is the point's, the position is elsewhere
        mis = rng.random(sel.size) < misplace_frac
        xy_in[mis] = rng.uniform([0, 0], [WIDTH, HEIGHT], size=(int(mis.sum()), 2))
        xy = np.concatenate([xy_in, rng.uniform([0, 0], [WIDTH, HEIGHT], size=(n_out, 2))])
        ids = np.concatenate([sel, np.full(n_out, -1)]).astype(np.int32)
        if orb:
            d_in = pbase[sel]
            flips = rng.random((sel.size, 256)) < 0.05
            d_in = d_in ^ np.packbits(flips, axis=1)
            d_out = rng.integers(0, 256, size=(n_out, 32), dtype=np.uint8)
        else:
            d_in = pbase[sel] + rng.normal(0.0, desc_noise, size=(sel.size, 128))
            d_out = _sift_bases(rng, n_out)
        d = np.concatenate([d_in, d_out])
        if not orb:
            d = np.clip(np.rint(d), 0, 255).astype(np.uint8)
        perm = rng.permutation(n_kp)
        kps[i] = xy[perm].astype(np.float32)
        desc[i] = d[perm]
        pid[i] = ids[perm]
    return dict(kps=kps, desc=desc, point_ids=pid, cams=cams, pp=pp, pts=pts,
                n_kp=np.full(n_img, n_kp, np.int32))


def camera_centres(cams: np.ndarray) -> np.ndarray:
    """World-frame centres -R^T t of [n, 8] cameras (angle-axis, t, f, k1)."""
    return np.array([-angle_axis_to_rotmat(c[:3]).T @ c[3:6] for c in np.asarray(cams)])


def similarity_align(src: np.ndarray, dst: np.ndarray):
    """Umeyama: the similarity (s, R, t) minimising |s R src + t - dst| over point sets [n, 3]
    (a reconstruction is defined up to one; compare it with the scene's truth after this)."""
    ms, md = src.mean(0), dst.mean(0)
    a, b = src - ms, dst - md
    U, S, Vt = np.linalg.svd(b.T @ a / len(src))
    D = np.eye(3)
    D[2, 2] = np.sign(np.linalg.det(U @ Vt))
    Rm = U @ D @ Vt
    s = np.trace(np.diag(S) @ D) / (a * a).sum(1).mean()
    return s, Rm, md - s * Rm @ ms


def unordered_pairs(n_img: int) -> np.ndarray:
    """All a<b pairs in row-major order (the shard axis)."""
    a, b = np.triu_indices(n_img, k=1)
    return np.stack([a, b], axis=1).astype(np.int32)


def make_ba_problem(n_cam: int, n_pt: int, obs_per_pt: int = 5, seed: int = 0,
                    noise_px: float = 0.5, perturb: float = 1e-3) -> dict:
    """Bundle-adjustment observations: each point seen by `obs_per_pt` cameras
    (an int, or one count per point).

    Observations are grouped by point (point-major), the layout the BA kernels shard on.
    Camera/point parameters are perturbed from the truth so residuals are non-trivial.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    sc = make_scene(n_cam, 8, seed=seed, n_pts=8, k1_range=0.05)
    cams_true = sc["cams"]
    pp = sc["pp"]
    pts_true = rng.uniform(-2.0, 2.0, size=(n_pt, 3))
    # obs_per_pt: one count for every point, or a count per point (long and short tracks mixed)
    counts = np.broadcast_to(np.asarray(obs_per_pt, np.int64), (n_pt,))
    cam_idx = np.concatenate([np.sort(rng.choice(n_cam, size=int(counts[p]), replace=False))
                              for p in range(n_pt)] or [np.zeros(0, np.int64)]).astype(np.int32)
    pt_idx = np.repeat(np.arange(n_pt, dtype=np.int32), counts)
    uv = np.empty((cam_idx.size, 2))
    Rs = [angle_axis_to_rotmat(c[:3]) for c in cams_true]
    for c in range(n_cam):
        sel = np.nonzero(cam_idx == c)[0]
        uv[sel], _ = project(Rs[c], cams_true[c, 3:6], cams_true[c, 6], cams_true[c, 7],
                             pp[c, 0], pp[c, 1], pts_true[pt_idx[sel]])
    uv += rng.normal(0.0, noise_px, size=uv.shape)
    cams = cams_true.copy()
    cams[:, :6] += rng.normal(0.0, perturb, size=(n_cam, 6))
    pts = pts_true + rng.normal(0.0, 10 * perturb, size=pts_true.shape)
    return dict(cams=cams, pp=pp, pts=pts, cam_idx=cam_idx, pt_idx=pt_idx, uv=uv)


def make_image(H: int, W: int, seed: int = 0, n_shapes: int = 120) -> np.ndarray:
    """Grayscale u8 test image with corners for the ORB extractor: a smooth gradient background
    and `n_shapes` filled rectangles, triangles and discs of random intensity, lightly blurred,
    plus pixel noise.  Seeded (PCG64), so every machine draws the same image."""
    rng = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    img = 60.0 + 40.0 * (xx / max(W, 1)) + 30.0 * (yy / max(H, 1))
    for _ in range(n_shapes):
        kind = rng.integers(0, 3)
        cx, cy = rng.uniform(0, W), rng.uniform(0, H)
        r = rng.uniform(0.02, 0.08) * min(H, W) + 3
        val = rng.uniform(0, 255)
        if kind == 0:
            a = rng.uniform(0, np.pi)
            u = (xx - cx) * np.cos(a) + (yy - cy) * np.sin(a)
            v = -(xx - cx) * np.sin(a) + (yy - cy) * np.cos(a)
            m = (np.abs(u) < r) & (np.abs(v) < 0.6 * r)
        elif kind == 1:
            m = (xx - cx) ** 2 + (yy - cy) ** 2 < r * r
        else:
            p = rng.uniform(-r, r, size=(3, 2)) + [cx, cy]
            d = lambda i, j: ((p[j, 0] - p[i, 0]) * (yy - p[i, 1]) - (p[j, 1] - p[i, 1]) * (xx - p[i, 0]))
            s1, s2, s3 = d(0, 1), d(1, 2), d(2, 0)
            m = ((s1 >= 0) & (s2 >= 0) & (s3 >= 0)) | ((s1 <= 0) & (s2 <= 0) & (s3 <= 0))
        img[m] = val
    k = np.array([1.0, 4.0, 6.0, 4.0, 1.0]) / 16.0
    img = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, img)
    img = np.apply_along_axis(lambda c: np.convolve(c, k, mode="same"), 0, img)
    img += rng.normal(0.0, 2.0, size=img.shape)
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8))
