"""Fills the reference's empty code/geometric_verification.py (0 bytes; the pipeline's
"Geometric Verification" section at code/pipeline.py:60 is a bare comment).

`pipeline.py` star-imports this module (code/pipeline.py:3).  Verification is the build's spec
(after papers/schoenberger2016sfm.pdf §4.1): 8-point fundamental-matrix RANSAC,
`n_hyp` hypotheses per pair drawn by a counter-based RNG keyed (seed, a, b, h), Sampson error in
squared pixels below `thr`, best = max inlier count (lowest hypothesis id on ties); a pair is
verified when the count reaches `min_inliers`.  All arithmetic runs in libsfmcore (HIP).
"""
from __future__ import annotations

import numpy as np

import sfmcore

DEFAULT_HYPOTHESES = 4096
DEFAULT_SEED = 42
DEFAULT_THRESHOLD = 1.0   # Sampson error, px^2
DEFAULT_MIN_INLIERS = 15  # COLMAP's default N_F


def denormalize_F(Fn, norm) -> np.ndarray:
    """Pixel-space F = T2^T Fn T1 (fp64), unit Frobenius norm.  norm = (cx1,cy1,s1,cx2,cy2,s2)."""
    Fn = np.asarray(Fn, np.float64).reshape(3, 3)
    cx1, cy1, s1, cx2, cy2, s2 = [float(v) for v in norm]
    T1 = np.array([[s1, 0, -s1 * cx1], [0, s1, -s1 * cy1], [0, 0, 1.0]])
    T2 = np.array([[s2, 0, -s2 * cx2], [0, s2, -s2 * cy2], [0, 0, 1.0]])
    F = T2.T @ Fn @ T1
    n = np.linalg.norm(F)
    return F / n if n > 0 else F


def verify_pair(kp1, kp2, matches, pair=(0, 1), n_hyp=DEFAULT_HYPOTHESES, seed=DEFAULT_SEED,
                thr=DEFAULT_THRESHOLD, min_inliers=DEFAULT_MIN_INLIERS, device=0):
    """kp1/kp2: [K,2] pixel coordinates; matches: list of DMatch or [M,2] (query, train) array.

    Returns dict(F [3,3] pixel F, inliers [n] match indices (ascending), count, verified,
    best_h)."""
    import torch
    mt = _match_array(matches)
    k1, k2 = np.asarray(kp1, np.float32), np.asarray(kp2, np.float32)
    k_max = max(len(k1), len(k2), len(mt), 1)
    kps = np.zeros((2, k_max, 2), np.float32)
    kps[0, :len(k1)] = k1
    kps[1, :len(k2)] = k2
    match = np.zeros((1, k_max, 2), np.int32)
    match[0, :len(mt)] = mt
    dev = torch.device("cuda", device)
    ctx = sfmcore.context(device)
    # the RNG is keyed by the pair's image ids; pass them through as a 1-pair batch
    a, b = int(pair[0]), int(pair[1])
    n_img = max(a, b) + 1
    kps_full = np.zeros((n_img, k_max, 2), np.float32)
    kps_full[a] = kps[0]
    kps_full[b] = kps[1]
    # one int32 upload (pair, match count, 61 pad, matches) and one byte download of the results
    head = np.zeros(64, np.int32)
    head[:3] = (a, b, len(mt))
    up = torch.from_numpy(np.concatenate([head, match.reshape(-1)])).to(dev)
    out = ctx.ransac_batch(torch.from_numpy(kps_full).to(dev), up[:2].view(1, 2), up[2:3],
                           up[64:].view(1, k_max, 2), n_hyp=n_hyp, seed=seed, thr=thr,
                           min_inliers=min_inliers)
    M = len(mt)
    u8 = lambda t: t.reshape(-1).view(torch.uint8)
    back = torch.cat([u8(out["inl_count"][:1]), u8(out["best_h"][:1]), u8(out["F"][0]),
                      u8(out["norm"][0]), out["mask"][0, :M]]).cpu().numpy()
    cnt = int(back[0:4].view(np.int32)[0])
    best_h = int(back[4:8].view(np.int32)[0])
    F = denormalize_F(back[8:44].view(np.float32).copy(), back[44:68].view(np.float32).copy())
    mask = back[68:68 + M].astype(bool)
    return dict(F=F, inliers=np.nonzero(mask)[0], count=max(cnt, 0),
                verified=cnt >= min_inliers, best_h=best_h)


def _match_array(matches) -> np.ndarray:
    if len(matches) and hasattr(matches[0], "queryIdx"):
        return np.array([[m.queryIdx, m.trainIdx] for m in matches], np.int32).reshape(-1, 2)
    return np.asarray(matches, np.int32).reshape(-1, 2)


def verify_pairs(pair_matches, keypoints, n_hyp=DEFAULT_HYPOTHESES, seed=DEFAULT_SEED,
                 thr=DEFAULT_THRESHOLD, min_inliers=DEFAULT_MIN_INLIERS, device=0,
                 chunk=8192):
    """Verifies the reference's pair list (code/pipeline.py:36-47: Pair objects with img_inx_1,
    img_inx_2, matches; the ordered N(N-1) enumeration or any subset) in batched calls of at most
    `chunk` pairs (host and device buffers are [chunk, k_max] — constant memory however long the
    list): keypoints[i] = [K_i,2] pixel coordinates of image i.  Returns the verified
    subset (input order) with `.matches` reduced to the inliers (ascending match index) and `.F`
    (pixel F, unit norm) attached.  Results equal verify_pair on each pair (the RNG is keyed by the
    pair's image ids, so they depend neither on the batch nor on the chunking)."""
    import torch
    chunk = int(chunk)
    if chunk < 1:   # a non-positive chunk used to return no verified pair, silently
        raise ValueError(f"verify_pairs: chunk must be >= 1, got {chunk}")
    if not pair_matches:
        return []
    pairs = np.array([[int(pr.img_inx_1), int(pr.img_inx_2)] for pr in pair_matches], np.int32)
    n_img = int(pairs.max()) + 1
    kl = [np.asarray(keypoints[i], np.float32).reshape(-1, 2) for i in range(n_img)]
    counts = np.array([len(pr.matches) for pr in pair_matches], np.int32)
    k_max = max([len(k) for k in kl] + [int(counts.max()), 1])
    kps = np.zeros((n_img, k_max, 2), np.float32)
    for i, k in enumerate(kl):
        kps[i, :len(k)] = k
    dev = torch.device("cuda", device)
    ctx = sfmcore.context(device)
    kps_d = torch.from_numpy(kps).to(dev)
    verified = []
    for c0 in range(0, len(pair_matches), chunk):
        prs = pair_matches[c0:c0 + chunk]
        P = len(prs)
        match = np.zeros((P, k_max, 2), np.int32)
        for p, pr in enumerate(prs):
            m = _match_array(pr.matches)
            match[p, :len(m)] = m
        cc = counts[c0:c0 + P]
        out = ctx.ransac_batch(kps_d, torch.from_numpy(np.ascontiguousarray(pairs[c0:c0 + P])).to(dev),
                               torch.from_numpy(np.ascontiguousarray(cc)).to(dev),
                               torch.from_numpy(match).to(dev), n_hyp=n_hyp, seed=seed, thr=thr,
                               min_inliers=min_inliers)
        cnt = out["inl_count"].cpu().numpy()
        mask = out["mask"].cpu().numpy()
        Fn, nrm = out["F"].cpu().numpy(), out["norm"].cpu().numpy()
        for p, pr in enumerate(prs):
            if cnt[p] >= min_inliers:
                keep = np.nonzero(mask[p, :cc[p]])[0]
                pr.matches = [pr.matches[i] for i in keep]
                pr.F = denormalize_F(Fn[p], nrm[p])
                verified.append(pr)
    return verified
