"""Incremental structure from motion over the GPU core ("rest of incremental
SfM for cfg5" — the pipeline papers/schoenberger2016sfm.pdf §2.1-2.2 describes and the reference's
empty code/3d_reconstruction.py would hold).

Every per-element stage runs on the GPU through the C-ABI: all-pairs matching (K1), F RANSAC (K2),
verified-graph rows, tracks (`sfm_tracks`), triangulation (`sfm_triangulate`), batched next-view
registration (`sfm_register_batch`, P3P RANSAC + refinement) and Levenberg-Marquardt bundle
adjustment (`sfm_ba_jtj` / `sfm_ba_solve`).  The host does the orchestration: which images and
tracks enter the model, and the one 3x3 essential-matrix decomposition of the initial pair (an
8-point fit on that pair's inliers, O(1) work with no GPU counterpart).

Cameras: angle-axis, t, f, k1 with known intrinsics (f, k1, principal point) per image.
"""
from __future__ import annotations

import os

import numpy as np

import match_graph
import reconstruction
import sfmcore


def _undistort(xy, intr, iters=10):
    """Normalised, undistorted coordinates (the triangulation kernel's fixed-point spec)."""
    f, k1, cx, cy = intr
    xd = (np.asarray(xy, np.float64) - [cx, cy]) / f
    x = xd.copy()
    for _ in range(iters):
        x = xd / (1.0 + k1 * np.sum(x * x, axis=1, keepdims=True))
    return x


def _angle_axis(R):
    c = np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = 0.5 * np.linalg.norm(w)
    th = np.arctan2(s, c)
    return w * (th / (2.0 * s)) if s > 1e-12 else 0.5 * w


def relative_pose(x1, x2):
    """Pose (R, t), |t| = 1, of camera 2 w.r.t. camera 1 from normalised correspondences: linear
    essential matrix on all pairs, projected to the essential manifold; the four decompositions
    are returned for the cheirality vote."""
    A = np.stack([x2[:, 0] * x1[:, 0], x2[:, 0] * x1[:, 1], x2[:, 0],
                  x2[:, 1] * x1[:, 0], x2[:, 1] * x1[:, 1], x2[:, 1],
                  x1[:, 0], x1[:, 1], np.ones(len(x1))], 1)
    E = np.linalg.svd(A)[2][-1].reshape(3, 3)
    U, _, Vt = np.linalg.svd(E)
    if np.linalg.det(U) < 0:
        U = -U
    if np.linalg.det(Vt) < 0:
        Vt = -Vt
    W = np.array([[0.0, -1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    out = []
    for R in (U @ W @ Vt, U @ W.T @ Vt):
        for t in (U[:, 2], -U[:, 2]):
            out.append((R, t / np.linalg.norm(t)))
    return out


class Reconstruction:
    def __init__(self, n_img):
        self.timings = {}          # wall seconds per stage (each stage ends in a device sync)
        self.cams = np.zeros((n_img, 8))
        self.registered = np.zeros(n_img, bool)
        self.pts_d = None          # device [n_tr, 3] f64 points and [n_tr] bool flags: the driver
        self.has_d = None          # keeps them on the GPU; .points / .has_point are host copies
        self.history = []
        self.ba_log = []           # per bundle adjustment: size, LM / CG iterations, PCG branch
        self.n_verified = 0        # rows of the verified match graph
        self.obs_d = None          # device (obs_track, timg, obs_xy) of the track observations
        self.gauge = None          # (reference camera, scale camera) of the initial pair
        self._tracks_d = None      # device (ptr, img, kp) of the tracks; host copies on first use
        self._tracks = None

    @property
    def tracks(self):
        """(ptr [n_tr + 1], img [n_obs], kp [n_obs]) host arrays of the tracks (copied from the
        device on first use: the reconstruction itself never reads them on the host)."""
        if self._tracks is None and self._tracks_d is not None:
            self._tracks = tuple(t.cpu().numpy() for t in self._tracks_d)
        return self._tracks

    @tracks.setter
    def tracks(self, v):
        self._tracks, self._tracks_d = v, None

    @property
    def points(self):
        """[n_tr, 3] host copy of the track points (valid where has_point); read-only — the model
        lives in pts_d, so writing to a copy would be lost (write to pts_d instead).  The copy is
        cached until pts_d is replaced or changed in place (repeated reads cost one
        device-to-host copy, not one each)."""
        return self._host("pts", self.pts_d)

    @property
    def has_point(self):
        """[n_tr] bool host copy: the track has a triangulated point (read-only and cached, see
        points)."""
        return self._host("has", self.has_d)

    def _host(self, name, t):
        if t is None:
            return None
        key = (id(t), t.data_ptr(), t._version)   # _version: bumped by every in-place write
        cache = self.__dict__.setdefault("_host_cache", {})
        c = cache.get(name)
        if c is None or c[0] != key or c[2] is not t:
            c = (key, _host_copy(t), t)
            cache[name] = c
        return c[1]


def _host_copy(t):
    if t is None:
        return None
    a = t.cpu().numpy()
    a.setflags(write=False)
    return a


def _match_graph(gb, pairs, pairs_t, n_kp, group):
    """Verified graph rows [n,3] (global pair, queryIdx, trainIdx) and every pair's inlier count.
    Under an initialised torch.distributed group (one process per GPU) each rank matches and
    verifies its contiguous shard_range of the pairs and the packed graph is all-gathered (the
    bench's exchange); the rows come back in pair order, so the result is the
    single-process one, bit for bit."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        count, match, _, rs = gb.run(pairs_t)
        return gb.graph_rows(0, count, match, rs), rs["inl_count"].cpu().numpy()
    rank = dist.get_rank(group)
    ranges = [match_graph.shard_range(pairs, r, world, n_kp) for r in range(world)]
    lo, hi = ranges[rank]
    dev = pairs_t.device
    if hi > lo:
        count, match, _, rs = gb.run(pairs_t[lo:hi].contiguous())
        packed, offs = gb.graph_rows(lo, count, match, rs, return_offsets=True, packed=True)
        cnt = (offs[1:] - offs[:-1]).to(torch.int32)
        inl_loc = rs["inl_count"]
    else:  # more ranks than pairs
        cnt = torch.zeros(0, dtype=torch.int32, device=dev)
        packed = torch.zeros(0, dtype=torch.int32, device=dev)
        inl_loc = torch.zeros(0, dtype=torch.int32, device=dev)
    graph = match_graph.all_gather_graph(cnt, packed, ranges, group)
    maxp = max(max(h - l for l, h in ranges), 1)
    ipad = torch.full((maxp,), -1, dtype=torch.int32, device=dev)
    ipad[:hi - lo] = inl_loc
    iall = match_graph._gather(ipad, world, group)
    inl = torch.cat([iall[r, :h - l] for r, (l, h) in enumerate(ranges)])
    return graph, inl.cpu().numpy()


def track_observations(ptr, img, kp, kps):
    """The observation arrays of the tracks (torch tensors of one device): (track id int64, image
    int64, keypoint [n, 2] f64) per observation, track-major — from the tracks CSR (ptr [T + 1],
    img / kp [n]) and the keypoints kps [n_img, K, 2] (any float dtype; f64 is exact)."""
    import torch
    n_tr, n_obs = int(ptr.numel()) - 1, int(img.numel())
    img_l = img.long()
    otr = torch.repeat_interleave(torch.arange(n_tr, dtype=torch.int64, device=ptr.device),
                                  (ptr[1:] - ptr[:-1]).long(), output_size=n_obs)
    xy = kps.reshape(-1, 2)[img_l * kps.shape[1] + kp.long()].to(torch.float64)
    return otr, img_l, xy


def track_obs(otr, timg, n_tr, tracks, in_img):
    """Observations of `tracks` (ascending track ids) whose image is flagged in `in_img`, as the
    triangulation kernel's CSR: (o, ptr) with o the observation indices in track order, ascending
    within a track (the observation arrays are track-major), ptr [len(tracks) + 1] int32.  Torch
    tensors of one device (the GPU in the driver; the CPU in tests/test_host_cpu.py)."""
    import torch
    want = torch.zeros(n_tr, dtype=torch.bool, device=otr.device)
    want[tracks] = True
    o = torch.nonzero(want[otr] & in_img[timg]).squeeze(1)
    cnt = torch.zeros(n_tr, dtype=torch.int64, device=otr.device)   # index_add: no sizing sync
    sel = otr[o]
    cnt.index_add_(0, sel, torch.ones_like(sel))
    ptr = torch.zeros(len(tracks) + 1, dtype=torch.int32, device=otr.device)
    ptr[1:] = torch.cumsum(cnt[tracks], 0)
    return o, ptr


def registration_obs(otr, timg, has_point, registered, min_corr=30):
    """2-D/3-D correspondences of every unregistered image with >= min_corr of them: observations
    of triangulated tracks in unregistered images, grouped by image (ascending) and ascending
    observation index within an image.  Returns (sel, ids, cptr): the selected observations, the
    candidate images and their CSR offsets (ids and cptr are small and come back to the host)."""
    import torch
    cand = torch.nonzero(has_point[otr] & ~registered[timg]).squeeze(1)
    img_sorted, by_img = torch.sort(timg[cand], stable=True)
    img_u, img_n = torch.unique_consecutive(img_sorted, return_counts=True)
    keep = img_n >= min_corr
    sel = cand[by_img][torch.repeat_interleave(keep, img_n)]
    n_keep = img_n[keep]
    cptr = torch.zeros(len(n_keep) + 1, dtype=torch.int64, device=otr.device)
    cptr[1:] = torch.cumsum(n_keep, 0)
    return sel, img_u[keep].cpu().numpy().astype(np.int32), cptr.cpu().numpy().astype(np.int32)


def point_mean(err, first):
    """Mean of `err` over each run of observations (runs start where `first` is set; every point's
    observations are contiguous), summed left to right within a run — the additions of
    numpy.bincount(pt_idx, err) / max(count, 1), so the same doubles — on the device: one
    masked gather-add per observation rank (tracks are short) instead of a host round trip."""
    import torch
    n_obs = err.shape[0]
    starts = torch.nonzero(first).squeeze(1)
    lens = torch.diff(starts, append=torch.tensor([n_obs], device=err.device))
    acc = torch.zeros(starts.shape[0], dtype=err.dtype, device=err.device)
    for k in range(int(lens.max()) if n_obs else 0):
        take = err[torch.clamp(starts + k, max=n_obs - 1)]
        acc = torch.where(lens > k, acc + take, acc)
    return acc / torch.clamp(lens, min=1).to(err.dtype)


def reconstruct(desc, kps, n_kp, intr, min_track=2, n_hyp=1024, reg_thr=4.0, max_err=4.0,
                ba_iter=20, loss_s=2.0, device=0, log=None, group=None, shard_ba=False,
                ba_cg_tol=0.1, ba_pcg="auto", ba_ftol=1e-6):
    """desc [n_img,K,D] u8, kps [n_img,K,2] pixels, n_kp [n_img], intr [n_img,4] = (f, k1, cx, cy).
    Returns a Reconstruction (cams [n_img,8], registered mask, points per track, track arrays).
    With torch.distributed initialised (one process per GPU, `group` or the default group) the
    all-pairs matching + verification is sharded across the ranks and the graph all-gathered; the
    later stages are deterministic, so every rank returns the single-process reconstruction.
    shard_ba additionally shards every bundle adjustment by point (reconstruction.bundle_adjust
    shard=True: camera-block and per-CG-iteration all-reduces); the ranks then still agree with
    each other exactly, and with the single-process run up to the fp64 summation order.
    ba_cg_tol: relative residual at which each LM step's Schur-complement PCG stops (Ceres'
    ITERATIVE_SCHUR forcing default, eta = 0.1): an inexact Newton step.  At 500 x 4096 the
    final BA takes 333 CG iterations instead of 3640 (1e-10) for the same optimum to 1e-7 of
    the cost and the same reconstruction.
    ba_pcg: the sharded bundle adjustments' PCG branch (reconstruction.bundle_adjust `pcg`:
    auto | sharded | replicated); rec.ba_log records the branch each one took.
    ba_ftol: an LM run stops once an accepted step lowers the cost by <= ba_ftol * cost (Ceres'
    and COLMAP's function tolerance, 1e-6); at 1e-12 every bundle adjustment of the 500-image
    cfg5 scene ran its 20 steps."""
    import time
    import torch
    dev = torch.device("cuda", device)
    ctx = sfmcore.context(device)
    say = log or (lambda *a: None)
    tim = {}

    def lap(key, t0):
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        tim[key] = tim.get(key, 0.0) + (t1 - t0)
        return t1

    tk = time.perf_counter()
    n_img = len(desc)
    intr = np.asarray(intr, np.float64)
    pairs = np.stack(np.triu_indices(n_img, 1), axis=1).astype(np.int32)  # (a < b), a-major
    gb = match_graph.GraphBuilder(desc, kps, n_kp, device=device)
    pairs_t = torch.from_numpy(pairs).to(dev)
    rows, inl = _match_graph(gb, pairs, pairs_t, n_kp, group)
    tk = lap("match_verify", tk)
    ptr_t, timg_t, tkp_t = match_graph.build_tracks(rows, pairs_t, n_kp, min_track, device)
    n_tr = int(ptr_t.numel()) - 1
    kps_np = np.asarray(kps)
    # the observation arrays, built on the device (every bundle adjustment, registration and
    # triangulation selects its observations there; the host numpy build of the 1.4 M cfg5
    # observations took ~25 ms): track id per observation, image, and the keypoint as f64 (exact
    # from the caller's dtype; the builder's f32 copy when that is the caller's)
    kps_d = gb.kps if kps_np.dtype == np.float32 else torch.from_numpy(
        np.ascontiguousarray(kps_np)).to(dev)
    obs_d = track_observations(ptr_t, timg_t, tkp_t, kps_d)
    say(f"graph: {len(rows)} verified matches, {n_tr} tracks")

    rec = Reconstruction(n_img)
    rec.obs_d = obs_d
    rec.timings = tim
    rec.n_verified = int(rows.shape[0])
    rec._tracks_d = (ptr_t, timg_t, tkp_t)
    tk = lap("tracks", tk)
    rec.pts_d = torch.zeros((n_tr, 3), dtype=torch.float64, device=dev)
    rec.has_d = torch.zeros(n_tr, dtype=torch.bool, device=dev)
    rec.cams[:, 6:8] = intr[:, :2]

    # ---- initial pair: most verified inliers; relative pose from that pair's RANSAC-verified
    # matches (tracks may still carry a wrong observation), then its tracks are triangulated
    # rows are pair-major in pair order: a pair's rows are one slice (no host copy of the graph)
    pair_col = rows[:, 0].contiguous()
    order = np.argsort(-inl, kind="stable")
    for p in order[:10]:
        a, b = (int(v) for v in pairs[p])
        pv = torch.tensor([int(p)], dtype=pair_col.dtype, device=dev)
        lo = int(torch.searchsorted(pair_col, pv).item())
        hi = int(torch.searchsorted(pair_col, pv, right=True).item())
        r = rows[lo:hi].cpu().numpy()
        if len(r) < 50:
            continue
        xa = _undistort(kps_np[a, r[:, 1]].astype(np.float64), intr[a])
        xb = _undistort(kps_np[b, r[:, 2]].astype(np.float64), intr[b])
        ta, tb = obs_d[0][obs_d[1] == a], obs_d[0][obs_d[1] == b]
        common = torch.unique(ta[torch.isin(ta, tb)]).cpu().numpy()   # sorted, as intersect1d
        best = None
        for R, t in relative_pose(xa, xb):
            cams = rec.cams.copy()
            cams[a, :6] = 0.0
            cams[b, :3] = _angle_axis(R)
            cams[b, 3:6] = t
            pts, st = (t.cpu().numpy() for t in
                       _triangulate(ctx, cams, intr, [a, b], common, rec.obs_d, n_tr))
            good = int(np.sum((st[:, 3] == 0) & (st[:, 0] < max_err)))
            if best is None or good > best[0]:
                best = (good, cams, pts, st)
        good, cams_b, pts, st = best
        ok = (st[:, 3] == 0) & (st[:, 0] < max_err) & (st[:, 1] > 1.0)
        # at least 30 points with a triangulation angle above 1 degree: a near-zero baseline
        # (neighbouring views of a dense sequence) cannot seed the model
        if good >= 30 and int(ok.sum()) >= 30:
            rec.cams = cams_b
            sel = torch.from_numpy(common[ok]).to(dev)
            rec.pts_d[sel] = torch.from_numpy(np.ascontiguousarray(pts[ok])).to(dev)
            rec.has_d[sel] = True
            rec.registered[[a, b]] = True
            rec.gauge = (a, b)
            say(f"initial pair ({a}, {b}): {len(r)} verified matches, {int(ok.sum())} points")
            break
    if not rec.registered.any():
        raise RuntimeError("reconstruct: no initial pair with enough well-conditioned matches")
    tk = lap("initial_pair", tk)
    _bundle(rec, intr, loss_s, ba_iter, max_err, device, shard_ba, group, ba_cg_tol, ba_pcg,
            ba_ftol)
    tk = lap("bundle_adjust", tk)
    tim["rounds"] = 0

    # ---- register, triangulate, adjust until no image can be added
    while not rec.registered.all():
        # 2-D/3-D correspondences of every unregistered image with >= 30 of them, grouped by
        # image (ascending) and ascending observation index within an image: one pass
        # (selected on the device from rec.obs_d: ~1.5 M observations at cfg5)
        otr_d, timg_d, oxy_d = obs_d
        sel, ids, cptr = registration_obs(otr_d, timg_d, rec.has_d,
                                          torch.from_numpy(rec.registered).to(dev))
        if len(ids) == 0:
            break
        T = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x, dt)).to(dev)
        pts_d = rec.pts_d
        cams_r, cnt, _, _ = ctx.register_batch(T(cptr, np.int32), oxy_d[sel].contiguous(),
                                               pts_d[otr_d[sel]].contiguous(),
                                               T(intr[ids], np.float64), T(ids, np.int32),
                                               n_hyp=n_hyp, thr=reg_thr)
        cams_r, cnt = cams_r.cpu().numpy(), cnt.cpu().numpy()
        tk = lap("register", tk)
        tim["rounds"] += 1
        added = 0
        for j, i in enumerate(ids):
            if cnt[j] >= 30:
                rec.cams[i] = cams_r[j]
                rec.registered[i] = True
                added += 1
        say(f"registered {added} of {len(ids)} candidates, total {int(rec.registered.sum())}")
        if not added:
            break
        _triangulate_new(rec, ctx, intr, max_err)
        tk = lap("triangulate", tk)
        _bundle(rec, intr, loss_s, ba_iter, max_err, device, shard_ba, group, ba_cg_tol,
                ba_pcg, ba_ftol)
        tk = lap("bundle_adjust", tk)
    return rec


def _triangulate(ctx, cams, intr, imgs, tracks, obs_d, n_tr):
    """Triangulate `tracks` (ascending ids: host array or device tensor) from their observations
    in the images `imgs` (GPU kernel; the observations are selected on the device from obs_d =
    (obs_track, timg, obs_xy)).  Returns device (pts [n, 3], stats [n, 4]) f64 tensors."""
    import torch
    otr_d, timg_d, oxy_d = obs_d
    dev = otr_d.device
    in_img = torch.zeros(len(cams), dtype=torch.bool, device=dev)
    in_img[torch.as_tensor(np.asarray(imgs, np.int64), device=dev)] = True
    tr = (tracks.long() if isinstance(tracks, torch.Tensor) else
          torch.as_tensor(np.asarray(tracks, np.int64), device=dev))
    o, ptr = track_obs(otr_d, timg_d, n_tr, tr, in_img)
    T = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x, dt)).to(dev)
    return ctx.triangulate(T(cams, np.float64), T(intr[:, 2:4], np.float64), ptr,
                           timg_d[o].to(torch.int32), oxy_d[o].contiguous())


def _triangulate_new(rec, ctx, intr, max_err):
    """Triangulate every track without a point that has >= 2 observations in registered images."""
    import torch
    otr_d, timg_d, _ = rec.obs_d
    dev = otr_d.device
    n_tr = int(rec.has_d.numel())
    reg_d = torch.from_numpy(rec.registered).to(dev)
    n_reg = torch.zeros(n_tr, dtype=torch.int64, device=dev)
    sel = otr_d[reg_d[timg_d]]
    n_reg.index_add_(0, sel, torch.ones_like(sel))
    todo_d = torch.nonzero(~rec.has_d & (n_reg >= 2)).squeeze(1)
    if todo_d.numel() == 0:
        return
    pts, st = _triangulate(ctx, rec.cams, intr, np.nonzero(rec.registered)[0], todo_d, rec.obs_d,
                           n_tr)
    ok = (st[:, 3] == 0) & (st[:, 0] < max_err) & (st[:, 1] > 1.0)
    rec.pts_d[todo_d[ok]] = pts[ok]
    rec.has_d[todo_d[ok]] = True


def _bundle(rec, intr, loss_s, ba_iter, max_err, device, shard_ba=False, group=None, cg_tol=0.1,
            pcg="auto", ftol=1e-6):
    """Global LM over the registered cameras and the triangulated points (GPU), then drop points
    whose mean reprojection error stays above max_err.  Gauge: the initial pair's first camera
    keeps its pose and the second one translation coordinate (the scale); the intrinsics are
    known, so f and k1 are held too (reconstruction.gauge_mask).  The observations are selected
    on the device from rec.obs_d = (obs_track, timg, obs_xy)."""
    import time
    import torch
    t0 = time.perf_counter()
    otr_d, timg_d, oxy_d = rec.obs_d
    dev = otr_d.device
    reg_d = torch.from_numpy(rec.registered).to(dev)
    use = torch.nonzero(reg_d[timg_d] & rec.has_d[otr_d]).squeeze(1)   # the one sizing sync
    n_use = int(use.shape[0])
    if n_use == 0:
        return
    ref, second = rec.gauge
    fixed = reconstruction.gauge_mask(rec.cams, ref=ref, second=second, fix_intrinsics=True)
    # the registered cameras only, renumbered 0 .. n_reg - 1 in image order (an unregistered
    # camera has no observation here: it only added an empty block row to every kernel's camera
    # side — 500 camera blocks per setup at the first bundle adjustment of two views)
    reg_idx = np.nonzero(rec.registered)[0]
    timg_use = timg_d[use]
    if os.environ.get("SFM_BA_COMPACT", "1") != "0":
        remap = torch.full((len(rec.registered),), -1, dtype=torch.int32, device=dev)
        remap[torch.from_numpy(reg_idx).to(dev)] = torch.arange(len(reg_idx), dtype=torch.int32,
                                                                device=dev)
        ba_cams, ba_pp, ba_fixed = rec.cams[reg_idx], intr[reg_idx, 2:4], fixed[reg_idx]
        cam_sel = remap[timg_use.long()]
    else:
        reg_idx = None
        ba_cams, ba_pp, ba_fixed = rec.cams, intr[:, 2:4], fixed
        cam_sel = timg_use.to(torch.int32)
    tr = otr_d[use]   # non-decreasing (track-major): unique tracks by run starts
    first = torch.ones(n_use, dtype=torch.bool, device=dev)
    first[1:] = tr[1:] != tr[:-1]
    pts_ids = tr[first]     # device: the BA's points, gathered and scattered on the GPU
    pt_idx_d = torch.cumsum(first, 0, dtype=torch.int32) - 1
    info = {}
    t_sel = time.perf_counter() - t0    # observation selection (ends in host syncs)
    cams, pts, hist = reconstruction.bundle_adjust(ba_cams, ba_pp, rec.pts_d[pts_ids],
                                                   cam_sel, pt_idx_d,
                                                   oxy_d[use], loss_s=loss_s, max_iter=ba_iter,
                                                   cg_tol=cg_tol, ftol=ftol, device=device,
                                                   fixed=ba_fixed, shard=shard_ba, group=group,
                                                   pcg=pcg, info=info, reproj_err="device",
                                                   device_out=True)
    err_d = info.pop("err")   # device, at the returned parameters (bundle_adjust reproj_err)
    rec.ba_log.append(dict(info, n_cam=int(rec.registered.sum()), n_pt=int(pts_ids.numel()),
                           n_obs=n_use, lm_steps=len(hist),
                           lm_rejected=int(sum(1 for h in hist if not h[2])),
                           cg_iters=int(sum(h[3] for h in hist))))
    reg = rec.registered
    if reg_idx is not None:
        rec.cams[reg_idx] = cams
    else:
        rec.cams[reg] = cams[reg]
    rec.pts_d[pts_ids] = pts
    mean = point_mean(err_d, first)
    rec.has_d[pts_ids[mean > max_err]] = False
    rec.ba_log[-1]["s"] = time.perf_counter() - t0   # setup + LM + reprojection filter
    rec.ba_log[-1]["select_s"] = t_sel
    rec.history.append((int(reg.sum()), int(rec.has_d.sum()),
                        float(hist[-1][0]) if hist else float("nan")))
