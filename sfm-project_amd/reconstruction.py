"""Fills the reference's empty code/3d_reconstruction.py (0 bytes; its import is commented out at
code/pipeline.py:4 because a module name cannot start with a digit).  `3d_reconstruction.py` in
this directory re-exports this module under the reference's file name.

Scope: the bundle-adjustment linearisation — residuals, Jacobians and the
J^TJ blocks of papers/schoenberger2016sfm.pdf eq. (1)/§4.4 — on the GPU; and (SURVEY.md §8f
item 3) the Levenberg-Marquardt step on them: Schur complement on the points, block-Jacobi PCG on
the reduced camera system, back-substitution, the SO(3)-aware parameter update and the trial
cost — `bundle_adjust` (restated by oracle/ba_lm.py).  Triangulation and
next-view registration remain "next".
"""
from __future__ import annotations

import contextlib

import numpy as np

import sfmcore


def build_jtj(cams, pp, pts, cam_idx, pt_idx, uv, loss_s: float = 0.0, device: int = 0,
              as_numpy: bool = True):
    """cams [n_cam,8] (angle-axis, t, f, k1), pp [n_cam,2], pts [n_pt,3], cam_idx/pt_idx [n_obs],
    uv [n_obs,2].  Observations are regrouped by point internally if needed.

    Returns dict(U [n_cam,8,8], V [n_pt,3,3], W [n_obs,8,3], gc, gp, res [n_obs,2], cost) with
    W / res in the caller's observation order."""
    import torch
    cam_idx = np.asarray(cam_idx, np.int32)
    pt_idx = np.asarray(pt_idx, np.int32)
    uv = np.asarray(uv, np.float64)
    n_cam, n_pt = len(cams), len(pts)
    order = None
    if len(pt_idx) and np.any(np.diff(pt_idx) < 0):
        order = np.argsort(pt_idx, kind="stable")
        cam_idx, pt_idx, uv = cam_idx[order], pt_idx[order], uv[order]
    dev = torch.device("cuda", device)
    T = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)
    cam_d, pt_d = T(cam_idx), T(pt_idx)
    pt_ptr, _ = sfmcore.csr_by_device(pt_d, n_pt)
    cam_ptr, cam_obs = sfmcore.csr_by_device(cam_d, n_cam)
    out = sfmcore.context(device).ba_jtj(T(cams, np.float64), T(pp, np.float64),
                                         T(pts, np.float64), cam_d, pt_d, T(uv),
                                         pt_ptr, cam_ptr, cam_obs, loss_s=loss_s)
    if not as_numpy:
        return out
    res = {k: v.cpu().numpy() for k, v in out.items()}
    res["cost"] = float(res["cost"][0])
    if order is not None:
        inv = np.empty_like(order)
        inv[order] = np.arange(len(order))
        res["W"] = res["W"][inv]
        res["res"] = res["res"][inv]
    return res


def reprojection_errors(cams, pp, pts, cam_idx, pt_idx, uv, device: int = 0) -> np.ndarray:
    """Per-observation reprojection error (px) from the GPU residuals, in the caller's order.
    The norms are formed on the device; only n_obs doubles cross PCIe (not the J^TJ blocks)."""
    import torch
    out = build_jtj(cams, pp, pts, cam_idx, pt_idx, uv, device=device, as_numpy=False)
    r = out["res"]
    err = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1]).cpu().numpy()
    pt_idx = np.asarray(pt_idx)
    if len(pt_idx) and np.any(np.diff(pt_idx) < 0):   # build_jtj regrouped by point
        order = np.argsort(pt_idx, kind="stable")
        e = np.empty_like(err)
        e[order] = err
        err = e
    return err


# ---- multi-GPU: observations sharded by point, camera blocks all-reduced --------

def shard_points(pt_ptr, rank: int, world: int):
    """[lo, hi) point range of `rank`: contiguous points, balanced by observation count.

    Sharding by point keeps V_p, W_cp, g_p and the residuals rank-local; only the camera blocks
    U_c / g_c (and the cost) are partial sums that need a reduction."""
    pt_ptr = np.asarray(pt_ptr, np.int64)
    n_pt = len(pt_ptr) - 1
    if world <= 1:
        return 0, n_pt
    n_obs = int(pt_ptr[-1])
    cuts = np.searchsorted(pt_ptr, n_obs * np.arange(world + 1) / world, side="left")
    cuts[0], cuts[-1] = 0, n_pt
    cuts = np.minimum(np.maximum.accumulate(cuts), n_pt)
    return int(cuts[rank]), int(cuts[rank + 1])


def shard_cuts_device(pt_idx, n_pt: int, world: int, ptr=None):
    """shard_points for every rank from a point-major device tensor pt_idx: the same cuts (float64
    searchsorted of the balanced observation targets in the point CSR, made monotone), computed
    on the GPU; returns host lists (point cuts [world + 1], observation cuts [world + 1]) — the
    only device -> host read of the sharded set-up (2 (world + 1) integers).  `ptr`: the point
    CSR offsets [n_pt + 1] when the caller has them (saves a bincount and its sync)."""
    import torch
    dev = pt_idx.device
    n_obs = int(pt_idx.numel())
    if world <= 1:
        return [0, n_pt], [0, n_obs]
    if ptr is None:
        ptr = torch.zeros(n_pt + 1, dtype=torch.int64, device=dev)
        if n_obs:
            ptr[1:] = torch.cumsum(torch.bincount(pt_idx.long(), minlength=n_pt), 0)
    else:
        ptr = ptr.long()
    tgt = n_obs * torch.arange(world + 1, dtype=torch.float64, device=dev) / world
    cuts = torch.searchsorted(ptr.double(), tgt, right=False)
    cuts[0], cuts[-1] = 0, n_pt
    cuts = torch.clamp(torch.cummax(cuts, 0).values, max=n_pt)
    both = torch.stack([cuts, ptr[cuts]]).cpu().tolist()
    return [int(v) for v in both[0]], [int(v) for v in both[1]]


def allreduce_camera_blocks(U, gc, cost, group=None):
    """Sum the per-rank camera blocks with ONE all-reduce: U [n_cam,8,8], g_c [n_cam,8] and the
    cost packed into a single fp64 buffer (~290 KB at n_cam = 500: latency-bound, so one
    collective instead of three).  RCCL (`nccl`) for device tensors, gloo on the CPU.
    In place; returns (U, gc, cost)."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return U, gc, cost
    nu, ng = U.numel(), gc.numel()
    buf = torch.cat([U.reshape(-1), gc.reshape(-1), cost.reshape(-1).to(U.dtype)])
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    U.copy_(buf[:nu].view_as(U))
    gc.copy_(buf[nu:nu + ng].view_as(gc))
    cost.copy_(buf[nu + ng:].view_as(cost))
    return U, gc, cost


def build_jtj_sharded(cams, pp, pts, cam_idx, pt_idx, uv, rank: int, world: int,
                      loss_s: float = 0.0, device: int = 0, group=None):
    """One process per GPU: this rank linearises the observations of its point shard on the GPU,
    then the camera blocks are all-reduced over RCCL.  Observations must be point-major.

    Returns dict like build_jtj(as_numpy=False) for the local points [lo, hi) plus `pt_range`;
    U / gc / cost are the global sums on every rank."""
    import torch
    pt_idx = np.asarray(pt_idx, np.int32)
    if len(pt_idx) and np.any(np.diff(pt_idx) < 0):
        raise ValueError("build_jtj_sharded: observations must be grouped by point")
    n_pt = len(pts)
    pt_ptr, _ = sfmcore.csr_by(pt_idx, n_pt)
    lo, hi = shard_points(pt_ptr, rank, world)
    o0, o1 = int(pt_ptr[lo]), int(pt_ptr[hi])
    out = build_jtj(cams, pp, np.asarray(pts)[lo:hi], np.asarray(cam_idx)[o0:o1],
                    pt_idx[o0:o1] - lo, np.asarray(uv)[o0:o1], loss_s=loss_s, device=device,
                    as_numpy=False)
    allreduce_camera_blocks(out["U"], out["gc"], out["cost"], group=group)
    torch.cuda.synchronize(device)
    out["pt_range"] = (lo, hi)
    return out


# ---- Levenberg-Marquardt bundle adjustment ---------------

# Sharding-invariant sums (include/sfmcore.h sfm_ba_set_chunks): the points of a bundle adjustment
# are cut into BA_CHUNKS fixed chunks (balanced by observations); every sum over points /
# observations into a camera-space or scalar value is formed per chunk and the chunk partials are
# combined by one canonical tree, so 1 to BA_CHUNKS ranks (a rank = a run of whole chunks) give the
# same bits.  SFM_BA_CHUNKS=0 selects the round-4 sums (A/B only; not sharding-invariant).
BA_CHUNKS = 8
BA_MAX_CHUNKS = 16   # SFM_BA_MAX_CHUNKS (include/sfmcore.h)


def ba_chunk_count():
    import os
    v = os.environ.get("SFM_BA_CHUNKS")
    return BA_CHUNKS if v is None else int(v)


class BAChunks:
    """A problem's chunk table (sfm_ba_set_chunks): chunk_pt / chunk_obs host lists of LOCAL point
    / observation offsets (n_chunk + 1), cam_bounds a device [n_cam, n_chunk + 1] i32 table,
    n_total 0 for the whole problem or the global chunk count for a shard (export form), k0 the
    global index of the first local chunk."""

    def __init__(self, chunk_pt, chunk_obs, cam_bounds, n_total=0, k0=0):
        self.chunk_pt, self.chunk_obs = list(chunk_pt), list(chunk_obs)
        self.cam_bounds, self.n_total, self.k0 = cam_bounds, int(n_total), int(k0)
        self.n_chunk = len(self.chunk_pt) - 1


def cam_bounds_device(cam_idx, cam_obs, n_cam: int, chunk_obs):
    """[n_cam, n_chunk + 1] i32 device: the positions in cam_obs (the camera-major CSR order, each
    camera's observations ascending) where camera c's list reaches observation chunk_obs[k] —
    one torch.searchsorted over keys c * (n_obs + 1) + observation."""
    import torch
    dev = cam_obs.device
    n_obs = int(cam_obs.numel())
    key = cam_idx.long()[cam_obs.long()] * (n_obs + 1) + cam_obs.long()
    q = (torch.arange(n_cam, dtype=torch.int64, device=dev)[:, None] * (n_obs + 1)
         + torch.as_tensor(chunk_obs, dtype=torch.int64, device=dev)[None, :])
    return torch.searchsorted(key, q.reshape(-1)).to(torch.int32).reshape(n_cam, -1).contiguous()


# Explicit reduced camera system (include/sfmcore.h sfm_ba_set_schur): the
# off-diagonal Schur blocks formed once per solve from the camera-pair products of every point,
# then the CG runs on S.  It pays when those products are few against the CG's per-iteration
# stream of W (344 B per observation per iteration against 456 B per product per solve, the
# iterations per solve 10-40): explicit iff products <= SCHUR_INST_PER_OBS * observations (short
# tracks: cfg5's ~5 views per point give ~1.7; long tracks of 100 views give ~50).
SCHUR_INST_PER_OBS = 4.0
# ... and when the structure is dense enough to use: T is built by a wave pair per (chunk, slot)
# group, which wants >= SCHUR_INST_PER_SEG products per group, and the product reads 1 KB per
# camera pair per iteration, which must stay under SCHUR_S_FRACTION of the implicit iteration's
# 344 B per observation (random visibility over 500 cameras: 4.4 products per group and every one
# of the 124 750 pairs: 4.0 ms per T build and 87 us per iteration, tests/perf/ba_schur_time.py)
SCHUR_INST_PER_SEG = 16.0
SCHUR_S_FRACTION = 0.25


def schur_rule(n_inst, n_seg, n_slot, n_obs):
    """True when the explicit reduced camera system pays (whole-problem counts)."""
    return (n_inst <= SCHUR_INST_PER_OBS * max(n_obs, 1) and n_inst >= SCHUR_INST_PER_SEG * n_seg
            and 1024.0 * n_slot <= SCHUR_S_FRACTION * 344.0 * max(n_obs, 1))


def schur_mode():
    """SFM_BA_SCHUR: 'auto' (default, the rule above), '1' (always), '0' (never)."""
    import os
    return os.environ.get("SFM_BA_SCHUR", "auto")


class SchurSpec:
    """Structure of the explicit reduced camera system of one (local) problem: device int32
    tensors slot_cam [n_slot, 2] (the WHOLE problem's camera pairs ci <= cj, sorted), seg [4, n_seg]
    (local chunk, slot, first, end instance: this problem's (chunk, slot) groups), inst [2, n_inst]
    (observation pairs, grouped, point order inside a group), row_ptr [n_cam + 1] / row_ent [n_ent]
    (2 slot + t, t = 1 for the slot's transpose: block row c of S); the WHOLE problem's groups:
    n_group, gk [n_group] (their chunk), sg_ptr [n_slot + 1] / sg [n_group] (each slot's groups in
    chunk order); g0 = this problem's first group among them."""

    def __init__(self, slot_cam, seg, inst, row_ptr, row_ent, sg_ptr, sg, gk, g0):
        self.slot_cam, self.seg, self.inst = slot_cam, seg, inst
        self.row_ptr, self.row_ent = row_ptr, row_ent
        self.sg_ptr, self.sg, self.gk, self.g0 = sg_ptr, sg, gk, int(g0)
        self.n_slot, self.n_seg = int(slot_cam.shape[0]), int(seg.shape[1])
        self.n_inst, self.n_ent = int(inst.shape[1]), int(row_ent.numel())
        self.n_group = int(gk.numel())


def schur_pair_count(pt_ptr):
    """Camera-pair products of a point-major problem: Σ_p m_p (m_p - 1) / 2 (device int64 scalar)."""
    import torch
    m = (pt_ptr[1:] - pt_ptr[:-1]).long()
    return (m * (m - 1) // 2).sum()


def schur_instances(cam_idx, pt_idx, pt_ptr, n_cam, chunk_pt, total=None):
    """The local camera-pair instances: for every point and every pair of its observations a < b
    (observation order), oriented so that cam(a) <= cam(b); a pair within one camera also as
    (b, a).  Returns (composite key chunk * n_cam^2 + ci * n_cam + cj, a, b) sorted stably by the
    key — inside a (chunk, slot) group the instances stay in point order.  Two host syncs (the
    instance count, unless the caller passes it as `total` — schur_pair_count — and the
    same-camera count)."""
    import torch
    dev = cam_idx.device
    n_obs = int(cam_idx.numel())
    if n_obs == 0:
        e = torch.zeros(0, dtype=torch.int64, device=dev)
        return e, e, e
    ptr = pt_ptr.long()
    end = ptr[1:][pt_idx.long()]                               # end of each observation's point
    o = torch.arange(n_obs, dtype=torch.int64, device=dev)
    cnt = end - o - 1                                          # partners after o in its point
    total = int(cnt.sum()) if total is None else int(total)
    a = torch.repeat_interleave(o, cnt, output_size=total)
    first = torch.cumsum(cnt, 0) - cnt
    b = a + 1 + (torch.arange(total, dtype=torch.int64, device=dev)
                 - torch.repeat_interleave(first, cnt, output_size=total))
    cam = cam_idx.long()
    ca, cb = cam[a], cam[b]
    sw = ca > cb
    a, b = torch.where(sw, b, a), torch.where(sw, a, b)
    same = ca == cb
    if int(same.sum()):
        a, b = torch.cat([a, b[same]]), torch.cat([b, a[same]])
    cpt = torch.as_tensor(list(chunk_pt[1:]), dtype=torch.int64, device=dev)
    k = torch.searchsorted(cpt, pt_idx.long()[a], right=True)
    key = (k * n_cam + cam[a]) * n_cam + cam[b]
    if len(chunk_pt) * n_cam * n_cam < 2 ** 31:
        key = key.to(torch.int32)                              # a 32-bit sort
    key, order = torch.sort(key, stable=True)
    return key.long(), a[order], b[order]


def schur_groups(key):
    """(composite keys of the (chunk, slot) groups, their sizes) of sorted instance keys."""
    import torch
    return torch.unique_consecutive(key, return_counts=True)


def schur_spec(comp, cnt, a, b, n_cam, all_groups, k0=0):
    """SchurSpec from this problem's (chunk, slot) groups (sorted local composite keys `comp`, sizes
    `cnt`, the sorted instances a / b) and the WHOLE problem's group keys `all_groups` (global chunk
    * n_cam^2 + ci * n_cam + cj, sorted, identical on every rank; this problem's chunks start at
    global chunk k0)."""
    import torch
    dev = all_groups.device
    i32 = torch.int32
    nn = n_cam * n_cam
    slot_keys = torch.unique(all_groups % nn)
    starts = torch.cumsum(cnt, 0) - cnt
    seg = torch.stack([comp // nn, torch.searchsorted(slot_keys, comp % nn), starts,
                       starts + cnt]).to(i32).contiguous()
    ci, cj = slot_keys // n_cam, slot_keys % n_cam
    slot_cam = torch.stack([ci, cj], 1).to(i32).contiguous()
    s = torch.arange(slot_keys.numel(), dtype=torch.int64, device=dev)
    off = ci != cj
    rows = torch.cat([ci, cj[off]])
    other = torch.cat([cj, ci[off]])
    ent = torch.cat([2 * s, 2 * s[off] + 1])
    rk, order = torch.sort(rows * n_cam + other, stable=True)
    row_ptr = torch.searchsorted(rk, torch.arange(n_cam + 1, dtype=torch.int64, device=dev) * n_cam)
    # the whole problem's groups: chunk, slot; each slot's groups in chunk order
    gk = all_groups // nn
    gslot = torch.searchsorted(slot_keys, all_groups % nn)
    gs_sorted, sg = torch.sort(gslot * 64 + gk, stable=True)
    sg_ptr = torch.searchsorted(gs_sorted, torch.arange(slot_keys.numel() + 1, dtype=torch.int64,
                                                        device=dev) * 64)
    g0 = 0 if k0 == 0 else int(torch.searchsorted(
        all_groups, torch.tensor([k0 * nn], dtype=all_groups.dtype, device=dev)).item())
    inst = torch.stack([a, b]).to(i32).contiguous()
    return SchurSpec(slot_cam, seg, inst, row_ptr.to(i32).contiguous(),
                     ent[order].to(i32).contiguous(), sg_ptr.to(i32).contiguous(),
                     sg.to(i32).contiguous(), gk.to(i32).contiguous(), g0)


class BAProblem:
    """Device-resident observations + CSR indices for repeated linearisation / solves."""

    def __init__(self, pp, cam_idx, pt_idx, uv, n_cam: int, n_pt: int, device: int = 0,
                 chunks=None, n_total: int = 0, k0: int = 0):
        """cam_idx / pt_idx / uv: numpy arrays, or device tensors (int32, int32, f64 [n,2]) that
        are used in place (no host round trip; the incremental driver selects its observations
        on the device).  `order` (numpy, or a device tensor for tensor inputs) is the stable
        regrouping by point when pt_idx was not already point-major, else None.
        chunks: None (the round-4 sums), an int C (the whole problem cut into C chunks balanced
        by observations) or a list of local chunk point offsets (a shard: n_total chunks in all,
        the first local one global chunk k0) — see BAChunks."""
        import torch
        self.dev = torch.device("cuda", device)
        self.order = None
        if isinstance(pt_idx, torch.Tensor):
            cam_d = cam_idx.to(self.dev, torch.int32).contiguous()
            pt_d = pt_idx.to(self.dev, torch.int32).contiguous()
            uv_d = uv.to(self.dev, torch.float64).contiguous()
            if pt_d.numel() > 1 and bool((pt_d[1:] < pt_d[:-1]).any()):
                self.order = torch.argsort(pt_d.long(), stable=True)
                cam_d, pt_d, uv_d = cam_d[self.order], pt_d[self.order], uv_d[self.order]
            self.cam_idx, self.pt_idx, self.uv = cam_d, pt_d, uv_d
        else:
            cam_idx = np.asarray(cam_idx, np.int32)
            pt_idx = np.asarray(pt_idx, np.int32)
            uv = np.asarray(uv, np.float64)
            if len(pt_idx) and np.any(np.diff(pt_idx) < 0):
                self.order = np.argsort(pt_idx, kind="stable")
                cam_idx, pt_idx, uv = cam_idx[self.order], pt_idx[self.order], uv[self.order]
            T = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a, dt)).to(self.dev)
            self.cam_idx, self.pt_idx, self.uv = T(cam_idx), T(pt_idx), T(uv)
        self.pp = torch.from_numpy(np.ascontiguousarray(pp, np.float64)).to(self.dev)
        self.pt_ptr = sfmcore.csr_ptr_device(self.pt_idx, n_pt, ascending=True)   # point-major
        self.cam_ptr, self.cam_obs = sfmcore.csr_by_device(self.cam_idx, n_cam)
        self.n_cam, self.n_pt = n_cam, n_pt
        self.ctx = sfmcore.context(device)
        self.chunks = None
        self.schur = None   # SchurSpec (set_schur), the explicit reduced camera system
        self._bound = False
        if chunks is not None and chunks != 0:
            if isinstance(chunks, int):
                cpt, cob = shard_cuts_device(self.pt_idx, n_pt, chunks, ptr=self.pt_ptr)
                n_total, k0 = 0, 0
            else:
                cpt = [int(v) for v in chunks]
                ptr = self.pt_ptr[torch.as_tensor(cpt, dtype=torch.int64, device=self.dev)]
                cob = [int(v) for v in ptr.cpu().tolist()]
            cb = cam_bounds_device(self.cam_idx, self.cam_obs, n_cam, cob)
            self.chunks = BAChunks(cpt, cob, cb, n_total, k0)

    def set_schur(self, union=None, n_pairs=None):
        """Turn the explicit reduced camera system on (needs chunk mode).  union: for a shard, maps
        this shard's group keys (global chunk * n_cam^2 + ci * n_cam + cj, sorted int64 device
        tensor) to the WHOLE problem's (every rank's, sorted; a collective, the same result on
        every rank); None = this problem's own.  n_pairs: this problem's schur_pair_count when
        the caller already read it (saves a host sync)."""
        if self.chunks is None:
            raise ValueError("BAProblem.set_schur: the explicit Schur system needs chunk mode")
        key, a, b = schur_instances(self.cam_idx, self.pt_idx, self.pt_ptr, self.n_cam,
                                    self.chunks.chunk_pt, total=n_pairs)
        comp, cnt = schur_groups(key)
        k0 = self.chunks.k0
        gkeys = comp + k0 * self.n_cam * self.n_cam
        all_groups = union(gkeys) if union is not None else gkeys
        self.schur = schur_spec(comp, cnt, a, b, self.n_cam, all_groups, k0)

    def _call(self, fn, *a, **kw):
        """fn under this problem's chunk mode and explicit-Schur structure (set on the shared
        context, then cleared; inside bind() they stay set)."""
        if self.chunks is None or self._bound:
            return fn(*a, **kw)
        self.ctx.ba_set_chunks(self.chunks)
        if self.schur is not None:
            self.ctx.ba_set_schur(self.schur)
        try:
            return fn(*a, **kw)
        finally:
            self.ctx.ba_set_chunks(None)
            if self.schur is not None:
                self.ctx.ba_set_schur(None)

    @contextlib.contextmanager
    def bind(self):
        """Keep this problem's chunk mode / Schur structure set on the shared context for a
        block of calls (an LM loop: 4 ctypes calls fewer per linearise / solve / cost).  No other
        BAProblem may use the context inside the block."""
        if self.chunks is None or self._bound:
            yield self
            return
        self.ctx.ba_set_chunks(self.chunks)
        if self.schur is not None:
            self.ctx.ba_set_schur(self.schur)
        self._bound = True
        try:
            yield self
        finally:
            self._bound = False
            self.ctx.ba_set_chunks(None)
            if self.schur is not None:
                self.ctx.ba_set_schur(None)

    def _slots(self):
        ck = self.chunks
        return ck.n_chunk if ck is not None and ck.n_total > 0 else None

    def linearize(self, cams, pts, loss_s=0.0):
        """sfm_ba_jtj; for a chunked shard U / gc / cost are the local chunks' partials."""
        return self._call(self.ctx.ba_jtj, cams, self.pp, pts, self.cam_idx, self.pt_idx, self.uv,
                          self.pt_ptr, self.cam_ptr, self.cam_obs, loss_s=loss_s,
                          n_slot=self._slots())

    def solve(self, lin, lam, max_iter=100, tol=1e-10, poll=8, poll_first=0):
        return self._call(self.ctx.ba_solve, lin, self.cam_idx, self.pt_idx, self.pt_ptr,
                          self.cam_ptr, self.cam_obs, lam, max_iter=max_iter, tol=tol, poll=poll,
                          poll_first=poll_first)

    def solve_sharded(self, lin, lam, allreduce, max_iter=100, tol=1e-10, **kw):
        return self._call(self.ctx.ba_solve_sharded, lin, self.cam_idx, self.pt_idx, self.pt_ptr,
                          self.cam_ptr, self.cam_obs, lam, allreduce, max_iter=max_iter, tol=tol,
                          chunks=self.chunks, schur=self.schur, **kw)

    def cost(self, cams, pts, loss_s=0.0):
        return self._call(self.ctx.ba_cost, cams, self.pp, pts, self.cam_idx, self.pt_idx, self.uv,
                          loss_s, n_slot=self._slots())

    def update(self, cams, dc, pts, dp):
        return self.ctx.ba_update(cams, dc, pts, dp)


def gauge_mask(cams, ref: int = 0, second=None, fix_intrinsics: bool = False,
               registered=None):
    """[n_cam, 8] bool mask of the parameters to hold in bundle adjustment.

    The reprojection error is invariant under a similarity of the whole scene (7 DoF: rotation,
    translation, scale), so without a gauge the reduced camera system is singular and only the LM
    damping keeps it solvable.  This fixes the reference camera's pose (angle-axis + t: 6) and
    the scale: the coordinate k of the second camera's translation relative to the reference
    centre, t2 - R2 R_ref^T t_ref (in camera 2's frame: what a scaling about the reference centre
    multiplies), with the largest magnitude — held by fixing t2[k].  fix_intrinsics additionally
    holds f and k1 of every camera (calibrated cameras).  `second`: the second camera (default:
    the registered camera farthest from the reference); `registered`: optional bool mask of
    the cameras that take part."""
    cams = np.asarray(cams, np.float64)
    n = len(cams)
    fixed = np.zeros((n, 8), bool)
    if fix_intrinsics:
        fixed[:, 6:8] = True
    if n == 0:
        return fixed
    reg = np.ones(n, bool) if registered is None else np.asarray(registered, bool)
    fixed[ref, :6] = True
    R = lambda c: _rotmat_np(cams[c, :3])
    C = lambda c: -R(c).T @ cams[c, 3:6]
    if second is None:
        cand = [c for c in np.nonzero(reg)[0] if c != ref]
        if not cand:
            return fixed
        second = max(cand, key=lambda c: np.linalg.norm(C(c) - C(ref)))
    rel = cams[second, 3:6] - R(second) @ R(ref).T @ cams[ref, 3:6]
    fixed[second, 3 + int(np.argmax(np.abs(rel)))] = True
    return fixed


def _rotmat_np(r):
    th = np.linalg.norm(r)
    if th < 1e-12:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


_rccl_comms = {}


def make_allreduce(group=None, direct: bool = True, device=None):
    """In-place fp64 sum over the ranks of `group`, ordered on the current stream.

    `nccl` groups: by default a direct RCCL communicator (rccl.RcclComm, created once per
    (group, device) and cached: collective, so every rank calls this at the same point) that
    enqueues ncclAllReduce on the current stream itself, without ProcessGroupNCCL's side stream
    and its two event waits per call; direct=False goes through torch.distributed.all_reduce.
    `device`: this rank's GPU (default: the current device) — with every GPU visible each rank
    passes its local rank, so the communicator lives on the GPU the tensors live on.  Both are
    marked graph_safe (ba_solve_sharded may replay its CG windows as HIP graphs).  Other
    backends (gloo: the CPU tests and the same-GPU rehearsals) sum through a host copy."""
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        if direct:
            import rccl
            import torch
            dev = torch.cuda.current_device() if device is None else int(device)
            key = (group if group is not None else dist.group.WORLD, dev)
            comm = _rccl_comms.get(key)
            if comm is None:
                comm = _rccl_comms[key] = rccl.RcclComm(group, device=dev)

            def allreduce(t):
                comm.allreduce_(t)
            allreduce.comm = comm
        else:
            def allreduce(t):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        allreduce.graph_safe = True
    else:
        def allreduce(t):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            t.copy_(h)
    return allreduce


def release_allreduce(group=None):
    """Destroys the RCCL communicators that make_allreduce opened for `group` (collective; call
    it on every rank before torch.distributed.destroy_process_group)."""
    import torch.distributed as dist
    g = group if group is not None else dist.group.WORLD
    for key in [k for k in _rccl_comms if k[0] is g or k[0] == g]:
        _rccl_comms.pop(key).close()
    for key in [k for k in _probe_cache if k[1] is g or k[1] == g]:   # probes of a dead comm
        del _probe_cache[key]


# ---- shard / replicate rule for the multi-GPU PCG --------------------------------
# Per-CG-iteration cost model of the Schur-complement PCG (world-size-1 measurements at cfg5,
# 500 cameras x 100 k points x 5 observations, profiles/r03/ba_solve_cfg5_r3q.json):
#   unsharded iteration   t(n_obs)      = PCG_FIXED_US + PCG_OBS_US * n_obs   (49.7 us at 500 k)
#   sharded, N ranks      t(n_obs / N)  + PCG_SPLIT_US + L_ar(8 n_cam doubles)
#     PCG_SPLIT_US: the split camera pass + finish launch measured at world size 1 (53.5 - 49.7)
#   replicated            t(n_obs) per iteration, plus once per linearisation an all-gather of
#                         the point-side blocks (W 192 B/obs, V 72 B + g_p 24 B per point)
# L_ar and the all-gather bandwidth are MEASURED on the group (probe_collectives, once per
# communicator and camera count, averaged over the ranks so every rank takes the same branch).
PCG_FIXED_US = 12.0       # three launches' floor (2 300-obs problems: 13.6 ms / 20 steps / ~55 it)
PCG_OBS_US = (49.7 - PCG_FIXED_US) / 500_000.0
PCG_SPLIT_US = 3.8
PCG_ITERS_PER_STEP = 20   # CG iterations per LM step assumed by the rule (cg_tol 0.1: 17 measured)
_probe_cache = {}


def probe_collectives(allreduce, n_cam: int, device, group=None, reps: int = 20,
                      big_mb: float = 8.0):
    """Measured (latency of one in-place all-reduce of 8·n_cam doubles in µs, all-reduce bus
    bandwidth in B/s) on this group: `reps` back-to-back calls of each size, timed on the
    current stream, then averaged over the ranks with the same all-reduce (every rank gets the
    same numbers, so the branch decision is collective-safe).  Cached per (backend, group, device,
    collective path, n_cam): a key every rank computes identically (not an object id, which a
    rank may or may not see reused), so all ranks hit or miss the cache together."""
    import time
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", device) if not isinstance(device, torch.device) else device
    key = _probe_key(allreduce, n_cam, dev, group)
    if key in _probe_cache:
        return _probe_cache[key]
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    small = torch.zeros(8 * n_cam, dtype=torch.float64, device=dev)
    big = torch.zeros(int(big_mb * 2 ** 20) // 8, dtype=torch.float64, device=dev)
    out = []
    for buf, n in ((small, reps), (big, max(2, reps // 4))):
        allreduce(buf)                         # warm the path
        torch.cuda.synchronize(dev)
        if dist.is_initialized():
            dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(n):
            allreduce(buf)
        torch.cuda.synchronize(dev)
        out.append((time.perf_counter() - t0) / n)
    lat_us = out[0] * 1e6
    # ring all-reduce bus bandwidth (2(N-1)/N of the bytes cross each link); world 1: bytes / time
    busbw = (2.0 * (world - 1) / world if world > 1 else 1.0) * big.numel() * 8 / max(out[1], 1e-9)
    m = torch.tensor([lat_us, busbw], dtype=torch.float64, device=dev)
    allreduce(m)
    lat_us, busbw = (float(v) / world for v in m.cpu().tolist())
    _probe_cache[key] = (lat_us, busbw)
    return lat_us, busbw


def _probe_key(allreduce, n_cam, dev, group=None):
    import torch.distributed as dist
    init = dist.is_available() and dist.is_initialized()
    g = group if group is not None else (dist.group.WORLD if init else None)
    return (dist.get_backend(group) if init else None, g, str(dev),
            "rccl-direct" if hasattr(allreduce, "comm") else "torch", int(n_cam))


def pcg_rule(n_obs: int, n_pt: int, n_cam: int, world: int, allreduce_us: float,
             busbw: float, iters: int = PCG_ITERS_PER_STEP):
    """'sharded' or 'replicated' for a world-rank PCG, and the model terms (µs per LM step).

    sharded    : iters * (t(n_obs / N) + PCG_SPLIT_US + allreduce_us)
    replicated : iters * t(n_obs) + gather (W, V, g_p of the other ranks once per linearisation:
                 (N-1)/N of the bytes at the measured bus bandwidth)
    with t(n) = PCG_FIXED_US + PCG_OBS_US * n.  Ties go to 'sharded'."""
    t = lambda n: PCG_FIXED_US + PCG_OBS_US * n
    sharded = iters * (t(n_obs / world) + PCG_SPLIT_US + allreduce_us)
    gbytes = (world - 1) / world * (192.0 * n_obs + 96.0 * n_pt)
    gather_us = gbytes / max(busbw, 1.0) * 1e6 + allreduce_us
    replicated = iters * t(n_obs) + gather_us
    mode = "sharded" if sharded <= replicated else "replicated"
    return mode, {"sharded_us_per_step": sharded, "replicated_us_per_step": replicated,
                  "gather_us": gather_us, "allreduce_us": allreduce_us, "busbw_GBs": busbw / 1e9,
                  "iters_assumed": iters, "n_obs": n_obs, "n_pt": n_pt, "world": world}


def _gather_rows(t, counts, group):
    """All-gather of a [n_r, ...] f64 device tensor whose first dimension differs per rank
    (counts[r]): zero-padded to max(counts), one collective, concatenated in rank order."""
    import torch
    import match_graph
    world = len(counts)
    mx = max(max(counts), 1)
    inner = t.shape[1:]
    pad = torch.zeros((mx,) + tuple(inner), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    g = match_graph._gather(pad.reshape(-1), world, group).reshape((world, mx) + tuple(inner))
    return torch.cat([g[r, :counts[r]] for r in range(world)]).contiguous()


# CG convergence polls after the first one (at the previous LM step's iteration count): with
# the hint the solve polls once where it expects to be done, and then often, instead of every 8
# iterations (a poll is a host round trip; an iteration past convergence two empty launches)
POLL_AFTER_HINT = 4


def _lm_loop(cams_d, pts_d, cost, linearize, solve, upd, lam0, max_iter, ftol):
    """bundle_adjust's Levenberg-Marquardt iterations (the step rule in its docstring); one host
    read of 7 scalars per step, and the solve's convergence poll placed at the previous step's
    CG iteration count (SFM_BA_POLL_HINT=0: every 8).  Returns (cams, pts, history, the
    linearisation at the returned parameters when the loop converged with one at hand, else
    None)."""
    import os
    import torch
    lam, nu = lam0, 2.0
    hist = []
    old = float(cost(cams_d, pts_d).item())
    lin = linearize(cams_d, pts_d)
    hint = 0
    use_hint = os.environ.get("SFM_BA_POLL_HINT", "1") != "0"
    # speculative linearisation: the next step's J^T J at the trial point is enqueued before the
    # host waits for this step's 7 scalars, so the GPU works through the host's round trip (a
    # rejected or final step wastes it)
    # (cfg5: 0 of 160 steps rejected, so only the 17 final steps waste it; skipping it where the
    # previous decrease was already small measured slower — profiles/r06/ba_study/s25, s26)
    spec = os.environ.get("SFM_BA_SPEC", "1") != "0"
    buf = ev = None
    final_lin = None
    for _ in range(max_iter):
        dc, dp, sinfo = solve(lin, lam, hint)
        c2, p2 = upd.update(cams_d, dc, pts_d, dp)
        new_t = cost(c2, p2)
        vals_d = torch.cat([sinfo, new_t])
        nxt = None
        if spec:
            if buf is None:
                buf = torch.empty(vals_d.numel(), dtype=vals_d.dtype, pin_memory=True)
                ev = torch.cuda.Event()
            buf.copy_(vals_d, non_blocking=True)
            ev.record()
            nxt = linearize(c2, p2)
            ev.synchronize()                                 # the one host wait of the step
            vals = buf.numpy()
        else:
            vals = vals_d.cpu().numpy()                      # the one host sync of the step
        it, gd, q, new = int(vals[0]), float(vals[2]), float(vals[3]), float(vals[5])
        hint = it if use_hint else 0
        pred = -(gd + 0.5 * q)
        if new < old and pred > 0:
            rho = (old - new) / pred
            cams_d, pts_d = c2, p2
            lam *= max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3)
            nu = 2.0
            hist.append((new, lam, True, it))
            done = old - new <= ftol * old
            old = new
            if done:
                final_lin = nxt   # the speculative K3 sits at the returned parameters
                break
            lin = nxt if nxt is not None else linearize(cams_d, pts_d)
        else:
            lam *= nu
            nu *= 2.0
            hist.append((old, lam, False, it))
            if lam > 1e16:
                break
    return cams_d, pts_d, hist, final_lin


def bundle_adjust(cams, pp, pts, cam_idx, pt_idx, uv, loss_s: float = 0.0, max_iter: int = 50,
                  lam0: float = 1e-4, ftol: float = 1e-12, max_cg: int = 200,
                  cg_tol: float = 1e-10, device: int = 0, fixed=None, shard: bool = False,
                  group=None, pcg: str = "auto", info=None, reproj_err=False, device_out=False):
    """Levenberg-Marquardt on paper eq. (1): every step on the GPU
    (J^TJ build, Schur-complement PCG, update, trial cost); the host reads 7 scalars per step to
    accept / reject it.  cam_idx / pt_idx / uv may be device tensors (used in place).

    Step rule (oracle/ba_lm.py, Nielsen): predicted decrease = -(gᵀδ + ½ δᵀJᵀJδ); accept iff
    the cost decreases, then λ *= max(1/3, 1 - (2ρ-1)³); otherwise λ *= ν, ν *= 2.  Stops after
    `max_iter` steps, when an accepted step lowers the cost by <= ftol·cost, or when λ > 1e16.

    fixed: optional [n_cam, 8] bool mask of parameters held at their values (gauge_mask;
    sfm_ba_fix_params after every linearisation).

    shard (multi-GPU; needs an initialised torch.distributed group): every rank
    linearises the points of its `shard_points` range with their observations and the camera
    blocks U / g_c are all-reduced after each linearisation (the north_star's J^TJ all-reduce);
    the trial cost is all-reduced.  The PCG then runs in one of two branches (`pcg`):
      'sharded'    — sfm_ba_solve_stage on the shard: one 8·n_cam fp64 all-reduce per CG
                     iteration; the points are gathered at the end;
      'replicated' — the point-side blocks (W, V, g_p) are all-gathered once per linearisation
                     and every rank runs the whole PCG itself (no collective per iteration);
      'auto'       — pcg_rule on the measured all-reduce latency / bandwidth of the group
                     (probe_collectives); world size 1 always takes 'sharded'.
    Every rank returns the same result, and (BA_CHUNKS) it is the
    single-process result BIT FOR BIT, for both branches and any world size up to BA_CHUNKS: the
    points are cut into BA_CHUNKS fixed chunks, a rank holds a run of whole chunks, every sum into
    a camera-space or scalar value is formed per chunk and combined by one canonical tree
    (include/sfmcore.h sfm_ba_set_chunks), and the exchanges are exact gathers of chunk partials
    (an all-reduce of zero-padded slots) instead of sums.  `info` (optional dict) receives the branch taken and the rule's terms; with
    reproj_err it also receives `err`: every observation's reprojection error (px) at the returned
    parameters, in the caller's order — from the device-resident problem (one more K3 launch;
    sharded: each rank's shard summed into a zero-padded vector), instead of a second host ->
    device copy of the whole problem through reprojection_errors.  reproj_err="device" leaves
    `err` as an f64 device tensor (same order) instead of a host array.

    pts may be a device tensor (used without a host round trip); device_out=True returns pts as
    an f64 device tensor instead of a host array.

    Returns (cams [n_cam,8], pts [n_pt,3], history [(cost, λ, accepted, cg_iterations)])."""
    import os
    import time
    import torch
    t_entry = time.perf_counter()
    if info is not None:   # the caller's queued GPU work is not this call's set-up
        torch.cuda.synchronize(device)
        info["entry_wait_s"] = time.perf_counter() - t_entry
        t_entry = time.perf_counter()
    n_cam, n_pt = len(cams), len(pts)
    allreduce = None
    world = 1
    if shard:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            allreduce = make_allreduce(group, device=device)
            rank, world = dist.get_rank(group), dist.get_world_size(group)
    mode = "single"
    deferred_rule = False
    lo, hi = 0, n_pt
    full = None
    tensors = isinstance(pt_idx, torch.Tensor)
    nchunk = ba_chunk_count()     # sharding-invariant sums (BAChunks); 0 = the round-4 sums
    k0, local_chunks = 0, None
    if allreduce is not None:
        # device-resident: point-major order, CSR and the shard cuts on the
        # GPU; the host reads world + 1 cut pairs, the observations never leave the device
        dev = torch.device("cuda", device)
        if not tensors:
            cam_idx, pt_idx, uv = (torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)
                                   for a, dt in ((cam_idx, np.int32), (pt_idx, np.int32),
                                                 (uv, np.float64)))
        cam_idx = cam_idx.to(dev, torch.int32).contiguous()
        pt_idx = pt_idx.to(dev, torch.int32).contiguous()
        uv = uv.to(dev, torch.float64).contiguous()
        order = None
        if pt_idx.numel() > 1 and bool((pt_idx[1:] < pt_idx[:-1]).any()):
            order = torch.argsort(pt_idx.long(), stable=True)
            cam_idx, pt_idx, uv = cam_idx[order], pt_idx[order], uv[order]
        n_obs_all = int(pt_idx.numel())
        if nchunk > 0:
            # the whole problem's chunks (balanced by observations); rank r takes chunks
            # [r C / N, (r + 1) C / N): every rank a run of whole chunks, so the sums match N = 1
            if world > nchunk:
                # every rank needs a whole chunk: raise the count to the rank count (the chunk
                # sums then differ from a run with BA_CHUNKS chunks in the last bits), or beyond
                # SFM_BA_MAX_CHUNKS fall back to the plain per-shard sums (no chunk table)
                nchunk = world if world <= BA_MAX_CHUNKS else 0
                if info is not None:
                    info["chunks_adjusted"] = {"world": world, "nchunk": nchunk}
        if nchunk > 0:
            gcuts, gocuts = shard_cuts_device(pt_idx, n_pt, nchunk)
            kr = [r * nchunk // world for r in range(world + 1)]
            cuts, ocuts = [gcuts[k] for k in kr], [gocuts[k] for k in kr]
            k0 = kr[rank]
            local_chunks = [gcuts[k] - gcuts[k0] for k in range(k0, kr[rank + 1] + 1)]
        else:
            cuts, ocuts = shard_cuts_device(pt_idx, n_pt, world)
        lo, hi = cuts[rank], cuts[rank + 1]
        o0, o1 = ocuts[rank], ocuts[rank + 1]
        mode = os.environ.get("SFM_BA_PCG", pcg)
        if mode not in ("auto", "sharded", "replicated"):
            raise ValueError(f"bundle_adjust: pcg must be auto|sharded|replicated, got {mode!r}")
        if mode == "auto":
            # the explicit reduced camera system (schur_rule) has no exchange per CG iteration:
            # then the sharded branch (one gather of T's chunk partials per solve) is the one;
            # the pair count is the whole problem's, the same on every rank
            likely_schur = False
            if nchunk > 0 and schur_mode() != "0":
                m = torch.bincount(pt_idx.long(), minlength=n_pt)
                pairs = float((m * (m - 1) // 2).sum())
                likely_schur = schur_mode() == "1" or pairs <= SCHUR_INST_PER_OBS * max(n_obs_all, 1)
            def rule():
                # the chunked sharded CG all-reduces nchunk camera-vector partials per iteration
                # (ADVICE r5): probe and price that payload, not one camera vector
                lat, bw = probe_collectives(allreduce, n_cam * max(nchunk, 1), device, group)
                m_, terms = pcg_rule(n_obs_all, n_pt, n_cam, world, lat, bw)
                terms["allreduce_doubles"] = 8 * n_cam * max(nchunk, 1)
                if info is not None:
                    info["rule"] = terms
                return m_
            if world == 1 or likely_schur:
                mode = "sharded"
                # the pair count alone made the explicit system the candidate: if schur_rule's
                # other tests reject it below, pcg_rule decides the branch then
                deferred_rule = world > 1
                if info is not None and world > 1:
                    info["rule"] = {"explicit_schur_candidate": True}
            else:
                mode = rule()
        whole = (cam_idx, pt_idx, uv)   # the whole problem, for a replicated branch decided late
        if mode == "replicated":
            # the whole problem for the solve (every rank), the shard for the linearisation
            full = BAProblem(pp, cam_idx, pt_idx, uv, n_cam, n_pt, device, chunks=nchunk or None)
            counts_pt = [cuts[r + 1] - cuts[r] for r in range(world)]
            counts_obs = [ocuts[r + 1] - ocuts[r] for r in range(world)]
        cam_idx, pt_idx, uv = cam_idx[o0:o1], pt_idx[o0:o1] - lo, uv[o0:o1]
    if info is not None:
        info.update(pcg=mode, world=world)
    if local_chunks is not None:    # a shard: its chunks' partials are exchanged (export form)
        prob = BAProblem(pp, cam_idx, pt_idx, uv, n_cam, hi - lo, device, chunks=local_chunks,
                         n_total=nchunk, k0=k0)
    else:
        prob = BAProblem(pp, cam_idx, pt_idx, uv, n_cam, hi - lo, device, chunks=nchunk or None)
    f64 = torch.float64
    # explicit reduced camera system (SchurSpec) when the camera-pair products are few: the rule
    # sees the WHOLE problem's counts, so every rank (and the single process) decides alike
    use_schur = False
    smode = schur_mode()
    if nchunk > 0 and smode != "0":
        tgt = full if full is not None else prob
        cnt = schur_pair_count(tgt.pt_ptr).double().reshape(1)
        own = cnt.clone()
        n_obs_tot = len(tgt.cam_idx)
        if allreduce is not None and full is None:
            allreduce(cnt)
            n_obs_tot = n_obs_all
        cnt, own = (float(v) for v in torch.cat([cnt, own]).tolist())   # one host read
        use_schur = smode == "1" or cnt <= SCHUR_INST_PER_OBS * max(n_obs_tot, 1)
        if use_schur:
            t_s = time.perf_counter()
            sharded_s = allreduce is not None and full is None
            if sharded_s:
                def union(keys):   # every shard's (chunk, slot) groups -> the whole problem's
                    nk = torch.zeros(world, dtype=f64, device=prob.dev)
                    nk[rank] = keys.numel()
                    allreduce(nk)
                    g = _gather_rows(keys.double().reshape(-1, 1), [int(v) for v in nk.tolist()],
                                     group)
                    return torch.sort(g.reshape(-1).long()).values
                prob.set_schur(union, n_pairs=own)
            else:
                tgt.set_schur(n_pairs=own)
            sp = tgt.schur
            n_inst_tot = float(sp.n_inst)
            if sharded_s:
                tot = torch.tensor([sp.n_inst], dtype=f64, device=prob.dev)
                allreduce(tot)   # the whole problem's products
                n_inst_tot = float(tot.item())
            n_seg_tot = float(sp.n_group)
            if smode != "1" and not schur_rule(n_inst_tot, n_seg_tot, sp.n_slot, n_obs_tot):
                tgt.schur = None
                use_schur = False
            if info is not None:
                info["schur_terms"] = {"n_inst": n_inst_tot, "n_seg": n_seg_tot,
                                       "n_slot": sp.n_slot, "n_obs": n_obs_tot}
                info["schur_s"] = time.perf_counter() - t_s   # structure + rule (ends in a sync)
    if deferred_rule and not use_schur:
        mode = rule()
        if mode == "replicated":
            full = BAProblem(pp, *whole, n_cam, n_pt, device, chunks=nchunk or None)
            counts_pt = [cuts[r + 1] - cuts[r] for r in range(world)]
            counts_obs = [ocuts[r + 1] - ocuts[r] for r in range(world)]
        if info is not None:
            info.update(pcg=mode, rule=dict(info["rule"], explicit_schur_rejected=True))
    if info is not None:
        info["schur"] = use_schur
        torch.cuda.synchronize(prob.dev)
        info["problem_s"] = time.perf_counter() - t_entry   # BAProblem: CSR, chunk table

    def gather_chunks(part, width):
        """This shard's chunk partials [n_local, width] -> the canonical tree over all chunks
        [width]: an all-reduce of a zero-filled [C, width] slot buffer (an exact all-gather)."""
        nl = prob.chunks.n_chunk
        slot = torch.zeros((nchunk, width), dtype=f64, device=prob.dev)
        slot[k0:k0 + nl] = part.reshape(nl, width)
        allreduce(slot.view(-1))
        return prob.ctx.ba_chunk_tree(slot)
    T = lambda a: (a.to(prob.dev, torch.float64).contiguous() if isinstance(a, torch.Tensor)
                   else torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(prob.dev))
    cams_d = T(cams)
    # replicated: every rank keeps all points (the solve's δp is whole); the shard is a view
    pts_d = T(pts) if full is not None else T(pts[lo:hi] if isinstance(pts, torch.Tensor)
                                              else np.asarray(pts, np.float64)[lo:hi])
    shard_of = (lambda p: p[lo:hi]) if full is not None else (lambda p: p)
    fixed_d = None
    if fixed is not None and np.any(fixed):
        fixed_d = torch.from_numpy(np.ascontiguousarray(fixed, np.uint8).reshape(n_cam, 8)).to(prob.dev)

    def linearize(c, p):
        lin = prob.linearize(c, shard_of(p), loss_s)
        if allreduce is not None and local_chunks is not None:   # chunk partials -> the tree
            nl = prob.chunks.n_chunk
            tot = gather_chunks(torch.cat([lin["U"].reshape(nl, -1), lin["gc"].reshape(nl, -1)],
                                          1), n_cam * 72)
            lin["U"] = tot[:n_cam * 64].view(n_cam, 8, 8)
            lin["gc"] = tot[n_cam * 64:].view(n_cam, 8)
        elif allreduce is not None:   # global camera blocks before the gauge is applied
            nu_, ng = lin["U"].numel(), lin["gc"].numel()
            buf = torch.cat([lin["U"].reshape(-1), lin["gc"].reshape(-1)])
            allreduce(buf)
            lin["U"].copy_(buf[:nu_].view_as(lin["U"]))
            lin["gc"].copy_(buf[nu_:nu_ + ng].view_as(lin["gc"]))
        if fixed_d is not None:
            prob.ctx.ba_fix_params(lin, prob.cam_idx, fixed_d)
        if full is not None:        # the point-side blocks of every rank, once per linearisation
            lin = dict(lin, W=_gather_rows(lin["W"], counts_obs, group),
                       V=_gather_rows(lin["V"], counts_pt, group),
                       gp=_gather_rows(lin["gp"], counts_pt, group))
        return lin

    def cost(c, p):
        t = prob.cost(c, shard_of(p), loss_s)
        if allreduce is not None and local_chunks is not None:
            t = gather_chunks(t[:prob.chunks.n_chunk], 1)
        elif allreduce is not None:
            allreduce(t)
        return t

    def solve(lin, lam, first=0):
        # first: where to poll the CG's convergence first (the previous solve's iteration count;
        # then every POLL_AFTER_HINT), instead of at every multiple of 8
        poll = POLL_AFTER_HINT if first > 0 else 8
        if full is not None:
            return full.solve(lin, lam, max_cg, cg_tol, poll=poll, poll_first=first)
        if allreduce is None:
            return prob.solve(lin, lam, max_cg, cg_tol, poll=poll, poll_first=first)
        return prob.solve_sharded(lin, lam, allreduce, max_iter=max_cg, tol=cg_tol, poll=poll,
                                  poll_first=first)
    upd = full if full is not None else prob
    if info is not None:
        torch.cuda.synchronize(prob.dev)
        t_lm = time.perf_counter()
        info["setup_s"] = t_lm - t_entry    # problem upload / CSR build before the first LM step
    # one problem on the context for the whole loop (replicated: two alternate, so per call)
    bound = (prob.bind() if full is None and os.environ.get("SFM_BA_BIND", "1") != "0"
             else contextlib.nullcontext())
    with bound:
        cams_d, pts_d, hist, final_lin = _lm_loop(cams_d, pts_d, cost, linearize, solve, upd,
                                                  lam0, max_iter, ftol)
    if info is not None:
        info["lm_s"] = time.perf_counter() - t_lm   # the loop ends in a host sync (the last step)
    if reproj_err and info is not None:
        # the residuals at the returned parameters: the LM's last speculative K3 when the loop
        # ended on convergence (the same call on the same parameters), else one more K3
        r = (final_lin["res"] if final_lin is not None
             else prob.linearize(cams_d, shard_of(pts_d), loss_s)["res"])
        e = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1])
        if allreduce is None:
            if prob.order is not None:   # BAProblem regrouped the observations by point
                back = torch.empty_like(e)
                back[torch.as_tensor(prob.order, device=e.device)] = e
                e = back
            err = e if reproj_err == "device" else e.cpu().numpy()
        else:
            ev = torch.zeros(n_obs_all, dtype=torch.float64, device=prob.dev)
            ev[o0:o1] = e
            allreduce(ev)
            if order is not None:       # back to the caller's observation order
                back = torch.empty_like(ev)
                back[order] = ev
                ev = back
            err = ev if reproj_err == "device" else ev.cpu().numpy()
        info["err"] = err
    if allreduce is not None and full is None:
        # gather the point shards: one all-reduce of the zero-padded set
        allp = torch.zeros((n_pt, 3), dtype=torch.float64, device=prob.dev)
        allp[lo:hi] = pts_d
        allreduce(allp.view(-1))
        pts_d = allp
    out = cams_d.cpu().numpy(), (pts_d if device_out else pts_d.cpu().numpy()), hist
    if info is not None:
        info["post_s"] = time.perf_counter() - t_lm - info["lm_s"]   # errors + results to host
    return out
