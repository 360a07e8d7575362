"""Fills the reference's empty code/3d_reconstruction.py (0 bytes; its import is commented out at
code/pipeline.py:4 because a module name cannot start with a digit).  `3d_reconstruction.py` in
this directory re-exports this module under the reference's file name.

Scope: the bundle-adjustment linearisation — residuals, Jacobians and the
J^TJ blocks of papers/schoenberger2016sfm.pdf eq. (1)/§4.4 — on the GPU.  The LM solve,
triangulation and registration are "next" (SURVEY.md §8f).
"""
from __future__ import annotations

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
    pt_ptr, _ = sfmcore.csr_by(pt_idx, n_pt)
    cam_ptr, cam_obs = sfmcore.csr_by(cam_idx, n_cam)
    dev = torch.device("cuda", device)
    T = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)
    out = sfmcore.context(device).ba_jtj(T(cams, np.float64), T(pp, np.float64),
                                         T(pts, np.float64), T(cam_idx), T(pt_idx), T(uv),
                                         T(pt_ptr), T(cam_ptr), T(cam_obs), loss_s=loss_s)
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
    """Per-observation reprojection error (px) from the GPU residuals."""
    r = build_jtj(cams, pp, pts, cam_idx, pt_idx, uv, device=device)["res"]
    return np.sqrt(np.sum(r * r, axis=1))
