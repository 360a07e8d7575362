"""CPU restatement of the bundle-adjustment solve (Schur-complement PCG + Levenberg-Marquardt).

TEST INFRASTRUCTURE ONLY (see oracle.py): imported by tests/ as the checker of
sfm-project_amd/csrc/ba_solve.hip and reconstruction.bundle_adjust.  Never used by the product.

SURVEY.md §8f item 3 ("rest of incremental SfM for cfg5: LM step with Schur complement + camera-
system Cholesky/PCG", papers/schoenberger2016sfm.pdf §2.2 eq. (1), §4.4-4.5).  The reference's
code/3d_reconstruction.py is empty, so the spec is the build's:

* damped normal equations (Marquardt): [U+λD_U  W; Wᵀ  V+λD_V] [δc; δp] = -[g_c; g_p], with
  D = diag clamped to [1e-6, 1e32] (the Ceres convention);
* Schur complement on the points: S = U_d - Σ_o W_o V_d⁻¹ W_oᵀ, b = -g_c + Σ_o W_o V_d⁻¹ g_p;
  solved by preconditioned CG with the block-Jacobi preconditioner diag-blocks(S)⁻¹ (Ceres'
  ITERATIVE_SCHUR + SCHUR_JACOBI) — S is never formed, S·x = U_d x - W V_d⁻¹ Wᵀ x;
* back-substitution δp = V_d⁻¹ (-g_p - Wᵀ δc);
* update: rotation by a left-multiplied increment R <- exp([δr]x) R (the tangent space the J^TJ
  build differentiates in, oracle/sfm_oracle_ba.c), everything else additive;
* LM: accept iff the cost decreases; ρ = actual / predicted decrease, predicted = -(gᵀδ +
  ½ δᵀ JᵀJ δ); accepted: λ *= max(1/3, 1 - (2ρ-1)³), ν = 2; rejected: λ *= ν, ν *= 2 (Nielsen).
"""
from __future__ import annotations

import numpy as np

import oracle as O

DIAG_MIN, DIAG_MAX = 1e-6, 1e32


def damp(A: np.ndarray, lam: float) -> np.ndarray:
    """A [..., n, n] + lam * clamp(diag(A))."""
    d = np.clip(np.diagonal(A, axis1=-2, axis2=-1), DIAG_MIN, DIAG_MAX)
    out = A.copy()
    idx = np.arange(A.shape[-1])
    out[..., idx, idx] += lam * d
    return out


def point_inverse(V: np.ndarray, lam: float, n_obs_pt: np.ndarray) -> np.ndarray:
    """V_d⁻¹ per point; zero for points without observations."""
    Vd = damp(V, lam)
    Vinv = np.zeros_like(V)
    ok = n_obs_pt > 0
    Vinv[ok] = np.linalg.inv(Vd[ok])
    return Vinv


def schur_rhs_and_precond(U, V, W, gc, gp, cam_idx, pt_idx, lam):
    n_cam, n_pt = U.shape[0], V.shape[0]
    n_obs_pt = np.bincount(pt_idx, minlength=n_pt)
    Vinv = point_inverse(V, lam, n_obs_pt)
    vg = np.einsum("pij,pj->pi", Vinv, gp)
    Ud = damp(U, lam)
    WV = np.einsum("oij,ojk->oik", W, Vinv[pt_idx])            # [o, 8, 3]
    S_diag = Ud.copy()
    np.subtract.at(S_diag, cam_idx, np.einsum("oik,ojk->oij", WV, W))
    b = -gc.copy()
    np.add.at(b, cam_idx, np.einsum("oij,oj->oi", W, vg[pt_idx]))
    return Ud, Vinv, vg, S_diag, b


def schur_matvec(Ud, Vinv, W, cam_idx, pt_idx, x):
    """S x = U_d x - Σ_o W_o V_d⁻¹ Σ_o' W_o'ᵀ x."""
    n_pt = Vinv.shape[0]
    t = np.zeros((n_pt, 3))
    np.add.at(t, pt_idx, np.einsum("oij,oi->oj", W, x[cam_idx]))
    t = np.einsum("pij,pj->pi", Vinv, t)
    y = np.einsum("cij,cj->ci", Ud, x)
    np.subtract.at(y, cam_idx, np.einsum("oij,oj->oi", W, t[pt_idx]))
    return y


def schur_pcg(U, V, W, gc, gp, cam_idx, pt_idx, lam, max_iter=100, tol=1e-10):
    """The GPU solver's algorithm (same recurrences; summation orders differ).

    Returns (dc [n_cam, 8], dp [n_pt, 3], iters, |r|/|b|)."""
    cam_idx = np.asarray(cam_idx)
    pt_idx = np.asarray(pt_idx)
    Ud, Vinv, vg, S_diag, b = schur_rhs_and_precond(U, V, W, gc, gp, cam_idx, pt_idx, lam)
    M = np.linalg.inv(S_diag)
    x = np.zeros_like(b)
    r = b.copy()
    bn = np.sqrt(np.sum(b * b))
    z = np.einsum("cij,cj->ci", M, r)
    p = z.copy()
    rz = np.sum(r * z)
    it = 0
    rn = np.sqrt(np.sum(r * r))
    while it < max_iter and rn > tol * bn:
        q = schur_matvec(Ud, Vinv, W, cam_idx, pt_idx, p)
        alpha = rz / np.sum(p * q)
        x += alpha * p
        r -= alpha * q
        it += 1
        rn = np.sqrt(np.sum(r * r))
        if rn <= tol * bn:
            break
        z = np.einsum("cij,cj->ci", M, r)
        rz_new = np.sum(r * z)
        p = z + (rz_new / rz) * p
        rz = rz_new
    dp = back_substitute(Vinv, vg, W, cam_idx, pt_idx, x)
    return x, dp, it, (rn / bn if bn > 0 else 0.0)


def back_substitute(Vinv, vg, W, cam_idx, pt_idx, dc):
    t = np.zeros_like(vg)
    np.add.at(t, pt_idx, np.einsum("oij,oi->oj", W, dc[cam_idx]))
    return -vg - np.einsum("pij,pj->pi", Vinv, t)


def dense_normal_matrix(U, V, W, cam_idx, pt_idx):
    """Full J^TJ (cameras first, then points) from the blocks — small problems only."""
    n_cam, n_pt = U.shape[0], V.shape[0]
    n = 8 * n_cam + 3 * n_pt
    H = np.zeros((n, n))
    for c in range(n_cam):
        H[8 * c:8 * c + 8, 8 * c:8 * c + 8] = U[c]
    for p in range(n_pt):
        o = 8 * n_cam + 3 * p
        H[o:o + 3, o:o + 3] = V[p]
    for k, (c, p) in enumerate(zip(cam_idx, pt_idx)):
        o = 8 * n_cam + 3 * p
        H[8 * c:8 * c + 8, o:o + 3] += W[k]
        H[o:o + 3, 8 * c:8 * c + 8] += W[k].T
    return H


def solve_dense(U, V, W, gc, gp, cam_idx, pt_idx, lam):
    """Direct solve of the damped normal equations (the Schur/PCG result's reference)."""
    H = dense_normal_matrix(U, V, W, cam_idx, pt_idx)
    d = np.clip(np.diag(H).copy(), DIAG_MIN, DIAG_MAX)
    n_obs_pt = np.bincount(pt_idx, minlength=V.shape[0])
    n_cam = U.shape[0]
    empty = np.repeat(n_obs_pt == 0, 3)                     # unobserved points: δp = 0
    keep = np.concatenate([np.ones(8 * n_cam, bool), ~empty])
    Hd = H + lam * np.diag(d)
    g = np.concatenate([gc.reshape(-1), gp.reshape(-1)])
    x = np.zeros_like(g)
    x[keep] = np.linalg.solve(Hd[np.ix_(keep, keep)], -g[keep])
    return x[:8 * n_cam].reshape(-1, 8), x[8 * n_cam:].reshape(-1, 3)


def model_terms(U, V, W, gc, gp, cam_idx, pt_idx, dc, dp):
    """(gᵀδ, δᵀ JᵀJ δ) from the blocks."""
    gd = np.sum(gc * dc) + np.sum(gp * dp)
    q = np.einsum("ci,cij,cj->", dc, U, dc) + np.einsum("pi,pij,pj->", dp, V, dp)
    q += 2.0 * np.einsum("oi,oij,oj->", dc[cam_idx], W, dp[pt_idx])
    return gd, q


def _rotmat(r):
    th2 = float(np.dot(r, r))
    if th2 <= 1e-20:                                       # as oracle_ba_obs / the GPU
        return np.array([[1.0, -r[2], r[1]], [r[2], 1.0, -r[0]], [-r[1], r[0], 1.0]])
    th = np.sqrt(th2)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def _angle_axis(R):
    """log map, stable near 0 and π."""
    c = np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = 0.5 * np.linalg.norm(w)
    th = np.arctan2(s, c)
    if s > 1e-7:
        return w * (th / (2.0 * s))
    if c > 0:                                              # th ~ 0
        return 0.5 * w
    # th ~ π: axis from the symmetric part
    B = 0.5 * (R + np.eye(3))
    i = int(np.argmax(np.diag(B)))
    a = B[:, i] / np.sqrt(B[i, i])
    if np.dot(a, w) < 0:
        a = -a
    return th * a / np.linalg.norm(a)


def update(cams, pts, dc, dp):
    """cams ⊕ dc (left rotation increment, additive t, f, k1), pts + dp."""
    out = np.array(cams, np.float64, copy=True)
    for c in range(len(out)):
        if np.any(dc[c, :3] != 0.0):  # δr = 0 exactly (a held rotation) keeps r bit for bit
            out[c, :3] = _angle_axis(_rotmat(dc[c, :3]) @ _rotmat(out[c, :3]))
        out[c, 3:] += dc[c, 3:]
    return out, np.asarray(pts, np.float64) + dp


def cost(cams, pp, pts, cam_idx, pt_idx, uv, loss_s=0.0):
    return O.ba_jtj(cams, pp, pts, cam_idx, pt_idx, uv, loss_s)["cost"]


def fix_params(lin, cam_idx, fixed):
    """Fixed parameters (sfm_ba_fix_params, csrc/ba_solve.hip): rows/columns of U for the
    parameters marked in fixed [n_cam, 8] become the identity's, their g_c entries and W rows 0,
    so the damped Schur solve returns delta = 0 for them.  In place; returns lin."""
    if fixed is None:
        return lin
    fixed = np.asarray(fixed, bool)
    U, W, gc = lin["U"], lin["W"], lin["gc"]
    for c, i in zip(*np.nonzero(fixed)):
        U[c, i, :] = 0.0
        U[c, :, i] = 0.0
        U[c, i, i] = 1.0
        gc[c, i] = 0.0
    rows = fixed[np.asarray(cam_idx)]             # [n_obs, 8]
    W[rows] = 0.0
    return lin


def bundle_adjust(cams, pp, pts, cam_idx, pt_idx, uv, loss_s=0.0, max_iter=50, lam0=1e-4,
                  ftol=1e-12, max_cg=200, cg_tol=1e-10, fixed=None):
    """LM loop of the spec; returns (cams, pts, history [(cost, lam, accepted, cg_iters)]).
    fixed: optional [n_cam, 8] bool mask of parameters held at their values (fix_params)."""
    cams = np.array(cams, np.float64, copy=True)
    pts = np.array(pts, np.float64, copy=True)
    lam, nu = lam0, 2.0
    hist = []
    lin = fix_params(O.ba_jtj(cams, pp, pts, cam_idx, pt_idx, uv, loss_s), cam_idx, fixed)
    for _ in range(max_iter):
        dc, dp, it, _ = schur_pcg(lin["U"], lin["V"], lin["W"], lin["gc"], lin["gp"], cam_idx,
                                  pt_idx, lam, max_cg, cg_tol)
        gd, q = model_terms(lin["U"], lin["V"], lin["W"], lin["gc"], lin["gp"], cam_idx, pt_idx,
                            dc, dp)
        pred = -(gd + 0.5 * q)
        c2, p2 = update(cams, pts, dc, dp)
        new = cost(c2, pp, p2, cam_idx, pt_idx, uv, loss_s)
        old = lin["cost"]
        if new < old and pred > 0:
            rho = (old - new) / pred
            cams, pts = c2, p2
            lam *= max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3)
            nu = 2.0
            hist.append((new, lam, True, it))
            if old - new <= ftol * old:
                break
            lin = fix_params(O.ba_jtj(cams, pp, pts, cam_idx, pt_idx, uv, loss_s), cam_idx, fixed)
        else:
            lam *= nu
            nu *= 2.0
            hist.append((old, lam, False, it))
            if lam > 1e16:
                break
    return cams, pts, hist


def _left_jacobian(r):
    th = np.linalg.norm(r)
    K = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
    if th < 1e-8:
        return np.eye(3) + 0.5 * K
    return np.eye(3) + (1 - np.cos(th)) / th ** 2 * K + (th - np.sin(th)) / th ** 3 * K @ K


def residuals_and_jacobian(cams, pp, pts, cam_idx, pt_idx, uv):
    """Residual vector [2 n_obs] and sparse Jacobian in the plain parametrisation
    (angle-axis, t, f, k1 per camera; X per point) for scipy.optimize.least_squares — the
    rotation column is the left-increment Jacobian times the SO(3) left Jacobian J_l(r)."""
    from scipy.sparse import csr_matrix
    cams = np.ascontiguousarray(cams, np.float64)
    pts = np.ascontiguousarray(pts, np.float64)
    pp = np.ascontiguousarray(pp, np.float64)
    uv = np.ascontiguousarray(uv, np.float64)
    n_cam, n_pt, n_obs = len(cams), len(pts), len(cam_idx)
    Jl = [_left_jacobian(c[:3]) for c in cams]
    rows, cols, vals = [], [], []
    res = np.zeros(2 * n_obs)
    r2, Jc, Jp, w, rho = (np.zeros(2), np.zeros(16), np.zeros(6), np.zeros(1), np.zeros(1))
    for o in range(n_obs):
        c, p = int(cam_idx[o]), int(pt_idx[o])
        O.lib().oracle_ba_obs(O._p(cams[c]), O._p(pp[c]), O._p(pts[p]), O._p(uv[o]), 0.0,
                              O._p(r2), O._p(Jc), O._p(Jp), O._p(w), O._p(rho))
        res[2 * o:2 * o + 2] = r2
        J = Jc.reshape(2, 8).copy()
        J[:, :3] = J[:, :3] @ Jl[c]
        for a in range(2):
            rows += [2 * o + a] * 11
            cols += list(range(8 * c, 8 * c + 8)) + list(range(8 * n_cam + 3 * p, 8 * n_cam + 3 * p + 3))
            vals += list(J[a]) + list(Jp[3 * a:3 * a + 3])
    Jm = csr_matrix((vals, (rows, cols)), shape=(2 * n_obs, 8 * n_cam + 3 * n_pt))
    return res, Jm
