"""CPU: the bundle-adjustment solve restatement (oracle/ba_lm.py) against independent checks.

* Schur-complement PCG vs a direct dense solve of the damped normal equations;
* the LM model terms (gᵀδ, δᵀJᵀJδ) vs the dense J^TJ;
* the SO(3) update vs the rotation-matrix product it defines (incl. angles near 0 and π);
* the LM loop vs scipy.optimize.least_squares (MINPACK 'lm', analytic Jacobian in the plain
  angle-axis parametrisation): converged per-observation reprojection errors within 1e-4 px
  (the north_star BA tolerance; they agree to ~1e-8 px).
"""
import numpy as np
import pytest

import ba_lm as L
import oracle as O
import synth


def _lin(prob, loss_s=0.0):
    return O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                    prob["uv"], loss_s)


@pytest.mark.parametrize("lam", [1e-4, 1e-1, 10.0])
def test_schur_pcg_matches_dense_solve(lam):
    prob = synth.make_ba_problem(6, 120, obs_per_pt=4, seed=3, perturb=2e-3)
    lin = _lin(prob)
    args = (lin["U"], lin["V"], lin["W"], lin["gc"], lin["gp"], prob["cam_idx"], prob["pt_idx"])
    dc, dp, it, rel = L.schur_pcg(*args, lam, max_iter=500, tol=1e-13)
    dc2, dp2 = L.solve_dense(*args, lam)
    assert rel <= 1e-13 and it < 500
    np.testing.assert_allclose(dc, dc2, rtol=0, atol=1e-9 * np.abs(dc2).max())
    np.testing.assert_allclose(dp, dp2, rtol=0, atol=1e-9 * np.abs(dp2).max())


def test_schur_pcg_unobserved_camera_and_point():
    prob = synth.make_ba_problem(5, 60, obs_per_pt=3, seed=5)
    prob["cams"] = np.concatenate([prob["cams"], prob["cams"][:1]])
    prob["pp"] = np.concatenate([prob["pp"], prob["pp"][:1]])
    prob["pts"] = np.concatenate([prob["pts"], prob["pts"][:1]])
    lin = _lin(prob)
    args = (lin["U"], lin["V"], lin["W"], lin["gc"], lin["gp"], prob["cam_idx"], prob["pt_idx"])
    dc, dp, _, _ = L.schur_pcg(*args, 1e-3, max_iter=500, tol=1e-13)
    dc2, dp2 = L.solve_dense(*args, 1e-3)
    assert np.all(dc[-1] == 0) and np.all(dp[-1] == 0)
    np.testing.assert_allclose(dc, dc2, rtol=0, atol=1e-9 * np.abs(dc2).max())
    np.testing.assert_allclose(dp, dp2, rtol=0, atol=1e-9 * np.abs(dp2).max())


def test_model_terms_match_dense():
    prob = synth.make_ba_problem(4, 50, obs_per_pt=3, seed=6)
    lin = _lin(prob, loss_s=3.0)
    rng = np.random.default_rng(0)
    dc, dp = rng.normal(size=(4, 8)), rng.normal(size=(50, 3))
    gd, q = L.model_terms(lin["U"], lin["V"], lin["W"], lin["gc"], lin["gp"], prob["cam_idx"],
                          prob["pt_idx"], dc, dp)
    H = L.dense_normal_matrix(lin["U"], lin["V"], lin["W"], prob["cam_idx"], prob["pt_idx"])
    d = np.concatenate([dc.reshape(-1), dp.reshape(-1)])
    g = np.concatenate([lin["gc"].reshape(-1), lin["gp"].reshape(-1)])
    assert abs(gd - g @ d) <= 1e-10 * abs(g) @ abs(d)
    assert abs(q - d @ H @ d) <= 1e-10 * abs(d) @ abs(H) @ abs(d)


def test_update_is_left_rotation_increment():
    rng = np.random.default_rng(1)
    rs = [rng.normal(size=3) * s for s in (1e-12, 1e-6, 0.3, 1.0, 2.5)]
    rs.append(np.array([np.pi - 1e-9, 0.0, 0.0]))
    rs.append(np.array([0.0, 0.0, -np.pi + 1e-4]))
    cams = np.zeros((len(rs), 8))
    cams[:, :3] = rs
    cams[:, 3:] = rng.normal(size=(len(rs), 5))
    dc = rng.normal(size=cams.shape) * 1e-2
    dc[0, :3] = 0.0
    out, _ = L.update(cams, np.zeros((1, 3)), dc, np.zeros((1, 3)))
    for c in range(len(rs)):
        R = L._rotmat(dc[c, :3]) @ L._rotmat(cams[c, :3])
        np.testing.assert_allclose(L._rotmat(out[c, :3]), R, atol=1e-9)
        assert np.linalg.norm(out[c, :3]) <= np.pi + 1e-12
    np.testing.assert_allclose(out[:, 3:], cams[:, 3:] + dc[:, 3:], rtol=0, atol=0)


def _scipy_solution(prob):
    from scipy.optimize import least_squares
    nc, npt = len(prob["cams"]), len(prob["pts"])
    unpack = lambda x: (x[:8 * nc].reshape(nc, 8), x[8 * nc:].reshape(npt, 3))

    def fj(x):
        c, p = unpack(x)
        return L.residuals_and_jacobian(c, prob["pp"], p, prob["cam_idx"], prob["pt_idx"],
                                        prob["uv"])
    x0 = np.concatenate([prob["cams"].reshape(-1), prob["pts"].reshape(-1)])
    r = least_squares(lambda x: fj(x)[0], x0, jac=lambda x: fj(x)[1].toarray(), method="lm",
                      ftol=1e-15, xtol=1e-15, gtol=1e-15, max_nfev=2000)
    return np.linalg.norm(r.fun.reshape(-1, 2), axis=1), r.cost


def test_lm_matches_scipy_least_squares():
    prob = synth.make_ba_problem(6, 120, obs_per_pt=4, seed=3, perturb=2e-3)
    cams, pts, hist = L.bundle_adjust(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"],
                                      prob["pt_idx"], prob["uv"], max_iter=100)
    assert hist[-1][0] < hist[0][0]
    o = O.ba_jtj(cams, prob["pp"], pts, prob["cam_idx"], prob["pt_idx"], prob["uv"])
    err = np.linalg.norm(o["res"], axis=1)
    err_ref, cost_ref = _scipy_solution(prob)
    assert np.abs(err - err_ref).max() < 1e-4            # px, the north_star BA tolerance
    assert abs(o["cost"] - cost_ref) <= 1e-9 * cost_ref


def test_fixed_params_give_zero_step():
    """fix_params (the spec of sfm_ba_fix_params): the damped Schur solve returns exactly 0 for
    every held parameter, and the free parameters still solve the reduced system."""
    prob = synth.make_ba_problem(7, 150, obs_per_pt=4, seed=8, perturb=2e-3)
    rng = np.random.default_rng(1)
    fixed = rng.random((7, 8)) < 0.3
    fixed[:, 6:] = True
    lin = L.fix_params(_lin(prob), prob["cam_idx"], fixed)
    dc, dp, it, _ = L.schur_pcg(lin["U"], lin["V"], lin["W"], lin["gc"], lin["gp"],
                                prob["cam_idx"], prob["pt_idx"], 1e-3, 500, 1e-12)
    assert (dc[fixed] == 0.0).all() and np.abs(dc[~fixed]).max() > 0
    dcd, dpd = L.solve_dense(lin["U"], lin["V"], lin["W"], lin["gc"], lin["gp"],
                             prob["cam_idx"], prob["pt_idx"], 1e-3)
    np.testing.assert_allclose(dc, dcd, rtol=0, atol=1e-8 * np.abs(dcd).max())


def test_gauge_fixed_lm_reaches_the_same_optimum():
    """The 7-DoF similarity gauge (reference pose + one translation coordinate of a second
    camera, reconstruction.gauge_mask) removes the null space without changing the optimum: the
    converged cost equals the gauge-free one, and the held parameters do not move."""
    import reconstruction as R
    prob = synth.make_ba_problem(8, 200, obs_per_pt=4, seed=9, perturb=3e-3)
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0)
    assert fixed.sum() == 7 and fixed[0, :6].all()
    cg, pg, hg = L.bundle_adjust(*args, max_iter=100, fixed=fixed)
    cf, pf, hf = L.bundle_adjust(*args, max_iter=100)
    assert abs(hg[-1][0] - hf[-1][0]) <= 1e-7 * hf[-1][0]
    np.testing.assert_array_equal(cg[fixed], prob["cams"][fixed])
