"""GPU parity: BA linearisation (K3) vs the CPU oracle (fp64, tolerance: reduction order differs).

north_star criterion: reprojection error within 1e-4 px — the residuals here agree to ~1e-9 px.
J^TJ blocks are compared relatively (1e-9) against the oracle's sequential sums.
"""
import numpy as np
import pytest

import oracle as O
import sfmcore
import synth

pytestmark = pytest.mark.gpu


def _gpu_ba(ctx, prob, loss_s=0.0):
    import torch
    nc, npt = prob["cams"].shape[0], prob["pts"].shape[0]
    pt_ptr, _ = sfmcore.csr_by(prob["pt_idx"], npt)
    cam_ptr, cam_obs = sfmcore.csr_by(prob["cam_idx"], nc)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    out = ctx.ba_jtj(T(prob["cams"]), T(prob["pp"]), T(prob["pts"]), T(prob["cam_idx"]),
                     T(prob["pt_idx"]), T(prob["uv"]), T(pt_ptr), T(cam_ptr), T(cam_obs),
                     loss_s=loss_s)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("loss_s", [0.0, 2.0])
def test_ba_jtj_matches_oracle(ctx, loss_s):
    prob = synth.make_ba_problem(20, 400, obs_per_pt=5, seed=1)
    g = _gpu_ba(ctx, prob, loss_s)
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"], loss_s=loss_s)
    np.testing.assert_allclose(g["res"], o["res"], rtol=0, atol=1e-7)
    for k in ("U", "V", "W", "gc", "gp"):
        scale = np.abs(o[k]).max()
        np.testing.assert_allclose(g[k], o[k], rtol=1e-9, atol=1e-11 * scale, err_msg=k)
    assert abs(g["cost"][0] - o["cost"]) <= 1e-9 * abs(o["cost"])


def test_ba_empty_camera_and_point(ctx):
    prob = synth.make_ba_problem(6, 50, obs_per_pt=2, seed=2)
    # add an unobserved camera and an unobserved point
    prob["cams"] = np.concatenate([prob["cams"], prob["cams"][:1]])
    prob["pp"] = np.concatenate([prob["pp"], prob["pp"][:1]])
    prob["pts"] = np.concatenate([prob["pts"], prob["pts"][:1]])
    g = _gpu_ba(ctx, prob)
    assert np.all(g["U"][-1] == 0) and np.all(g["V"][-1] == 0)
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"])
    np.testing.assert_allclose(g["U"], o["U"], rtol=1e-9, atol=1e-6)


def test_ba_long_tracks_and_gaps(ctx):
    """Points observed by up to 150 cameras (segments spanning several 64-observation waves of
    the fused point reduction), points with 1 observation, and unobserved points in between."""
    rng = np.random.default_rng(7)
    long = synth.make_ba_problem(160, 6, obs_per_pt=150, seed=3)
    short = synth.make_ba_problem(160, 300, obs_per_pt=3, seed=4)
    # interleave: point-major order with long tracks at varying offsets, drop every 7th point
    n_long, n_short = 6, 300
    pts = np.concatenate([long["pts"], short["pts"]])
    cam_idx, pt_idx, uv = [], [], []
    order = rng.permutation(n_long + n_short)
    for new_id, old in enumerate(order):
        if new_id % 7 == 3:
            continue  # unobserved point
        src, k = (long, old) if old < n_long else (short, old - n_long)
        sel = np.nonzero(src["pt_idx"] == k)[0]
        if old >= n_long and new_id % 5 == 0:
            sel = sel[:1]  # single observation
        cam_idx.append(src["cam_idx"][sel])
        pt_idx.append(np.full(len(sel), new_id, np.int32))
        uv.append(src["uv"][sel])
    prob = dict(cams=long["cams"], pp=long["pp"], pts=pts[order],
                cam_idx=np.concatenate(cam_idx).astype(np.int32),
                pt_idx=np.concatenate(pt_idx).astype(np.int32), uv=np.concatenate(uv))
    g = _gpu_ba(ctx, prob, loss_s=1.0)
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"], loss_s=1.0)
    np.testing.assert_allclose(g["res"], o["res"], rtol=0, atol=1e-7)
    for k in ("U", "V", "W", "gc", "gp"):
        scale = np.abs(o[k]).max()
        np.testing.assert_allclose(g[k], o[k], rtol=1e-9, atol=1e-11 * scale, err_msg=k)
    assert np.all(g["V"][3::7] == 0) and np.all(g["gp"][3::7] == 0)
    assert abs(g["cost"][0] - o["cost"]) <= 1e-9 * abs(o["cost"])
