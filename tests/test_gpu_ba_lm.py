"""GPU parity: the bundle-adjustment step (K4: Schur-complement PCG, update, trial cost) and the
LM loop built on it, vs oracle/ba_lm.py and scipy.optimize.least_squares.

Tolerances (fp64; reduction orders differ from the oracle's, so not bit-exact):
  solve: δ vs the oracle's PCG and the dense direct solve, relative 1e-8 of max|δ|;
  cost / model terms: relative 1e-11;  update: 1e-12 absolute;
  LM end to end: per-observation reprojection error within 1e-4 px of scipy's converged
  solution (the north_star BA criterion; they agree to ~1e-8 px).
"""
import numpy as np
import pytest

import ba_lm as L
import oracle as O
import reconstruction as R
import sfmcore
import synth

pytestmark = pytest.mark.gpu


def _problem(prob, loss_s=0.0):
    import torch
    P = R.BAProblem(prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], len(prob["cams"]),
                    len(prob["pts"]))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    return P, cams, pts, P.linearize(cams, pts, loss_s)


@pytest.mark.parametrize("lam,loss_s", [(1e-4, 0.0), (1e-1, 0.0), (1e-3, 2.0)])
def test_solve_matches_oracle(lam, loss_s):
    prob = synth.make_ba_problem(12, 400, obs_per_pt=4, seed=11, perturb=2e-3)
    P, _, _, lin = _problem(prob, loss_s)
    dc, dp, info = P.solve(lin, lam, max_iter=500, tol=1e-12)
    dc, dp, info = dc.cpu().numpy(), dp.cpu().numpy(), info.cpu().numpy()
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"], loss_s)
    args = (o["U"], o["V"], o["W"], o["gc"], o["gp"], prob["cam_idx"], prob["pt_idx"])
    odc, odp, oit, _ = L.schur_pcg(*args, lam, max_iter=500, tol=1e-12)
    ddc, ddp = L.solve_dense(*args, lam)
    assert info[1] <= 1e-12 and abs(info[0] - oit) <= 3 and info[4] == 0
    for a, b in ((dc, odc), (dc, ddc)):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-8 * np.abs(b).max())
    for a, b in ((dp, odp), (dp, ddp)):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-8 * np.abs(b).max())
    gd, q = L.model_terms(*args[:5], prob["cam_idx"], prob["pt_idx"], dc, dp)
    assert abs(info[2] - gd) <= 1e-11 * abs(gd) and abs(info[3] - q) <= 1e-11 * abs(q)


def test_solve_long_tracks_match_oracle():
    """Points with more than 64 observations (taken by the point pass's long-track blocks, a wave
    per point) mixed with short ones in the same blocks: δ as the oracle's PCG and the dense
    solve."""
    counts = np.where(np.arange(90) % 7 == 0, 100 + np.arange(90) % 50, 4)
    prob = synth.make_ba_problem(160, 90, obs_per_pt=counts, seed=29, perturb=2e-3)
    assert (np.bincount(prob["pt_idx"]) > 64).sum() == 13
    P, _, _, lin = _problem(prob, 2.0)
    dc, dp, info = P.solve(lin, 1e-3, max_iter=500, tol=1e-12)
    dc, dp, info = dc.cpu().numpy(), dp.cpu().numpy(), info.cpu().numpy()
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"], 2.0)
    args = (o["U"], o["V"], o["W"], o["gc"], o["gp"], prob["cam_idx"], prob["pt_idx"])
    odc, odp, oit, _ = L.schur_pcg(*args, 1e-3, max_iter=500, tol=1e-12)
    ddc, ddp = L.solve_dense(*args, 1e-3)
    assert info[1] <= 1e-12 and abs(info[0] - oit) <= 3 and info[4] == 0
    for a, b in ((dc, odc), (dc, ddc)):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-8 * np.abs(b).max())
    for a, b in ((dp, odp), (dp, ddp)):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-8 * np.abs(b).max())


def test_solve_unobserved_camera_and_point():
    prob = synth.make_ba_problem(5, 60, obs_per_pt=3, seed=5)
    for k in ("cams", "pp", "pts"):
        prob[k] = np.concatenate([prob[k], prob[k][:1]])
    P, _, _, lin = _problem(prob)
    dc, dp, info = (t.cpu().numpy() for t in P.solve(lin, 1e-3, max_iter=500, tol=1e-13))
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"])
    ddc, ddp = L.solve_dense(o["U"], o["V"], o["W"], o["gc"], o["gp"], prob["cam_idx"],
                             prob["pt_idx"], 1e-3)
    assert np.all(dc[-1] == 0) and np.all(dp[-1] == 0)
    np.testing.assert_allclose(dc, ddc, rtol=0, atol=1e-8 * np.abs(ddc).max())
    np.testing.assert_allclose(dp, ddp, rtol=0, atol=1e-8 * np.abs(ddp).max())


def test_solve_zero_iterations_and_determinism():
    prob = synth.make_ba_problem(8, 200, obs_per_pt=3, seed=12)
    P, _, _, lin = _problem(prob)
    dc0, dp0, info0 = (t.cpu().numpy() for t in P.solve(lin, 1e-2, max_iter=0))
    assert np.all(dc0 == 0) and info0[0] == 0
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"])
    Vinv = L.point_inverse(o["V"], 1e-2, np.bincount(prob["pt_idx"], minlength=200))
    np.testing.assert_allclose(dp0, -np.einsum("pij,pj->pi", Vinv, o["gp"]), rtol=1e-10,
                               atol=1e-14)
    a = [t.cpu().numpy() for t in P.solve(lin, 1e-2, max_iter=50, tol=1e-9)]
    b = [t.cpu().numpy() for t in P.solve(lin, 1e-2, max_iter=50, tol=1e-9)]
    for x, y in zip(a, b):
        assert np.array_equal(x, y)        # fixed-order sums: bit-identical reruns


@pytest.mark.parametrize("loss_s", [0.0, 1.5])
def test_cost_matches_oracle(loss_s):
    prob = synth.make_ba_problem(10, 300, obs_per_pt=4, seed=13)
    P, cams, pts, _ = _problem(prob)
    c = float(P.cost(cams, pts, loss_s).item())
    o = L.cost(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
               prob["uv"], loss_s)
    assert abs(c - o) <= 1e-11 * o


def test_update_matches_oracle():
    import torch
    rng = np.random.default_rng(2)
    rs = [rng.normal(size=3) * s for s in (0.0, 1e-12, 1e-6, 0.3, 1.0, 2.5)]
    rs += [np.array([np.pi - 1e-9, 0.0, 0.0]), np.array([0.0, 0.0, -np.pi + 1e-4])]
    cams = np.zeros((len(rs), 8))
    cams[:, :3] = rs
    cams[:, 3:] = rng.normal(size=(len(rs), 5))
    dc = rng.normal(size=cams.shape) * 1e-2
    pts, dp = rng.normal(size=(37, 3)), rng.normal(size=(37, 3))
    ctx = R.sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    co, po = (t.cpu().numpy() for t in ctx.ba_update(T(cams), T(dc), T(pts), T(dp)))
    oc, op = L.update(cams, pts, dc, dp)
    for c in range(len(rs)):
        np.testing.assert_allclose(L._rotmat(co[c, :3]), L._rotmat(oc[c, :3]), atol=1e-12)
    np.testing.assert_allclose(co[:, 3:], oc[:, 3:], rtol=0, atol=0)
    np.testing.assert_allclose(po, op, rtol=0, atol=0)


def test_bundle_adjust_matches_scipy_and_oracle():
    from test_ba_lm_cpu import _scipy_solution
    prob = synth.make_ba_problem(6, 120, obs_per_pt=4, seed=3, perturb=2e-3)
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    cams, pts, hist = R.bundle_adjust(*args, max_iter=100)
    ocams, opts, ohist = L.bundle_adjust(*args, max_iter=100)
    o = O.ba_jtj(cams, prob["pp"], pts, prob["cam_idx"], prob["pt_idx"], prob["uv"])
    err = np.linalg.norm(o["res"], axis=1)
    err_ref, cost_ref = _scipy_solution(prob)
    assert np.abs(err - err_ref).max() < 1e-4            # px
    assert abs(hist[-1][0] - ohist[-1][0]) <= 1e-9 * ohist[-1][0]
    assert abs(hist[-1][0] - cost_ref) <= 1e-9 * cost_ref


def test_bundle_adjust_cauchy_descends():
    prob = synth.make_ba_problem(10, 300, obs_per_pt=4, seed=14, perturb=3e-3)
    prob["uv"][::17] += 40.0                              # gross outliers
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    cams, pts, hist = R.bundle_adjust(*args, loss_s=2.0, max_iter=60)
    ocams, opts, ohist = L.bundle_adjust(*args, loss_s=2.0, max_iter=60)
    costs = [h[0] for h in hist if h[2]]
    assert all(b <= a for a, b in zip(costs, costs[1:]))
    assert abs(hist[-1][0] - ohist[-1][0]) <= 1e-7 * ohist[-1][0]


def test_fix_params_matches_oracle():
    """sfm_ba_fix_params on the GPU blocks == oracle/ba_lm.py fix_params on the oracle's."""
    import torch
    prob = synth.make_ba_problem(9, 150, obs_per_pt=4, seed=17, perturb=2e-3)
    P, cams, pts, lin = _problem(prob)
    rng = np.random.default_rng(5)
    fixed = rng.random((9, 8)) < 0.3
    P.ctx.ba_fix_params(lin, P.cam_idx, torch.from_numpy(fixed.astype(np.uint8)).cuda())
    o = L.fix_params(O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"],
                              prob["pt_idx"], prob["uv"]), prob["cam_idx"], fixed)
    for k in ("U", "W", "gc"):
        g = lin[k].cpu().numpy()
        np.testing.assert_allclose(g, o[k], rtol=1e-9, atol=1e-11 * np.abs(o[k]).max(), err_msg=k)
    g = lin["U"].cpu().numpy()
    c, i = np.nonzero(fixed)
    assert (g[c, i, i] == 1.0).all() and (lin["gc"].cpu().numpy()[fixed] == 0.0).all()


def test_bundle_adjust_gauge_and_known_intrinsics():
    """with the similarity gauge (reference pose + a scale coordinate) and known
    intrinsics held, the GPU LM matches the oracle LM under the same mask, every held parameter
    stays bit-identical, and the free cameras still converge; without the mask f drifts."""
    prob = synth.make_ba_problem(10, 300, obs_per_pt=4, seed=21, perturb=3e-3)
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    assert fixed.sum() == 7 + 2 * 10
    cams, pts, hist = R.bundle_adjust(*args, max_iter=60, fixed=fixed)
    ocams, opts, ohist = L.bundle_adjust(*args, max_iter=60, fixed=fixed)
    np.testing.assert_array_equal(cams[fixed], prob["cams"][fixed])
    assert abs(hist[-1][0] - ohist[-1][0]) <= 1e-9 * ohist[-1][0]
    assert hist[-1][0] < 0.1 * L.cost(*args)
    fcams, _, _ = R.bundle_adjust(*args, max_iter=60)
    assert np.abs(fcams[:, 6] - prob["cams"][:, 6]).max() > 1e-6   # the free gauge lets f move


def test_solve_without_observations():
    """An empty problem (no points, no observations; e.g. the incremental driver before any
    point survives): the solve runs on U / g_c alone, δc = -(U + λ diag U)⁻¹ g_c."""
    import torch
    import sfmcore
    ctx = sfmcore.context(0)
    f64, i32 = torch.float64, torch.int32
    U = torch.eye(8, dtype=f64, device="cuda").repeat(2, 1, 1) * 2.0
    lin = dict(U=U, V=torch.empty((0, 3, 3), dtype=f64, device="cuda"),
               W=torch.empty((0, 8, 3), dtype=f64, device="cuda"),
               gc=torch.ones((2, 8), dtype=f64, device="cuda"),
               gp=torch.empty((0, 3), dtype=f64, device="cuda"))
    e = torch.empty(0, dtype=i32, device="cuda")
    cam_ptr = torch.zeros(3, dtype=i32, device="cuda")
    pt_ptr = torch.zeros(1, dtype=i32, device="cuda")
    dc, dp, info = ctx.ba_solve(lin, e, e, pt_ptr, cam_ptr, e, 0.5, max_iter=20, tol=1e-12)
    torch.cuda.synchronize()
    np.testing.assert_allclose(dc.cpu().numpy(), -1.0 / 3.0, rtol=1e-12)
    assert dp.numel() == 0


def test_solve_async_default_under_graph_capture():
    """the zero-initialised poll is fully asynchronous — the solve can be captured in a
    HIP graph (torch.cuda.CUDAGraph on ROCm) and replayed; the replay equals the eager solve and
    the polled solve bit for bit."""
    import torch
    prob = synth.make_ba_problem(10, 300, obs_per_pt=4, seed=21, perturb=2e-3)
    P, _, _, lin = _problem(prob)
    eager = [t.clone() for t in P.solve(lin, 1e-3, max_iter=60, tol=1e-10, poll=0)]
    polled = [t.clone() for t in P.solve(lin, 1e-3, max_iter=60, tol=1e-10, poll=8)]
    out = [torch.empty_like(t) for t in eager]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):     # warm-up on the capture stream (workspace already sized)
        P.ctx.ba_solve(lin, P.cam_idx, P.pt_idx, P.pt_ptr, P.cam_ptr, P.cam_obs, 1e-3,
                       max_iter=60, tol=1e-10, out=out, poll=0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    for t in out:
        t.zero_()
    with torch.cuda.graph(g, stream=s):  # the context stays bound to s: no cross-stream hand-off
        P.ctx.ba_solve(lin, P.cam_idx, P.pt_idx, P.pt_ptr, P.cam_ptr, P.cam_obs, 1e-3,
                       max_iter=60, tol=1e-10, out=out, poll=0)
    g.replay()
    torch.cuda.synchronize()
    for a, b, c in zip(out, eager, polled):
        assert torch.equal(a, b) and torch.equal(b, c)


def test_c_abi_capture_with_zero_initialised_poll():
    """a C caller that captures sfm_ba_solve in a HIP graph with a zero-initialised
    sfm_ba_solve_params (sfm_version 1: poll 0 = never; version 2: poll 0 = every 8) must not hit
    a host synchronisation inside the capture: the library never polls on a capturing stream.
    Called through the raw ctypes binding (poll 0 and poll -1 structs); the replays equal the
    eager polled solve bit for bit."""
    import ctypes as C
    import torch
    prob = synth.make_ba_problem(10, 300, obs_per_pt=4, seed=22, perturb=2e-3)
    P, _, _, lin = _problem(prob)
    ref = [t.clone() for t in P.solve(lin, 1e-3, max_iter=60, tol=1e-10, poll=8)]
    ctx = P.ctx
    p = lambda t: C.c_void_p(t.data_ptr())
    s = torch.cuda.Stream()
    for poll in (0, -1):
        out = [torch.empty_like(t) for t in ref]
        prm = sfmcore.BaSolveParams(1e-3, 1e-10, 60, poll)

        def call():
            ctx._bind_stream()
            rc = ctx.lib.sfm_ba_solve(ctx.handle, ref[0].shape[0], ref[1].shape[0],
                                      P.cam_idx.shape[0], p(P.cam_idx), p(P.pt_idx), p(P.pt_ptr),
                                      p(P.cam_ptr), p(P.cam_obs), p(lin["U"]), p(lin["V"]),
                                      p(lin["W"]), p(lin["gc"]), p(lin["gp"]), C.byref(prm),
                                      p(out[0]), p(out[1]), p(out[2]))
            assert rc == 0, ctx.lib.sfm_last_error()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            call()                      # eager on the capture stream (polls: poll 0 = every 8)
        torch.cuda.synchronize()
        for a, b in zip(out, ref):
            assert torch.equal(a, b)
            a.zero_()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            call()
        g.replay()
        torch.cuda.synchronize()
        for a, b in zip(out, ref):
            assert torch.equal(a, b), poll


def _explicit_vs_oracle(prob, lam, loss_s, chunks=8):
    """The explicit reduced camera system (SchurSpec, sfm_ba_set_schur) against the oracle's PCG,
    the dense solve and the implicit chunked solve of the same problem."""
    import torch
    n_cam, n_pt = len(prob["cams"]), len(prob["pts"])
    args = (prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    Pi = R.BAProblem(*args, chunks=chunks)
    Pe = R.BAProblem(*args, chunks=chunks)
    Pe.set_schur()
    assert Pe.schur.n_slot > 0
    out = []
    for P in (Pi, Pe):
        lin = P.linearize(cams, pts, loss_s)
        dc, dp, info = P.solve(lin, lam, max_iter=500, tol=1e-12)
        out.append((dc.cpu().numpy(), dp.cpu().numpy(), info.cpu().numpy()))
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"], loss_s)
    oargs = (o["U"], o["V"], o["W"], o["gc"], o["gp"], prob["cam_idx"], prob["pt_idx"])
    odc, odp, oit, _ = L.schur_pcg(*oargs, lam, max_iter=500, tol=1e-12)
    ddc, ddp = L.solve_dense(*oargs, lam)
    dc, dp, info = out[1]
    assert info[1] <= 1e-12 and abs(info[0] - oit) <= 3 and info[4] == 0
    for a, b in ((dc, odc), (dc, ddc), (dc, out[0][0])):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-8 * np.abs(b).max())
    for a, b in ((dp, odp), (dp, ddp), (dp, out[0][1])):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-8 * np.abs(b).max())
    gd, q = L.model_terms(*oargs[:5], prob["cam_idx"], prob["pt_idx"], dc, dp)
    assert abs(info[2] - gd) <= 1e-11 * abs(gd) and abs(info[3] - q) <= 1e-11 * abs(q)
    return Pe


@pytest.mark.parametrize("lam,loss_s,chunks", [(1e-4, 0.0, 8), (1e-1, 0.0, 3), (1e-3, 2.0, 8)])
def test_explicit_schur_solve_matches_oracle(lam, loss_s, chunks):
    prob = synth.make_ba_problem(12, 400, obs_per_pt=4, seed=11, perturb=2e-3)
    _explicit_vs_oracle(prob, lam, loss_s, chunks)


def test_explicit_schur_duplicate_camera_and_long_tracks():
    """A point seen twice by one camera (its cross term lands on the diagonal block, both
    orientations), long tracks (many camera pairs per point) and an unobserved camera."""
    counts = np.where(np.arange(60) % 9 == 0, 40, 3)
    prob = synth.make_ba_problem(50, 60, obs_per_pt=counts, seed=31, perturb=2e-3)
    o = np.nonzero(prob["pt_idx"] == 1)[0]
    prob["cam_idx"] = prob["cam_idx"].copy()
    prob["cam_idx"][o[1]] = prob["cam_idx"][o[0]]       # same camera twice for point 1
    prob["cams"] = np.concatenate([prob["cams"], prob["cams"][:1]])
    prob["pp"] = np.concatenate([prob["pp"], prob["pp"][:1]])
    Pe = _explicit_vs_oracle(prob, 1e-3, 1.5)
    sc = Pe.schur.slot_cam.cpu().numpy()
    assert np.any(sc[:, 0] == sc[:, 1])                  # a diagonal slot from the duplicate


def test_explicit_schur_sharded_world1_bit_identical():
    """The explicit system through the sharded stages (SETUP + SCHUR, one exchange, local CG) in a
    world-size-1 RCCL group: the same bits as sfm_ba_solve with it."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    prob = synth.make_ba_problem(20, 600, obs_per_pt=5, seed=17, perturb=2e-3)
    n_cam, n_pt = len(prob["cams"]), len(prob["pts"])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    args = (prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt)
    P = R.BAProblem(*args, chunks=8)
    P.set_schur()
    lin = P.linearize(cams, pts)
    ref = [t.cpu().numpy() for t in P.solve(lin, 1e-3, max_iter=200, tol=1e-10)]
    # the same problem as a 1-rank shard (export form: n_total = 8, k0 = 0)
    S = R.BAProblem(*args, chunks=list(P.chunks.chunk_pt), n_total=8, k0=0)
    S.set_schur()
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        ar = R.make_allreduce()
        ls = S.linearize(cams, pts)
        tot = S.ctx.ba_chunk_tree(torch.cat([ls["U"].reshape(8, -1), ls["gc"].reshape(8, -1)], 1))
        ls["U"] = tot[:n_cam * 64].view(n_cam, 8, 8)
        ls["gc"] = tot[n_cam * 64:].view(n_cam, 8)
        got = [t.cpu().numpy() for t in S.solve_sharded(ls, 1e-3, ar, max_iter=200, tol=1e-10)]
        R.release_allreduce()
    finally:
        dist.destroy_process_group()
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("schur", [False, True])
def test_poll_first_and_look_ahead_give_the_same_bits(schur):
    """sfm_version 5 (round 6): where the solve polls its convergence flag — the first poll at
    `poll_first`, then every `poll`, each read after look-ahead iterations — moves no result: the
    iterations enqueued past convergence are empty.  The implicit CG and the explicit reduced
    camera system (chunk mode + sfm_ba_set_schur), against the every-8 default, bit for bit."""
    import torch
    prob = synth.make_ba_problem(10, 300, obs_per_pt=4, seed=23, perturb=2e-3)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    args = (prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], len(prob["cams"]),
            len(prob["pts"]))
    P = R.BAProblem(*args, chunks=R.ba_chunk_count() if schur else None)
    if schur:
        P.set_schur()
    lin = P.linearize(cams, pts)
    ref = [t.clone() for t in P.solve(lin, 1e-3, max_iter=60, tol=1e-6, poll=8)]
    assert 0 < ref[2][0].item() < 60   # converged before the cap: polls decide where it stops
    for poll, first in ((4, 1), (4, 3), (1, 0), (8, 100), (3, 7)):
        out = P.solve(lin, 1e-3, max_iter=60, tol=1e-6, poll=poll, poll_first=first)
        for a, b in zip(out, ref):
            assert torch.equal(a, b), (poll, first)
