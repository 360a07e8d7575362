"""GPU: the point-sharded bundle-adjustment step —
sfm_ba_solve_stage and reconstruction.bundle_adjust(shard=True).

Tolerances (fp64; sharding re-associates the camera-space sums over observations):
  world-size-1 RCCL group: δ bit-identical to sfm_ba_solve (the phases split the same sums), the
    LM model terms to 1e-12 relative (one extra fixed-order reduction), the LM end state to 1e-9;
  two ranks (gloo, one GPU): every rank returns the same bits; δ within 1e-8 of max|δ| of the
    unsharded solve, the LM end cost within 1e-9 relative, cameras within 1e-7 relative.
"""
import os

import numpy as np
import pytest

import reconstruction as R
import sfmcore
import synth

pytestmark = pytest.mark.gpu


def problem():
    return synth.make_ba_problem(9, 300, obs_per_pt=4, seed=17, perturb=3e-3)


def tiny_problem():
    return synth.make_ba_problem(4, 2, obs_per_pt=3, seed=5, perturb=1e-3)


def shard_solve(prob, rank, world, allreduce, lam=1e-3, **kw):
    """One sharded solve from the initial linearisation of `prob` on this rank's point shard."""
    import torch
    n_cam, n_pt = len(prob["cams"]), len(prob["pts"])
    pt_ptr, _ = sfmcore.csr_by(prob["pt_idx"], n_pt)
    lo, hi = R.shard_points(pt_ptr, rank, world)
    o0, o1 = int(pt_ptr[lo]), int(pt_ptr[hi])
    P = R.BAProblem(prob["pp"], prob["cam_idx"][o0:o1], prob["pt_idx"][o0:o1] - lo,
                    prob["uv"][o0:o1], n_cam, hi - lo)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    lin = P.linearize(T(prob["cams"]), T(prob["pts"][lo:hi]), 2.0)
    allreduce(lin["U"].view(-1))
    allreduce(lin["gc"].view(-1))
    dc, dp, info = P.ctx.ba_solve_sharded(lin, P.cam_idx, P.pt_idx, P.pt_ptr, P.cam_ptr,
                                          P.cam_obs, lam, allreduce, **dict(dict(max_iter=500,
                                                                                 tol=1e-12), **kw))
    return dc.cpu().numpy(), dp.cpu().numpy(), info.cpu().numpy(), lo, hi


def _reference_solve(prob, lam=1e-3, max_iter=500, tol=1e-12):
    import torch
    P = R.BAProblem(prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], len(prob["cams"]),
                    len(prob["pts"]))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).cuda()
    lin = P.linearize(T(prob["cams"]), T(prob["pts"]), 2.0)
    return tuple(t.cpu().numpy() for t in P.solve(lin, lam, max_iter=max_iter, tol=tol))


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ba_sharded_world1_rccl():
    """World-size-1 `nccl` group: the sharded solve runs its RCCL all-reduces and reproduces the
    unsharded solve; the sharded LM matches the unsharded LM."""
    import torch
    import torch.distributed as dist
    assert not dist.is_initialized()
    prob = problem()
    rdc, rdp, rinfo = _reference_solve(prob)
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    rcams, rpts, rhist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        dc, dp, info, lo, hi = shard_solve(prob, 0, 1, R.make_allreduce())
        assert (lo, hi) == (0, len(prob["pts"]))
        np.testing.assert_array_equal(dc, rdc)
        np.testing.assert_array_equal(dp, rdp)
        assert info[0] == rinfo[0] and info[1] == rinfo[1] and info[4] == rinfo[4]
        np.testing.assert_allclose(info[2:4], rinfo[2:4], rtol=1e-12)
        cams, pts, hist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed, shard=True)
        assert abs(hist[-1][0] - rhist[-1][0]) <= 1e-9 * rhist[-1][0]
        np.testing.assert_allclose(cams, rcams, rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(pts, rpts, rtol=1e-9, atol=1e-12)
    finally:
        R.release_allreduce()
        dist.destroy_process_group()


def test_ba_sharded_world1_graph_and_launch_modes():
    """World-size-1 RCCL group: the CG windows replayed as HIP graphs (poll 8 and 4), launched
    one by one (graph=False; odd poll, where no graph is used), with max_iter ending inside a
    window, the two-launch finish above 1024 cameras and long tracks (more than 64 observations
    per point) all reproduce sfm_ba_solve bit for bit."""
    import torch
    import torch.distributed as dist
    assert not dist.is_initialized()
    prob = problem()
    big = synth.make_ba_problem(1030, 2500, obs_per_pt=3, seed=3, perturb=1e-3)
    counts = np.where(np.arange(120) % 9 == 0, 90, 4)  # long tracks: the point pass's wave path
    mixed = synth.make_ba_problem(140, 120, obs_per_pt=counts, seed=8, perturb=1e-3)
    refs = {(id(p), it): _reference_solve(p, max_iter=it)
            for p in (prob, big, mixed) for it in (500, 21)}
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        ar = R.make_allreduce()
        assert ar.graph_safe
        cases = [(prob, 500, dict(graph=True, poll=8)), (prob, 500, dict(graph=True, poll=4)),
                 (prob, 500, dict(graph=False, poll=8)), (prob, 500, dict(poll=3)),
                 (prob, 21, dict(graph=True, poll=4)), (prob, 21, dict(poll=0)),
                 (big, 500, dict(poll=8)), (big, 21, dict(graph=True, poll=4)),
                 (mixed, 500, dict(poll=8)), (mixed, 21, dict(graph=True, poll=4))]
        for p, it, kw in cases:
            rdc, rdp, rinfo = refs[(id(p), it)]
            dc, dp, info, _, _ = shard_solve(p, 0, 1, ar, max_iter=it, **kw)
            np.testing.assert_array_equal(dc, rdc, err_msg=str((len(p["cams"]), it, kw)))
            np.testing.assert_array_equal(dp, rdp, err_msg=str((len(p["cams"]), it, kw)))
            assert info[0] == rinfo[0] and info[4] == rinfo[4], (info, rinfo, kw)
    finally:
        R.release_allreduce()
        dist.destroy_process_group()


def _run_ranks(tmp_path, n, *extra, env_extra=None):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "ba")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "tests", "dist_ba_worker.py"), out, *extra]
    env = dict(os.environ, OMP_NUM_THREADS="4", **(env_extra or {}))
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return [np.load(f"{out}.rank{k}.npz") for k in range(n)]


def test_ba_sharded_three_ranks_with_an_empty_shard(tmp_path):
    """Three ranks on a 2-point problem: one rank owns no point and no observation, and still
    takes part in every collective; all ranks agree bit for bit and match the single process."""
    prob = tiny_problem()
    pt_ptr, _ = sfmcore.csr_by(prob["pt_idx"], len(prob["pts"]))
    assert min(h - l for l, h in (R.shard_points(pt_ptr, r, 3) for r in range(3))) == 0
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    rcams, rpts, rhist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed)
    rdc, rdp, _ = _reference_solve(prob)
    d = _run_ranks(tmp_path, 3, "tiny")
    for k in (1, 2):
        for key in ("cams", "pts", "hist", "dc", "info"):
            np.testing.assert_array_equal(d[0][key], d[k][key])
    # a 2-point problem is under-determined (the LM damping regularises it), so the tolerances
    # against the single process are looser than the 300-point test's
    np.testing.assert_allclose(d[0]["dc"], rdc, rtol=0, atol=1e-6 * np.abs(rdc).max())
    np.testing.assert_allclose(np.concatenate([d[k]["dp"] for k in range(3)]), rdp, rtol=0,
                               atol=1e-6 * np.abs(rdp).max())
    # the LM itself is sharding-invariant (BA chunks): the single process's result, bit for bit
    np.testing.assert_array_equal(d[0]["hist"], np.array(rhist, np.float64))
    np.testing.assert_array_equal(d[0]["cams"], rcams)
    np.testing.assert_array_equal(d[0]["pts"], rpts)
    assert len(d[2]["dp"]) == 0


def test_ba_sharded_more_ranks_than_chunks(tmp_path):
    """three ranks with SFM_BA_CHUNKS=2 (more ranks than chunks): bundle_adjust raises
    the chunk count to the rank count instead of failing, says so in info, and the ranks agree bit
    for bit and match a single process that uses 3 chunks."""
    prob = problem()
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    d = _run_ranks(tmp_path, 3, env_extra={"SFM_BA_CHUNKS": "2"})
    for k in (1, 2):
        for key in ("cams", "pts", "hist"):
            np.testing.assert_array_equal(d[0][key], d[k][key])
    assert all(int(d[k]["nchunk_adj"]) == 3 for k in range(3))
    old = os.environ.get("SFM_BA_CHUNKS")
    os.environ["SFM_BA_CHUNKS"] = "3"
    try:
        rcams, rpts, rhist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed)
    finally:
        if old is None:
            os.environ.pop("SFM_BA_CHUNKS")
        else:
            os.environ["SFM_BA_CHUNKS"] = old
    np.testing.assert_array_equal(d[0]["hist"], np.array(rhist, np.float64))
    np.testing.assert_array_equal(d[0]["cams"], rcams)
    np.testing.assert_array_equal(d[0]["pts"], rpts)


@pytest.mark.parametrize("schur", ["auto", "1"])
def test_ba_sharded_two_ranks(tmp_path, monkeypatch, schur):
    """Two ranks (torch.distributed.run, gloo, both on GPU 0) shard the points: the ranks agree
    bit for bit, and the sharded solve / LM match the single-process ones to fp64 reassociation.
    schur "1" forces the explicit reduced camera system (sfm_ba_set_schur) in both: the shards'
    T partials are gathered once per solve and the CG runs on every rank without an exchange."""
    monkeypatch.setenv("SFM_BA_SCHUR", schur)
    prob = problem()
    rdc, rdp, rinfo = _reference_solve(prob)
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    rcams, rpts, rhist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed)
    d = _run_ranks(tmp_path, 2)
    for key in ("cams", "pts", "hist", "dc", "info"):
        np.testing.assert_array_equal(d[0][key], d[1][key])
    assert int(d[0]["hi"]) == int(d[1]["lo"]) and 0 < int(d[0]["hi"]) < len(prob["pts"])
    np.testing.assert_allclose(d[0]["dc"], rdc, rtol=0, atol=1e-8 * np.abs(rdc).max())
    dp = np.concatenate([d[k]["dp"] for k in range(2)])
    np.testing.assert_allclose(dp, rdp, rtol=0, atol=1e-8 * np.abs(rdp).max())
    assert d[0]["info"][0] > 0 and d[0]["info"][1] <= 1e-12 and d[0]["info"][4] == 0
    np.testing.assert_allclose(d[0]["info"][2:4], rinfo[2:4], rtol=1e-8)
    # the LM (chunked sums) equals the single process bit for bit
    np.testing.assert_array_equal(d[0]["hist"], np.array(rhist, np.float64))
    np.testing.assert_array_equal(d[0]["cams"], rcams)
    np.testing.assert_array_equal(d[0]["pts"], rpts)
    np.testing.assert_array_equal(d[0]["cams"][fixed], prob["cams"][fixed])


@pytest.mark.parametrize("pcg", ["sharded", "replicated"])
def test_ba_two_ranks_both_pcg_branches_match_oracle(tmp_path, pcg):
    """both PCG branches of the multi-GPU bundle adjustment — 'sharded' (one
    all-reduce per CG iteration) and 'replicated' (W / V / g_p all-gathered once per
    linearisation, every rank runs the whole PCG) — on 2 gloo ranks: the ranks agree bit for
    bit, the branch taken is the one asked for, and the LM end state equals the oracle LM
    (oracle/ba_lm.py) and the single-process GPU LM to fp64 reassociation."""
    import ba_lm as L
    prob = problem()
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    rcams, rpts, rhist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed)
    ocams, opts, ohist = L.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed)
    d = _run_ranks(tmp_path, 2, "std", pcg)
    for key in ("cams", "pts", "hist"):
        np.testing.assert_array_equal(d[0][key], d[1][key])
    assert str(d[0]["pcg"]) == str(d[1]["pcg"]) == pcg
    cost = d[0]["hist"][-1][0]
    assert abs(cost - ohist[-1][0]) <= 1e-9 * ohist[-1][0]
    np.testing.assert_array_equal(d[0]["hist"], np.array(rhist, np.float64))
    np.testing.assert_array_equal(d[0]["cams"], rcams)
    np.testing.assert_array_equal(d[0]["pts"], rpts)
    np.testing.assert_allclose(d[0]["cams"], ocams, rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(d[0]["cams"][fixed], prob["cams"][fixed])


def test_ba_replicated_three_ranks_with_an_empty_shard(tmp_path):
    """The replicated branch with a rank that owns no point: its zero-length W / V / g_p take
    part in the all-gathers; all ranks agree bit for bit and match the single process."""
    prob = tiny_problem()
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    rcams, rpts, rhist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed)
    d = _run_ranks(tmp_path, 3, "tiny", "replicated")
    for k in (1, 2):
        for key in ("cams", "pts", "hist"):
            np.testing.assert_array_equal(d[0][key], d[k][key])
    np.testing.assert_array_equal(d[0]["hist"], np.array(rhist, np.float64))
    np.testing.assert_array_equal(d[0]["cams"], rcams)
    np.testing.assert_array_equal(d[0]["pts"], rpts)


def test_ba_auto_rule_reports_its_branch():
    """World size 1: 'auto' takes the sharded branch (bit-identical to sfm_ba_solve there) and
    says so; the rule itself is covered on the CPU (tests/test_host_cpu.py)."""
    import torch
    import torch.distributed as dist
    assert not dist.is_initialized()
    prob = problem()
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        info = {}
        R.bundle_adjust(*args, loss_s=2.0, max_iter=3, shard=True, info=info)
        assert info["pcg"] == "sharded" and info["world"] == 1
        lat, bw = R.probe_collectives(R.make_allreduce(), len(prob["cams"]), 0)
        assert lat > 0 and bw > 0
    finally:
        R.release_allreduce()
        dist.destroy_process_group()


@pytest.mark.parametrize("schur", ["0", "auto"])
def test_ba_auto_mode_repeated_on_three_ranks(tmp_path, monkeypatch, schur):
    """several sequential auto-mode bundle adjustments on 3 gloo ranks — the
    collective probe's cache key is the same on every rank (backend, group, device, path, n_cam),
    so every rank hits or misses it together and takes the same branch; the ranks agree bit for
    bit and every call gives the same result.  schur "0" keeps the explicit Schur candidate out of
    the branch decision (so the probe runs); "auto" lets its pair count make the explicit system
    the candidate, and since schur_rule then rejects it (random visibility: 6 products per
    (chunk, camera pair) group, fewer than 16) pcg_rule decides the branch after all,
    on every rank alike."""
    monkeypatch.setenv("SFM_BA_SCHUR", schur)
    d = _run_ranks(tmp_path, 3, "std", "auto", "3")
    for k in (1, 2):
        for key in ("cams", "pts", "hist", "branches", "deferred"):
            np.testing.assert_array_equal(d[0][key], d[k][key])
    assert len(set(d[0]["branches"].tolist())) == 1
    assert bool(d[0]["deferred"].all()) == (schur == "auto")
