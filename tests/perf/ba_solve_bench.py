"""Times the bundle-adjustment step solve (K4) and a full LM step at cfg5 scale on one GPU.

Usage: python tests/perf/ba_solve_bench.py [n_cam n_pt obs_per_pt [cg_iters]]
Prints one JSON line: per-CG-iteration time and its HBM roofline (algorithmic bytes: W read once
= 192 B/obs, u_o = W_o t_p written and read = 128 B/obs, indices 8 B/obs, per point V_d⁻¹ 72 B and
pt_ptr 4 B, per camera U_d, M and the CG vectors), setup / back-substitution time, and one LM step
(J^TJ + solve + update + trial cost).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import reconstruction as R
import synth

PEAK_HBM = 8.0e12


def timed(fn, reps):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    a = [int(x) for x in sys.argv[1:]]
    n_cam, n_pt, k = (a + [500, 100_000, 5][len(a):])[:3]
    cg = a[3] if len(a) > 3 else 50
    prob = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=k, seed=0)
    n_obs = len(prob["cam_idx"])
    P = R.BAProblem(prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    lin = P.linearize(cams, pts)
    lam = 1e-3
    # tol = 0: exactly `cg` iterations (the convergence flag never fires)
    t0 = timed(lambda: P.solve(lin, lam, max_iter=0, tol=0.0), 20)
    tn = timed(lambda: P.solve(lin, lam, max_iter=cg, tol=0.0), 10)
    per_it = (tn - t0) / cg
    _, _, info = P.solve(lin, lam, max_iter=500, tol=1e-6)
    it6 = int(info[0].item())
    bytes_it = n_obs * (192 + 128 + 8) + n_pt * (72 + 4) + n_cam * (64 * 8 + 4 * 8 * 8)

    def lm_step():
        ln = P.linearize(cams, pts)
        dc, dp, _ = P.solve(ln, lam, max_iter=it6, tol=1e-6)
        c2, p2 = P.update(cams, dc, pts, dp)
        P.cost(c2, p2)
    t_step = timed(lm_step, 5)

    def lm_step_default(poll):  # what bundle_adjust runs: max_cg = 200, cg_tol = 1e-10
        ln = P.linearize(cams, pts)
        dc, dp, _ = P.solve(ln, lam, max_iter=200, tol=1e-10, poll=poll)
        c2, p2 = P.update(cams, dc, pts, dp)
        P.cost(c2, p2)
    t_def = timed(lambda: lm_step_default(8), 5)
    t_def_async = timed(lambda: lm_step_default(-1), 5)
    _, _, info = P.solve(lin, lam, max_iter=200, tol=1e-10)
    it10 = int(info[0].item())
    t_jtj = timed(lambda: P.linearize(cams, pts), 10)
    # the sharding-invariant form bundle_adjust runs (BA_CHUNKS chunks, reconstruction.BAChunks)
    Pc = R.BAProblem(prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt,
                     chunks=R.BA_CHUNKS)
    linc = Pc.linearize(cams, pts)
    c0 = timed(lambda: Pc.solve(linc, lam, max_iter=0, tol=0.0), 20)
    cn = timed(lambda: Pc.solve(linc, lam, max_iter=cg, tol=0.0), 10)
    t_jtj_c = timed(lambda: Pc.linearize(cams, pts), 10)
    t_cost = timed(lambda: P.cost(cams, pts), 20)
    t_cost_c = timed(lambda: Pc.cost(cams, pts), 20)
    out = {
        "stage": "K4 BA step (Schur-complement PCG)", "n_cam": n_cam, "n_pt": n_pt, "n_obs": n_obs,
        "cg_iter_ms": per_it, "setup_backsub_ms": t0,
        "roofline": {"bound": "hbm", "bytes_per_iter": bytes_it,
                     "achieved_GBs": bytes_it / (per_it * 1e-3) / 1e9, "peak_GBs": PEAK_HBM / 1e9,
                     "frac": bytes_it / (per_it * 1e-3) / PEAK_HBM},
        "cg_iters_to_1e-6": it6, "lm_step_ms": t_step, "jtj_ms": t_jtj,
        "chunked": {"chunks": R.BA_CHUNKS, "cg_iter_ms": (cn - c0) / cg, "setup_backsub_ms": c0,
                    "jtj_ms": t_jtj_c, "cost_ms": t_cost_c, "cost_ms_unchunked": t_cost},
        "default_lm_step": {"max_cg": 200, "cg_tol": 1e-10, "cg_iters": it10,
                            "ms_poll_every_8": t_def, "ms_no_poll_all_launches": t_def_async},
    }
    # the sharded solve (sfm_ba_solve_stage) in a world-size-1 RCCL group: the cost of its
    # split camera passes and of one all-reduce per CG iteration (at N ranks each rank's point
    # pass shrinks to 1/N; the camera-side all-reduce of 8 n_cam doubles stays)
    import socket
    import torch.distributed as dist
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ar = R.make_allreduce()
    shs = lambda it: P.ctx.ba_solve_sharded(lin, P.cam_idx, P.pt_idx, P.pt_ptr, P.cam_ptr,
                                            P.cam_obs, lam, ar, max_iter=it, tol=0.0)
    s0 = timed(lambda: shs(0), 10)
    sn = timed(lambda: shs(cg), 5)
    sh_it = (sn - s0) / cg
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    import time
    tw = time.perf_counter()
    _, _, h1 = R.bundle_adjust(*args, max_iter=5, fixed=fixed)
    t_un = time.perf_counter() - tw
    tw = time.perf_counter()
    _, _, h2 = R.bundle_adjust(*args, max_iter=5, fixed=fixed, shard=True)
    t_sh = time.perf_counter() - tw
    R.release_allreduce()
    dist.destroy_process_group()
    out["sharded_world1_rccl"] = {
        "cg_iter_ms": sh_it, "setup_backsub_ms": s0, "cg_iter_overhead_ms": sh_it - per_it,
        "bundle_adjust_5_steps_s": {"unsharded": t_un, "sharded": t_sh},
        "final_cost_rel_diff": abs(h1[-1][0] - h2[-1][0]) / h1[-1][0]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
