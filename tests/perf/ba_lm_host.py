"""Where an LM step's time goes at cfg5's BA sizes: the host's enqueue time of each call of the
step (linearise, solve, update, trial cost — perf_counter over back-to-back calls with no sync,
so the GPU queue absorbs them) against the GPU time of the same calls (HIP events), and
bundle_adjust's own lm_s per step.  A call whose host time exceeds its GPU time starves the GPU
between the step's one host sync and the next.
python tests/perf/ba_lm_host.py [n_cam ...]   (defaults 24 100 250 500; ~520 points per camera,
4 observations per point as in cfg5's final model)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import reconstruction as R
import synth


def host_gpu(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    host = (time.perf_counter() - t0) / reps
    torch.cuda.synchronize()
    return {"host_us": host * 1e6, "gpu_us": e0.elapsed_time(e1) / reps * 1e3}


def local_problem(n_cam, n_pt, seed=0, sorted_pts=False):
    """make_ba_problem's cameras, but each point seen by 4 cameras adjacent on a ring (cfg5's
    views see their grid neighbours, so the reduced camera system stays sparse)."""
    base = synth.make_ba_problem(n_cam, 8, obs_per_pt=4, seed=seed)
    rng = np.random.default_rng(seed)
    cams_true, pp = base["cams"], base["pp"]
    pts_true = rng.uniform(-2.0, 2.0, size=(n_pt, 3))
    b = rng.integers(0, n_cam, n_pt)
    if sorted_pts:   # points in the order of their first camera (tracks in image order)
        b = np.sort(b)
    cam_idx = np.sort((b[:, None] + np.arange(4)[None, :]) % n_cam, 1).reshape(-1).astype(np.int32)
    pt_idx = np.repeat(np.arange(n_pt, dtype=np.int32), 4)
    uv = np.empty((cam_idx.size, 2))
    for c in range(n_cam):
        sel = np.nonzero(cam_idx == c)[0]
        Rm = synth.angle_axis_to_rotmat(cams_true[c, :3])
        uv[sel], _ = synth.project(Rm, cams_true[c, 3:6], cams_true[c, 6], cams_true[c, 7],
                                   pp[c, 0], pp[c, 1], pts_true[pt_idx[sel]])
    uv += rng.normal(0.0, 0.5, size=uv.shape)
    pts = pts_true + rng.normal(0.0, 1e-2, size=pts_true.shape)
    return dict(cams=base["cams"], pp=pp, pts=pts, cam_idx=cam_idx, pt_idx=pt_idx, uv=uv)


def one(n_cam):
    n_pt = 516 * n_cam
    prob = local_problem(n_cam, n_pt)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    P = R.BAProblem(prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt,
                    chunks=R.ba_chunk_count())
    P.set_schur()
    lin = P.linearize(cams, pts)
    dc, dp, sinfo = P.solve(lin, 1e-4, 200, 1e-10)
    c2, p2 = P.update(cams, dc, pts, dp)
    out = {"n_cam": n_cam, "n_pt": n_pt, "n_obs": len(prob["cam_idx"]), "n_slot": P.schur.n_slot,
           "linearize": host_gpu(lambda: P.linearize(cams, pts)),
           "solve": host_gpu(lambda: P.solve(lin, 1e-4, 200, 1e-10)),
           "update": host_gpu(lambda: P.update(cams, dc, pts, dp)),
           "cost": host_gpu(lambda: P.cost(c2, p2)),
           "sync": host_gpu(lambda: torch.cat([sinfo, P.cost(c2, p2)]).cpu().numpy())}
    info = {}
    noisy = prob["cams"].copy()
    noisy[:, :6] += np.random.default_rng(1).normal(0, 1e-3, noisy[:, :6].shape)
    fixed = R.gauge_mask(noisy)
    for _ in range(2):
        info = {}
        _, _, hist = R.bundle_adjust(noisy, prob["pp"], prob["pts"], prob["cam_idx"],
                                     prob["pt_idx"], prob["uv"], max_iter=10, fixed=fixed,
                                     info=info)
    out["ba"] = {k: info.get(k) for k in ("lm_s", "setup_s", "problem_s", "schur")}
    out["ba"]["steps"] = len(hist)
    out["ba"]["cg_iters"] = int(sum(h[3] for h in hist))
    out["ba"]["lm_us_per_step"] = info["lm_s"] / max(len(hist), 1) * 1e6
    return out


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [24, 100, 250, 500]
    for n in sizes:
        print(json.dumps(one(n)), flush=True)


if __name__ == "__main__":
    main()
