"""Incremental SfM at 500 x 4096 with the bundle adjustments' PCG tolerance varied (cg_tol, the
relative residual |r| <= cg_tol |b| of the Schur system): wall, BA time, CG iterations and the
reconstruction's quality against the scene's ground truth, per setting, interleaved twice.

Usage: python tests/perf/incremental_cgtol_ab.py [tol ...]   -> one JSON line per run."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "tests")]

import numpy as np
import torch

import incremental
import reconstruction as R
import synth
from test_gpu_incremental import _centres, _umeyama

ORIG = R.bundle_adjust
STATS = []
TOL = [None]


def wrapped(*a, **k):
    if TOL[0] is not None:
        k["cg_tol"] = TOL[0]
    t = time.perf_counter()
    out = ORIG(*a, **k)
    torch.cuda.synchronize()
    h = out[2]
    STATS.append({"n_obs": len(a[3]), "lm_steps": len(h), "cg_total": int(sum(x[3] for x in h)),
                  "accepted": int(sum(1 for x in h if x[2])), "final_cost": float(h[-1][0]),
                  "s": time.perf_counter() - t})
    return out


R.bundle_adjust = wrapped


def run(scene, intr, tol):
    TOL[0] = tol
    STATS.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rec = incremental.reconstruct(scene["desc"], scene["kps"], scene["n_kp"], intr)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tptr, timg, tkp = rec.tracks
    obs_track = np.repeat(np.arange(len(tptr) - 1), np.diff(tptr))
    use = rec.has_point[obs_track] & rec.registered[timg]
    pts_ids, pt_idx = np.unique(obs_track[use], return_inverse=True)
    err = R.reprojection_errors(rec.cams, scene["pp"], rec.points[pts_ids], timg[use],
                                pt_idx.astype(np.int32), scene["kps"][timg[use], tkp[use]])
    reg = rec.registered
    s, Rm, t = _umeyama(_centres(rec.cams[reg]), _centres(scene["cams"][reg]))
    al = (s * (Rm @ _centres(rec.cams[reg]).T)).T + t
    return {"cg_tol": tol, "wall_s": wall, "registered": int(reg.sum()),
            "points": int(rec.has_point.sum()), "observations": int(use.sum()),
            "median_reproj_px": float(np.median(err)), "mean_reproj_px": float(err.mean()),
            "max_centre_err_rel_radius": float(np.abs(al - _centres(scene["cams"][reg])).max() / 8.0),
            "ba": list(STATS), "stage_s": {k: (round(v, 4) if isinstance(v, float) else v)
                                           for k, v in rec.timings.items()}}


def main():
    tols = [float(x) for x in sys.argv[1:]] or [1e-10, 1e-3, 1e-1]
    scene = synth.make_scene(500, 4096, seed=21, k1_range=0.02)
    intr = np.c_[scene["cams"][:, 6:8], scene["pp"]]
    w = np.linspace(0, 499, 4).astype(int)  # warm-up on 4 views
    incremental.reconstruct(scene["desc"][w], scene["kps"][w], scene["n_kp"][w], intr[w])
    for _ in range(2):
        for tol in tols:
            print(json.dumps(run(scene, intr, tol)), flush=True)


if __name__ == "__main__":
    main()
