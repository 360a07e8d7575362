"""The explicit reduced camera system at one BA size: structure build (SchurSpec, once per bundle
adjustment), per-solve build of T (bas_schur_build + tree), per-CG-iteration cost, against the
implicit chunked solve.  Usage: python tests/perf/ba_schur_time.py [n_cam n_pt obs_per_pt]
(obs_per_pt 0: the cfg5-like grid scene's track lengths, 3 .. 9, mean ~5)."""
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


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def wall(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    a = [int(x) for x in sys.argv[1:]]
    n_cam, n_pt, k = (a + [500, 258000, 0][len(a):])[:3]
    counts = k if k > 0 else np.random.default_rng(1).integers(3, 10, n_pt)
    prob = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=counts, seed=0)
    args = (prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    Pi = R.BAProblem(*args, chunks=R.BA_CHUNKS)
    Pe = R.BAProblem(*args, chunks=R.BA_CHUNKS)
    t_struct = wall(lambda: Pe.set_schur(), 5)
    sp = Pe.schur
    out = {"n_cam": n_cam, "n_pt": n_pt, "n_obs": len(prob["cam_idx"]), "n_inst": sp.n_inst,
           "n_slot": sp.n_slot, "n_seg": sp.n_seg, "inst_per_obs": sp.n_inst / len(prob["cam_idx"]),
           "structure_ms": t_struct}
    lam, cg = 1e-3, 32
    for name, P in (("implicit", Pi), ("explicit", Pe)):
        lin = P.linearize(cams, pts)
        s0 = timed(lambda: P.solve(lin, lam, max_iter=0, tol=0.0), 20)
        sn = timed(lambda: P.solve(lin, lam, max_iter=cg, tol=0.0, poll=-1), 5)
        _, _, info = P.solve(lin, lam, max_iter=200, tol=0.1)
        out[name] = {"setup_backsub_ms": s0, "cg_iter_ms": (sn - s0) / cg,
                     "cg_iters_tol_0.1": int(info[0].item()),
                     "solve_tol_0.1_ms": timed(lambda: P.solve(lin, lam, max_iter=200, tol=0.1), 5)}
    # T's algorithmic bytes per solve: per instance W_a half rows + W_b + V_d⁻¹ per wave pair
    out["explicit"]["schur_build_bytes"] = sp.n_inst * (192 + 192 + 72)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
