"""Host-side set-up cost of one bundle adjustment (reconstruction.bundle_adjust's problem phase:
BAProblem with its chunk table + the explicit Schur structure), small and full cfg5-like sizes:
wall time per piece and a torch.profiler table of the full phase.
python tests/perf/ba_problem_time.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import reconstruction as R


def problem(n_cam, n_pt, seed=0):
    rng = np.random.default_rng(seed)
    m = rng.integers(3, 10, n_pt)
    w = min(4, (n_cam - 1) // 2)
    cam = np.concatenate([np.sort((p % n_cam + rng.choice(np.arange(-w, w + 1), size=min(k, 2 * w + 1),
                                                          replace=False)) % n_cam)
                          for p, k in zip(range(n_pt), m)]).astype(np.int32)
    pt = np.repeat(np.arange(n_pt, dtype=np.int32), np.minimum(m, 2 * w + 1))
    return cam, pt


def main():
    dev = torch.device("cuda", 0)
    for n_cam, n_pt in ((9, 5000), (100, 50000), (500, 258000)):
        cam, pt = problem(n_cam, n_pt)
        cam_d, pt_d = torch.from_numpy(cam).to(dev), torch.from_numpy(pt).to(dev)
        uv_d = torch.zeros((len(cam), 2), dtype=torch.float64, device=dev)
        pp = np.zeros((n_cam, 2))
        res = {}
        for rep in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            P = R.BAProblem(pp, cam_d, pt_d, uv_d, n_cam, n_pt, chunks=8)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            P.set_schur()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if rep:
                res.setdefault("problem_ms", []).append((t1 - t0) * 1e3)
                res.setdefault("set_schur_ms", []).append((t2 - t1) * 1e3)
        print({"n_cam": n_cam, "n_pt": n_pt, "n_obs": len(cam),
               **{k: round(float(np.median(v)), 3) for k, v in res.items()}}, flush=True)
    from torch.profiler import profile, ProfilerActivity
    cam, pt = problem(100, 50000)
    cam_d, pt_d = torch.from_numpy(cam).to(dev), torch.from_numpy(pt).to(dev)
    uv_d = torch.zeros((len(cam), 2), dtype=torch.float64, device=dev)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(3):
            P = R.BAProblem(np.zeros((100, 2)), cam_d, pt_d, uv_d, 100, 50000, chunks=8)
            P.set_schur()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=30))


if __name__ == "__main__":
    main()
