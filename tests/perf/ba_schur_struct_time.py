"""Host-side cost of the explicit Schur structure (BAProblem.set_schur) on a problem with local
visibility (cfg5-like: point p seen by 3-9 of the cameras within +-4 of camera p mod n_cam):
wall time and a torch.profiler table of the ops.  python tests/perf/ba_schur_struct_time.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import reconstruction as R


def main():
    rng = np.random.default_rng(0)
    n_cam, n_pt = 500, 258000
    m = rng.integers(3, 10, n_pt)
    cam = np.concatenate([np.sort((p % n_cam + rng.choice(np.arange(-4, 5), size=k, replace=False))
                                  % n_cam) for p, k in zip(range(n_pt), m)]).astype(np.int32)
    pt = np.repeat(np.arange(n_pt, dtype=np.int32), m)
    uv = np.zeros((len(cam), 2))
    P = R.BAProblem(np.zeros((n_cam, 2)), cam, pt, uv, n_cam, n_pt, chunks=8)
    P.set_schur()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        P.set_schur()
    torch.cuda.synchronize()
    print({"n_obs": len(cam), "n_inst": P.schur.n_inst, "n_slot": P.schur.n_slot,
           "n_seg": P.schur.n_seg, "set_schur_ms": (time.perf_counter() - t) / 10 * 1e3})
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(3):
            P.set_schur()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25))


if __name__ == "__main__":
    main()
