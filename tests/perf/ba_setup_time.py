"""Times the BAProblem set-up (device tensors in, cfg5 final-model size) without and with the
sharding-invariant chunk table, and its pieces (shard_cuts_device, cam_bounds_device).
Usage: python tests/perf/ba_setup_time.py [n_cam n_pt obs_per_pt]"""
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


def wall(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    a = [int(x) for x in sys.argv[1:]]
    n_cam, n_pt, k = (a + [500, 258000, 4][len(a):])[:3]
    prob = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=k, seed=0)
    d = torch.device("cuda", 0)
    cam = torch.from_numpy(prob["cam_idx"].astype(np.int32)).to(d)
    pt = torch.from_numpy(prob["pt_idx"].astype(np.int32)).to(d)
    uv = torch.from_numpy(prob["uv"]).to(d)
    pp = prob["pp"]
    P = R.BAProblem(pp, cam, pt, uv, n_cam, n_pt)
    out = {"n_obs": int(cam.numel()),
           "problem_ms": wall(lambda: R.BAProblem(pp, cam, pt, uv, n_cam, n_pt)),
           "problem_chunked_ms": wall(lambda: R.BAProblem(pp, cam, pt, uv, n_cam, n_pt, chunks=8)),
           "shard_cuts_ms": wall(lambda: R.shard_cuts_device(P.pt_idx, n_pt, 8)),
           "cam_bounds_ms": wall(lambda: R.cam_bounds_device(P.cam_idx, P.cam_obs, n_cam,
                                                              R.shard_cuts_device(P.pt_idx, n_pt, 8)[1]))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
