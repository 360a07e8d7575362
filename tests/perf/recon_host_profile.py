"""Host-side profile of one cfg5 reconstruction (bench.py's scene, N = 1): cProfile of
incremental.reconstruct after the bench's 4-view warm-up, top functions by own time and by
cumulative time.  python tests/perf/recon_host_profile.py [n_img [k]]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import bench
import incremental


def main():
    a = [int(x) for x in sys.argv[1:]]
    n_img, k = (a + [500, 4096][len(a):])[:2]
    scene, grid = bench.local_scene(n_img, k)
    intr = np.c_[scene["cams"][:, 6:8], scene["pp"]]
    w = np.array(sorted({0, 1, grid[1], grid[1] + 1} & set(range(n_img))))
    incremental.reconstruct(scene["desc"][w], scene["kps"][w], scene["n_kp"][w], intr[w])
    torch.cuda.synchronize()
    t = time.perf_counter()
    incremental.reconstruct(scene["desc"], scene["kps"], scene["n_kp"], intr)
    torch.cuda.synchronize()
    print("wall without profiler", round(time.perf_counter() - t, 4), flush=True)
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    rec = incremental.reconstruct(scene["desc"], scene["kps"], scene["n_kp"], intr)
    torch.cuda.synchronize()
    pr.disable()
    print("wall under cProfile", round(time.perf_counter() - t, 4), rec.timings, flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
