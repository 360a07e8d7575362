"""Times the forward MFMA scan of the ratio-test L2 path alone (SFM_L2FR_DEBUG=1 stops the launch
after prep + order + scan + a record dump) on the cfg3 workload (N_IMG, K override).  Usage (variants via SFMCORE_LIB):
python tests/perf/l2fr_scan_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]

import numpy as np
import torch

import sfmcore
import synth


def main():
    n_img, K = int(os.environ.get("N_IMG", "50")), int(os.environ.get("K", "2048"))
    s = synth.make_scene(n_img, K, seed=0)
    pairs = synth.unordered_pairs(n_img)
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, pr = T(s["desc"]), T(s["n_kp"]), T(pairs)
    os.environ["SFM_L2FR_DEBUG"] = "1"
    out = ctx.match_batch(desc, n_kp, pr, cross_check=0, ratio=(4, 5))
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 20
    ev[0].record()
    for _ in range(reps):
        out = ctx.match_batch(desc, n_kp, pr, cross_check=0, ratio=(4, 5), out=out)
    ev[1].record()
    torch.cuda.synchronize()
    lib = os.path.basename(os.environ.get("SFMCORE_LIB", "base"))
    print(f"{lib}: scan-only launch {ev[0].elapsed_time(ev[1]) / reps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
