"""Times the K2 RANSAC schedules (SFM_RANSAC_MODE 0 ordered, 1 single-pass pruned, 2 unpruned;
MODES=0,1 selects) on
the cfg3 workload and checks each against the CPU oracle on a sample of pairs.
Usage: python tests/perf/ransac_variants.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]

import numpy as np
import torch

import oracle as O
import sfmcore
import synth


def main():
    n_img = int(os.environ.get("N_IMG", "50"))
    s = synth.make_scene(n_img, 2048, seed=0)
    pairs = synth.unordered_pairs(n_img)
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, kps, pr = T(s["desc"]), T(s["n_kp"]), T(s["kps"]), T(pairs)
    cnt, mt, _ = ctx.match_batch(desc, n_kp, pr, ratio=(4, 5))
    torch.cuda.synchronize()
    cnt_np, mt_np = cnt.cpu().numpy(), mt.cpu().numpy()
    sample = np.arange(0, len(pairs), max(1, len(pairs) // 16))
    ref = {}
    for p in sample:
        a, b = pairs[p]
        M = cnt_np[p]
        ref[p] = O.ransac_f(s["kps"][a][mt_np[p, :M, 0]], s["kps"][b][mt_np[p, :M, 1]], H=4096,
                            seed=42, pa=int(a), pb=int(b))
    for v in [int(x) for x in os.environ.get("MODES", "0,1,2").split(",")]:
        os.environ["SFM_RANSAC_MODE"] = str(v)
        for _ in range(2):
            out = ctx.ransac_batch(kps, pr, cnt, mt, n_hyp=4096)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        reps = 10
        for _ in range(reps):
            out = ctx.ransac_batch(kps, pr, cnt, mt, n_hyp=4096)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        ic = out["inl_count"].cpu().numpy()
        bh = out["best_h"].cpu().numpy()
        mask = out["mask"].cpu().numpy()
        ok = all(ic[p] == ref[p]["count"] and bh[p] == ref[p]["best_h"]
                 and (mask[p, :cnt_np[p]] == ref[p]["mask"]).all() for p in sample)
        print(f"mode={v}: {ms:.3f} ms/launch  parity({len(sample)} pairs)={ok}  "
              f"sum_inl={int(np.maximum(ic, 0).sum())}", flush=True)


if __name__ == "__main__":
    main()
