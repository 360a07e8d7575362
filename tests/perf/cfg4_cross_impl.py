"""Full-size cross-implementation agreement at cfg4 (500 images x 4096 SIFT-like descriptors, all
124 750 pairs — the bench's scene, seed 0): size-independent evidence that the shipped path is
exact where the CPU oracle is too slow to check every pair.

K1, L2 mutual cross check + ratio 4/5, by three independent GPU implementations of the same rule
(SFM_L2_PATH): the mutual kernel (value-only rows + column winners, the default), the forward /
reverse ratio path (match_l2fr.hip) and the fused packed-key kernel — counts, match indices and
squared distances compared bit for bit.  K2 on the default K1 output under the three schedules
(SFM_RANSAC_MODE 0 ordered + pruned, 1 single pass pruned, 2 unpruned): inlier counts, winners,
F, normalisation and inlier masks compared bit for bit (exact pruning must change nothing).  The
verified graph's checksum is the bench's (bench.graph_checksum; 793920861 for this scene).
Usage: python tests/perf/cfg4_cross_impl.py [n_img [k]]  -> one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), ROOT]

import numpy as np
import torch

import bench
import sfmcore
import synth


def main():
    a = [int(x) for x in sys.argv[1:]]
    n_img, k = (a + [500, 4096][len(a):])[:2]
    t0 = time.time()
    s = synth.make_scene(n_img, k, seed=0)
    pairs = synth.unordered_pairs(n_img)
    P = len(pairs)
    dev = torch.device("cuda", 0)
    ctx = sfmcore.context(0)
    desc = torch.from_numpy(s["desc"]).to(dev)
    n_kp = torch.from_numpy(s["n_kp"]).to(dev)
    kps = torch.from_numpy(np.ascontiguousarray(s["kps"], np.float32)).to(dev)
    pt = torch.from_numpy(pairs).to(dev)
    ar = torch.arange(k, device=dev)[None, :]
    out = {"n_img": n_img, "k": k, "pairs": P}

    def k1(path):
        os.environ["SFM_L2_PATH"] = path
        try:
            t = time.time()
            r = ctx.match_batch(desc, n_kp, pt, metric=sfmcore.METRIC_L2,
                                cross_check=sfmcore.XC_MUTUAL, ratio=(4, 5))
            torch.cuda.synchronize()
            return r, time.time() - t
        finally:
            os.environ.pop("SFM_L2_PATH", None)

    (c0, m0, d0), _ = k1("mutual")
    valid = ar < c0[:, None]
    out["k1_matches"] = int(c0.sum())
    for path in ("fr", "fused"):
        (c, m, d), dt = k1(path)
        same = bool(torch.equal(c, c0))
        if same:
            same = bool(torch.equal(m[valid], m0[valid]) and torch.equal(d[valid], d0[valid]))
        out[f"k1_{path}_identical"] = same
        out[f"k1_{path}_s"] = round(dt, 3)
        del c, m, d
    ref = None
    for mode in ("0", "1", "2"):
        os.environ["SFM_RANSAC_MODE"] = mode
        try:
            t = time.time()
            rs = ctx.ransac_batch(kps, pt, c0, m0, n_hyp=4096, seed=42, thr=1.0, min_inliers=15)
            torch.cuda.synchronize()
            dt = time.time() - t
        finally:
            os.environ.pop("SFM_RANSAC_MODE", None)
        rs = {key: v.clone() for key, v in rs.items()}
        if ref is None:
            ref = rs
            rows = ctx.graph_rows(0, c0, m0, rs["inl_count"], rs["mask"], 15)
            out["verified_rows"] = int(rows.shape[0])
            out["graph_checksum"] = bench.graph_checksum(torch, rows)
        else:
            same = all(torch.equal(rs[key], ref[key]) for key in ("inl_count", "best_h", "F", "norm"))
            same = same and bool(torch.equal(rs["mask"][valid], ref["mask"][valid]))
            out[f"k2_mode{mode}_identical"] = same
        out[f"k2_mode{mode}_s"] = round(dt, 3)
    out["wall_s"] = round(time.time() - t0, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
