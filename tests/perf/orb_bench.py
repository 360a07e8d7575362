"""ORB extraction throughput (sfm_orb_batch) on a batch of synthetic 1920x1080 images (the
reference reads photos, code/pipeline.py:25, and extracts ORB per pair, code/pipeline.py:38-41 ->
code/feature_matching.py:42-45).  Reports images/s on the GPU (HIP events, inputs resident),
the oracle (scalar C restatement, one core) on one image, and a parity check of 2 images.
Usage: python tests/perf/orb_bench.py [n_img [H W]]"""
import json
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
    a = [int(x) for x in sys.argv[1:]]
    n = a[0] if a else 64
    H, W = (a[1], a[2]) if len(a) >= 3 else (1080, 1920)
    base = [synth.make_image(H, W, seed=s) for s in range(8)]
    imgs = np.stack([base[i % 8] for i in range(n)])
    ctx = sfmcore.context(0)
    t = torch.from_numpy(np.ascontiguousarray(imgs)).cuda()
    out = ctx.orb_batch(t)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 10
    ev[0].record()
    for _ in range(reps):
        out = ctx.orb_batch(t, out=out)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    kp, desc, cnt = (x.cpu().numpy() for x in out)
    parity = True
    for i in range(2):
        okp, odesc, _ = O.orb(imgs[i])
        parity &= bool(cnt[i] == len(okp) and (desc[i, :cnt[i]] == odesc).all()
                       and (kp[i, :cnt[i], :3] == okp[:, :3]).all())
    O.set_threads(1)
    t0 = time.perf_counter()
    O.orb(imgs[0])
    cpu_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"stage": "ORB extraction (sfm_orb_batch)", "images": n, "H": H, "W": W,
                      "batch_ms": ms, "images_per_s": n / (ms * 1e-3),
                      "us_per_image": ms * 1e3 / n, "keypoints_mean": float(cnt.mean()),
                      "cpu_oracle_ms_per_image_1core": cpu_ms, "parity_2_images": parity}))


if __name__ == "__main__":
    main()
