"""K1 / K2 overlap on the cfg4 scene (500 x 4096, all 124 750 pairs, the bench's match + verify
parameters): the pairs in chunks, either in series on one stream (K1 c, K2 c, K1 c+1 ...), or
pipelined — K1 of every chunk on stream A with one context, K2 of chunk c on stream B with a second
context (its own workspace) after K1 c's event, so K2 c runs beside K1 c+1 on the same CUs (K1 is
VALU + MFMA with ~28 % of its cycles waiting, K2 VALU only).  Reports ms per pass and checks the
verified counts identical.  python tests/perf/k1k2_overlap.py [chunk ...] (default 31250 62500; N_HYP, N_IMG, K override)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import sfmcore
import synth


def main():
    chunks = [int(x) for x in sys.argv[1:]] or [31250, 62500]
    n_img, K = int(os.environ.get("N_IMG", "500")), int(os.environ.get("K", "4096"))
    s = synth.make_scene(n_img, K, seed=0)
    pairs = synth.unordered_pairs(n_img)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    desc, n_kp, kps = T(s["desc"]), T(s["n_kp"]), T(s["kps"].astype(np.float32))
    ctx_a = sfmcore.context(0)
    ctx_b = sfmcore.Context(0)   # a second context: its own workspace for K2
    mkw = dict(cross_check=sfmcore.XC_MUTUAL, ratio=(4, 5))
    rkw = dict(n_hyp=int(os.environ.get("N_HYP", "4096")), seed=42, thr=1.0, min_inliers=15)
    P = len(pairs)

    def buffers(n):
        return ((torch.empty(n, dtype=torch.int32, device=dev),
                 torch.empty((n, K, 2), dtype=torch.int32, device=dev),
                 torch.empty((n, K), dtype=torch.int32, device=dev)),
                dict(inl_count=torch.empty(n, dtype=torch.int32, device=dev),
                     best_h=torch.empty(n, dtype=torch.int32, device=dev),
                     mask=torch.empty((n, K), dtype=torch.uint8, device=dev),
                     F=torch.empty((n, 9), dtype=torch.float32, device=dev),
                     norm=torch.empty((n, 6), dtype=torch.float32, device=dev)))

    out = {}
    for chunk in [P] + chunks:
        cuts = list(range(0, P, chunk)) + [P]
        parts = [T(pairs[a:b]) for a, b in zip(cuts, cuts[1:])]
        bufs = [buffers(len(p)) for p in parts]
        sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

        def serial():
            for pt, (mb, rb) in zip(parts, bufs):
                c, m, _ = ctx_a.match_batch(desc, n_kp, pt, out=mb, **mkw)
                ctx_a.ransac_batch(kps, pt, c, m, out=rb, **rkw)

        def piped():
            evs = []
            with torch.cuda.stream(sa):
                for pt, (mb, rb) in zip(parts, bufs):
                    ctx_a.match_batch(desc, n_kp, pt, out=mb, **mkw)
                    e = torch.cuda.Event()
                    e.record(sa)
                    evs.append(e)
            with torch.cuda.stream(sb):
                for pt, (mb, rb), e in zip(parts, bufs, evs):
                    sb.wait_event(e)
                    ctx_b.ransac_batch(kps, pt, mb[0], mb[1], out=rb, **rkw)
            torch.cuda.current_stream(dev).wait_stream(sa)
            torch.cuda.current_stream(dev).wait_stream(sb)

        res = {}
        for name, fn in (("serial", serial), ("piped", piped)):
            if name == "piped" and len(parts) == 1:
                continue
            fn()
            torch.cuda.synchronize()
            ms = []
            for _ in range(3):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - t0) * 1e3)
            verified = int(sum(int((rb["inl_count"] >= 15).sum()) for _, rb in bufs))
            inl = int(sum(int(rb["inl_count"].clamp(min=0).sum()) for _, rb in bufs))
            res[name] = {"ms": ms, "verified_pairs": verified, "inliers": inl}
        out[str(chunk)] = res
        print(json.dumps({"chunk": chunk, **res}), flush=True)


if __name__ == "__main__":
    main()
