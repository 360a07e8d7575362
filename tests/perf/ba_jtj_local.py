"""K3 (sfm_ba_jtj) plain vs chunk mode on a cfg5-like LOCAL-visibility problem: each point seen by
4 cameras adjacent on a ring, points ordered by their first camera (as the incremental driver's
tracks come out in image order), so a camera's observations fall in one or two of the 8 chunks —
unlike synth.make_ba_problem's random visibility, where every camera touches every chunk.
HIP graph replays timed with events (the kernels' GPU time).  SFMCORE_LIB / SFM_BA_CKW: variants.
python tests/perf/ba_jtj_local.py [n_cam] [order: sorted|random]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "tests", "perf")]

import numpy as np
import torch

import reconstruction as R
from ba_lm_host import local_problem


def graph_ms(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n_cam = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    order = sys.argv[2] if len(sys.argv) > 2 else "sorted"
    n_pt = 516 * n_cam
    prob = local_problem(n_cam, n_pt, sorted_pts=(order == "sorted"))
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    args = (prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt)
    P = R.BAProblem(*args)
    Pc = R.BAProblem(*args, chunks=R.ba_chunk_count())
    out = {"n_cam": n_cam, "n_obs": len(prob["cam_idx"]), "order": order,
           "ckw": os.environ.get("SFM_BA_CKW", "default"),
           "lib": os.path.basename(os.environ.get("SFMCORE_LIB", "libsfmcore.so"))}
    for _ in range(2):
        out["plain_ms"] = graph_ms(lambda: P.linearize(cams, pts))
        with Pc.bind():
            out["chunked_ms"] = graph_ms(lambda: Pc.linearize(cams, pts))
    l0 = P.linearize(cams, pts)
    l1 = Pc.linearize(cams, pts)
    out["rel_U"] = float((l0["U"] - l1["U"]).abs().max() / l0["U"].abs().max())
    ck = Pc.chunks
    cb = ck.cam_bounds.reshape(n_cam, -1).cpu().numpy()
    seg = np.diff(cb, axis=1)
    out["cam_chunks_nonempty_mean"] = float((seg > 0).sum(1).mean())
    out["cam_max_seg"] = int(seg.max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
