"""Times K3 (sfm_ba_jtj) and the trial cost, unchunked and in chunk mode, at one BA size.

Usage: python tests/perf/ba_jtj_time.py [n_cam n_pt obs_per_pt]   (SFM_BA_CKW: camera waves per
camera in chunk mode; BA_JTJ_ONLY=plain|chunked times one form only, for PMC passes).  Prints one JSON line; the chunked U / g_c / V / cost are checked equal to
the unchunked ones within 1e-9 relative (the sums associate differently)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import reconstruction as R
import synth


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    a = [int(x) for x in sys.argv[1:]]
    n_cam, n_pt, k = (a + [500, 258000, 4][len(a):])[:3]
    prob = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=k, seed=0)
    args = (prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt)
    P = R.BAProblem(*args)
    Pc = R.BAProblem(*args, chunks=R.BA_CHUNKS)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    cams, pts = T(prob["cams"]), T(prob["pts"])
    only = os.environ.get("BA_JTJ_ONLY")   # "plain" / "chunked": one form only (PMC passes)
    if only:
        Q = P if only == "plain" else Pc
        print(json.dumps({"only": only, "jtj_ms": timed(lambda: Q.linearize(cams, pts), 20)}))
        return
    out = {"n_cam": n_cam, "n_pt": n_pt, "n_obs": len(prob["cam_idx"]),
           "ckw": os.environ.get("SFM_BA_CKW", "default"),
           "jtj_ms": timed(lambda: P.linearize(cams, pts), 20),
           "jtj_chunked_ms": timed(lambda: Pc.linearize(cams, pts), 20),
           "cost_ms": timed(lambda: P.cost(cams, pts), 20),
           "cost_chunked_ms": timed(lambda: Pc.cost(cams, pts), 20)}
    l0, l1 = P.linearize(cams, pts), Pc.linearize(cams, pts)
    for key in ("U", "gc", "V", "gp", "cost"):
        x, y = l0[key].cpu().numpy(), l1[key].cpu().numpy()
        out[f"rel_{key}"] = float(np.abs(x - y).max() / max(np.abs(x).max(), 1e-300))
    out["cost_fn_vs_lin_chunked"] = float(abs(Pc.cost(cams, pts).item() - l1["cost"][0].item()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
