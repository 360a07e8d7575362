"""K3 (BA J^TJ build) at BASELINE cfg5 scale: 500 cameras, 100k points, 5 observations/point.

Inputs resident on the device; times sfm_ba_jtj with HIP events on torch's stream, reports the
achieved algorithmic HBM bandwidth against the 8 TB/s peak, and checks U/V/W/g/residuals against
the CPU oracle (fp64; U, g_c are reassociated sums: rel 1e-9; residuals 1e-4 px per north_star).
Usage: python tests/perf/ba_bench.py [n_cam n_pt obs_per_pt]"""
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

PEAK_HBM = 8.0e12


def main():
    n_cam, n_pt, k = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (500, 100000, 5)))
    t0 = time.time()
    pr = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=k, seed=5)
    n_obs = len(pr["pt_idx"])
    pt_ptr, _ = sfmcore.csr_by(pr["pt_idx"], n_pt)
    cam_ptr, cam_obs = sfmcore.csr_by(pr["cam_idx"], n_cam)
    print(f"problem {n_cam} cams, {n_pt} pts, {n_obs} obs (gen {time.time() - t0:.1f}s)",
          file=sys.stderr)
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    args = [T(pr["cams"]), T(pr["pp"]), T(pr["pts"]), T(pr["cam_idx"]), T(pr["pt_idx"]),
            T(pr["uv"]), T(pt_ptr), T(cam_ptr), T(cam_obs)]
    out = ctx.ba_jtj(*args, loss_s=2.0)
    torch.cuda.synchronize()
    reps = 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        out = ctx.ba_jtj(*args, loss_s=2.0)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    # algorithmic bytes: every input read once, every output written once
    rd = (pr["cams"].nbytes + pr["pp"].nbytes + pr["pts"].nbytes + pr["cam_idx"].nbytes
          + pr["pt_idx"].nbytes + pr["uv"].nbytes + pt_ptr.nbytes + cam_ptr.nbytes
          + cam_obs.nbytes)
    wr = 8 * (64 * n_cam + 9 * n_pt + 24 * n_obs + 8 * n_cam + 3 * n_pt + 2 * n_obs + 1)
    bw = (rd + wr) / (ms * 1e-3)
    o = O.ba_jtj(pr["cams"], pr["pp"], pr["pts"], pr["cam_idx"], pr["pt_idx"], pr["uv"],
                 loss_s=2.0)
    g = {kk: v.cpu().numpy() for kk, v in out.items()}
    rel = lambda a, b: float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))
    res = {
        "metric": "BA J^TJ build", "n_cam": n_cam, "n_pt": n_pt, "n_obs": n_obs,
        "ms": ms, "obs_per_s": n_obs / (ms * 1e-3),
        "algorithmic_bytes": rd + wr, "bytes_per_obs": (rd + wr) / n_obs,
        "roofline": {"bound": "hbm", "achieved": bw / 1e9, "peak": PEAK_HBM / 1e9,
                     "unit": "GB/s", "frac": bw / PEAK_HBM},
        "parity": {"U_rel": rel(g["U"], o["U"]), "V_rel": rel(g["V"], o["V"]),
                   "W_rel": rel(g["W"], o["W"]), "gc_rel": rel(g["gc"], o["gc"]),
                   "res_max_abs_px": float(np.abs(g["res"] - o["res"]).max()),
                   "cost_rel": abs(float(g["cost"][0]) - o["cost"]) / abs(o["cost"])},
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
