"""BASELINE configs[1] (cfg2): all 1225 pairs of 50 x 2048 128-D, L2 match with the fused ratio
test (4/5) and no cross check — the dispatcher's ratio path (forward MFMA scan + recovery) — and,
for comparison, the mutual + ratio rule of the bench (mutual kernel).  Per call ms (HIP events,
20 calls) and the i8 fraction of the call.  python tests/perf/k1_cfg2_time.py [rule ...]
(rules: ratio, mutual; default both)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import sfmcore
import synth

PEAK_I8_TOPS = 5033.1648


def main():
    rules = sys.argv[1:] or ["ratio", "mutual"]
    s = synth.make_scene(50, 2048, seed=0)
    pairs = synth.unordered_pairs(50)
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, pr = T(s["desc"]), T(s["n_kp"]), T(pairs)
    ops = 2.0 * 128 * float(sum(int(s["n_kp"][a]) * int(s["n_kp"][b]) for a, b in pairs))
    for rule in rules:
        xc = 0 if rule == "ratio" else sfmcore.XC_MUTUAL
        out = ctx.match_batch(desc, n_kp, pr, cross_check=xc, ratio=(4, 5))
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        reps = 20
        ev[0].record()
        for _ in range(reps):
            out = ctx.match_batch(desc, n_kp, pr, cross_check=xc, ratio=(4, 5), out=out)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        print(json.dumps({"rule": rule, "pairs": len(pairs), "ms_per_call": ms,
                          "matches": int(out[0].sum().item()),
                          "tops_i8": ops / (ms * 1e-3) / 1e12,
                          "frac_dense_i8": ops / (ms * 1e-3) / 1e12 / PEAK_I8_TOPS}), flush=True)


if __name__ == "__main__":
    main()
