"""Simulation: does scoring each pair's matches in a different (fixed) order make K2's exact
pruning stop earlier?  Any order gives identical counts (pruning is exact), so only the work
changes.  Orders of the matches after the PV-match preview: natural (the kernel today), outliers
of the best-PREVIEW hypothesis first (computable before scoring), and outliers of the final
winner first (the ideal of this idea).  Same block/wave/bound model as ransac_prune_sim.py
(ordered schedule; block bx's bound = best final count of the blocks before it).  CPU only.
Usage: python tests/perf/ransac_match_order_sim.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
import synth  # noqa: E402

PV = 64


def main():
    s = synth.make_scene(50, 2048, seed=0)
    pairs = synth.unordered_pairs(50)
    rng = np.random.default_rng(1)
    tot = np.zeros(4)
    for p in rng.choice(len(pairs), 6, replace=False):
        a, b = pairs[p]
        q, t, _ = O.match(s["desc"][a], s["desc"][b], 0, 1, (4, 5))
        M, H = len(q), 4096
        masks, _, ok = O.ransac_masks(s["kps"][a][q], s["kps"][b][t], H=H, seed=42, pa=int(a),
                                      pb=int(b), thr=1.0)
        masks = masks.astype(bool) & ok[:, None]
        cnt = masks.sum(1)
        prev = masks[:, :PV].sum(1)
        horder = np.argsort(-prev, kind="stable")

        def work(morder):
            # morder: permutation of matches PV..M-1 (scored after the preview)
            mk = masks[:, morder]
            cum = np.cumsum(mk, 1) + prev[:, None]
            n = M - PV
            chk = np.arange(64, n + 64, 64).clip(max=n)
            w = 0
            for bx in range(H // 256):
                hs = horder[bx * 256:(bx + 1) * 256]
                bnd = cnt[horder[:bx * 256]].max() if bx > 0 else 0
                for wv in range(4):
                    lanes = hs[wv * 64:(wv + 1) * 64]
                    done = n
                    for m in chk:
                        if np.all(cum[lanes, m - 1] + (n - m) < bnd):
                            done = m
                            break
                    w += 64 * done
            return w + H * PV

        nat = np.arange(PV, M)
        hp = horder[0]
        rest = nat
        by_prev = np.r_[rest[~masks[hp, rest]], rest[masks[hp, rest]]]
        hb = int(np.argmax(cnt))
        by_best = np.r_[rest[~masks[hb, rest]], rest[masks[hb, rest]]]
        r = np.array([work(nat), work(by_prev), work(by_best), H * M], float)
        tot += r
        print(p, M, cnt.max(), "natural %.3f  preview-best outliers first %.3f  winner outliers "
              "first %.3f" % tuple(r[:3] / r[3]), flush=True)
    print("all: natural %.3f  preview-best outliers first %.3f  winner outliers first %.3f"
          % tuple(tot[:3] / tot[3]))


if __name__ == "__main__":
    main()
