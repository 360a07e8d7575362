"""Tracks (sfm_tracks) on the 500 x 4096 incremental scene's verified graph (all 124 750 pairs,
1024 hypotheses as in incremental.reconstruct): wall per build_tracks call (device-synchronised,
10 calls) and a digest of the tracks for cross-build comparison.

Usage: python tests/perf/tracks_time.py   -> one JSON line."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import match_graph
import synth


def main():
    s = synth.make_scene(500, 4096, seed=21, k1_range=0.02)
    pairs = synth.unordered_pairs(500)
    gb = match_graph.GraphBuilder(s["desc"], s["kps"], s["n_kp"], n_hyp=1024)
    pt = torch.from_numpy(pairs).cuda()
    count, match, _, rs = gb.run(pt)
    rows = gb.graph_rows(0, count, match, rs)
    out = match_graph.build_tracks(rows, pt, s["n_kp"], 2, 0)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        out = match_graph.build_tracks(rows, pt, s["n_kp"], 2, 0)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    h = hashlib.sha256()
    for t in out:
        h.update(t.cpu().numpy().tobytes())
    print(json.dumps({"rows": int(rows.shape[0]), "tracks": int(out[0].shape[0] - 1),
                      "observations": int(out[1].shape[0]), "ms_min": 1e3 * min(ts),
                      "ms_median": 1e3 * float(np.median(ts)), "digest": h.hexdigest()[:16]}))


if __name__ == "__main__":
    main()
