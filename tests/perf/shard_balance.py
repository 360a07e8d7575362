"""Load balance of the cfg4 pair sharding (bench.py --gpus N), measured on one GPU:
each rank's shard is run in turn (K1 + K2 + graph rows, HIP events, best of 2) for N = 2, 4, 8,
for the contiguous cost-balanced shards of match_graph.shard_range and for block-cyclic shards
(blocks of B consecutive pairs dealt round-robin).  The step at N GPUs is the slowest rank, so
max/mean of the per-rank times is the scaling loss that the sharding itself causes.
Usage: python tests/perf/shard_balance.py   (B = 256 by default)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import match_graph
import synth


def time_shard(gb, pairs_np, idx, chunk=16384):
    ts = []
    for _ in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        rows = 0
        for c0 in range(0, len(idx), chunk):
            sel = torch.from_numpy(np.ascontiguousarray(pairs_np[idx[c0:c0 + chunk]])).cuda()
            count, match, dist, rs = gb.run(sel)
            r = gb.graph_rows(0, count, match, rs)
            rows += int(r.shape[0])
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts), rows


def main():
    B = int(os.environ.get("BLOCK", "256"))
    s = synth.make_scene(500, 4096, seed=0)
    pairs = synth.unordered_pairs(500)
    gb = match_graph.GraphBuilder(s["desc"], s["kps"], s["n_kp"], device=0)
    time_shard(gb, pairs, np.arange(min(len(pairs), 16384)))  # warm-up
    out = {"block": B, "n_pairs": int(len(pairs))}
    for world in (2, 4, 8):
        for kind in ("contiguous", "block_cyclic"):
            ms, rows = [], []
            for r in range(world):
                if kind == "contiguous":
                    lo, hi = match_graph.shard_range(pairs, r, world, s["n_kp"])
                    idx = np.arange(lo, hi)
                else:
                    blk = np.arange(len(pairs)) // B
                    idx = np.nonzero(blk % world == r)[0]
                t, n = time_shard(gb, pairs, idx)
                ms.append(round(t, 2))
                rows.append(n)
            out[f"n{world}_{kind}"] = {"rank_ms": ms, "rank_rows": rows,
                                       "max_over_mean": round(max(ms) / (sum(ms) / world), 4)}
            print(world, kind, ms, f"max/mean {max(ms) / (sum(ms) / world):.3f}", flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
