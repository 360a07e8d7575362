"""Time the graph exchange's expansion at cfg4 size on one GPU: the gathered packed graph of 8 ranks
(124 750 pairs, ~113 M rows in padded per-rank slots) expanded to [n,3] rows by the torch ops the
exchange used before (repeat_interleave + shifts + stack + cat) and by sfm_graph_expand (one
launch, after four small torch scans); the two results are compared bit for bit.

Usage: python tests/perf/graph_expand_time.py [world]   -> one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import match_graph
import synth


def torch_expand(call, rall, tot, ranges):
    out = []
    for r, (lo, hi) in enumerate(ranges):
        c, pk = call[r, :hi - lo], rall[r, :tot[r]]
        pair = torch.repeat_interleave(torch.arange(lo, hi, device=pk.device, dtype=torch.int32),
                                       c.long(), output_size=pk.shape[0])
        out.append(torch.stack([pair, (pk >> 16) & 0xFFFF, pk & 0xFFFF], dim=1))
    return torch.cat(out)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        out = fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps, out


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n_img = 500
    pairs = synth.unordered_pairs(n_img)
    n_kp = np.full(n_img, 4096, np.int32)
    ranges = [match_graph.shard_range(pairs, r, world, n_kp) for r in range(world)]
    rng = np.random.default_rng(0)
    maxp = max(hi - lo for lo, hi in ranges)
    call = np.zeros((world, maxp), np.int32)
    for r, (lo, hi) in enumerate(ranges):
        call[r, :hi - lo] = rng.poisson(907, hi - lo)   # cfg4: 113.2 M rows over 124 750 pairs
    tot = [int(x) for x in call.sum(1)]
    maxn = max(tot)
    rall = torch.from_numpy(rng.integers(0, 1 << 28, (world, maxn), dtype=np.int64)
                            .astype(np.int32) & 0x0FFF0FFF).cuda()
    call_d = torch.from_numpy(call).cuda()
    t_old, a = timed(lambda: torch_expand(call_d, rall, tot, ranges))
    t_new, b = timed(lambda: match_graph.expand_gathered(call_d, rall, tot, ranges, maxn))
    same = bool(torch.equal(a, b))
    rows = sum(tot)
    print(json.dumps({"world": world, "pairs": int(len(pairs)), "rows": rows,
                      "torch_ms": t_old, "kernel_ms": t_new, "identical": same,
                      "kernel_GBps": (rows * 16) / (t_new * 1e-3) / 1e9,
                      "note": "kernel bytes: 4 B read + 12 B written per row"}))


if __name__ == "__main__":
    main()
