#!/usr/bin/env python3
"""bench.py — verified matches/sec (match + RANSAC) on MI355X, 1..8 GPUs (BASELINE.json metric).

Workload (BASELINE.json configs[2]): 50 synthetic images x 2048 SIFT-like
128-D u8 descriptors, all 1225 unordered pairs; per pair K1 (MFMA L2 match, mutual cross check +
Lowe ratio 0.8) then K2 (8-point RANSAC, 4096 hypotheses, seed 42, Sampson 1 px^2, min 15 inliers).
A step = one pass of match + verify over the pair list with descriptors/keypoints already resident
in HBM, plus, for N > 1, the graph exchange: per-pair counts + 4-byte packed rows, RCCL
all-gather, expanded to (pair, queryIdx, trainIdx) rows on every rank.

Scaling is weak: at N GPUs the scene has n_img images with n_img(n_img-1)/2 ~= 1225*N pairs, cut
into N contiguous cost-balanced shards (one process per GPU, no collective on the data path).
value = verified matches (all ranks) per step * steps / max-over-ranks wall time.

Also reported (rank 0): `roofline` of K1 (algorithmic 2*Ka*Kb*128 ops per pair over the K1 time
measured with HIP events on the launch stream, against the dense i8 MFMA peak), the RANSAC stage
against the fp32 vector peak, and `cpu_baseline`: the CPU oracle (oracle/, OpenMP over pairs) timed
on a bounded sample of the same pairs on this host, with a bit-exact comparison of the sampled
pairs' inlier counts against the GPU's.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "oracle")]

# MI355X dense peaks (MI355X_MICROARCH.md): i8 MFMA 2x bf16 = 2048 op/clk/SIMD * 1024 SIMD * 2.4 GHz
PEAK_I8_TOPS = 2048 * 4 * 256 * 2.4e9 / 1e12        # 5033 TOP/s
PEAK_F32_VALU_TFLOPS = 157.3
RANSAC_FLOP_PER_EVAL = 33      # Sampson test: 16 fma + 1 mul (ransac.hip sampson_inlier)
RANSAC_FLOP_PER_FIT = 1400     # sample + fit_f8: Householder QR 8x9 + Q e9 + adj(F^T F) power iteration


def pmc_traffic(kernel, n_img, k, world):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this exact workload
    (tools/pmc_traffic.sh -> profiles/r01_traffic_cfg3.json: FETCH_SIZE x2 + WRITE_SIZE, separate
    passes, MI355X_MICROARCH.md corrections), or None for any other workload."""
    f = os.path.join(ROOT, "profiles", "r01_traffic_cfg3.json")
    if not (os.path.exists(f) and n_img == 50 and k == 2048 and world == 1):
        return None
    try:
        return float(json.load(open(f))["kernels"][kernel]["hbm_bytes"])
    except (KeyError, ValueError):
        return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-img", type=int, default=0, help="override image count")
    ap.add_argument("--k", type=int, default=2048)
    ap.add_argument("--n-hyp", type=int, default=4096)
    ap.add_argument("--cpu-pairs", type=int, default=384,
                    help="CPU baseline sample (pairs; ~20 s of CPU work at cfg3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="rehearsal only: 'gloo' lets N ranks share one GPU (RCCL cannot)")
    ap.add_argument("--device", type=int, default=-1, help="rehearsal only: force this GPU")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import match_graph
    import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device >= 0:
        local = args.device
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    n_img = args.n_img or (50 if world == 1 else
                           int(round((1 + math.sqrt(1 + 8 * 1225 * world)) / 2)))
    t0 = time.time()
    scene = synth.make_scene(n_img, args.k, seed=0)
    pairs = synth.unordered_pairs(n_img)
    ranges = [match_graph.shard_range(pairs, r, world, scene["n_kp"]) for r in range(world)]
    pair_base, pair_end = ranges[rank]
    shard = pairs[pair_base:pair_end]
    log(f"[rank {rank}] scene {n_img} imgs x {args.k} kps, {len(pairs)} pairs, shard "
        f"{len(shard)} (gen {time.time() - t0:.1f}s)")

    gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"], device=local,
                                  ratio=(4, 5), n_hyp=args.n_hyp, seed=42, thr=1.0,
                                  min_inliers=15)
    pairs_t = torch.from_numpy(np.ascontiguousarray(shard)).cuda()

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        count, match, _ = gb.match(pairs_t)
        if ev is not None:
            ev[1].record()
        rs = gb.verify(pairs_t, count, match)
        if ev is not None:
            ev[2].record()
        if world == 1:  # the local rows are the whole graph: no exchange
            return gb.graph_rows(pair_base, count, match, rs), count, rs
        rows, offs = gb.graph_rows(pair_base, count, match, rs, return_offsets=True)
        counts, packed = match_graph.pack_rows(rows, offs)
        graph = match_graph.all_gather_graph(counts, packed, ranges)
        return graph, count, rs

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t_start = time.perf_counter()
    for k in range(args.steps):
        graph, count, rs = step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64,
                      device="cuda" if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    verified_per_step = int(graph.shape[0])
    match_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    ransac_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    n_kp = scene["n_kp"].astype(np.float64)
    k1_ops = 2.0 * 128 * float(np.sum(n_kp[shard[:, 0]] * n_kp[shard[:, 1]]))
    k1_tops = k1_ops / (match_ms * 1e-3) / 1e12
    cnt_np = count.cpu().numpy()
    m_valid = np.where(cnt_np >= 8, cnt_np, 0).astype(np.float64)
    r_flops = args.n_hyp * float(np.sum(m_valid * RANSAC_FLOP_PER_EVAL + (m_valid > 0) * RANSAC_FLOP_PER_FIT))
    r_tflops = r_flops / (ransac_ms * 1e-3) / 1e12

    value = verified_per_step * args.steps / elapsed
    result = {
        "metric": "verified matches/sec (match+RANSAC)",
        "value": value,
        "unit": "verified matches/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8 MFMA -> exact int32 (K1), f32 (K2)",
        "data": "synthetic (seeded scene: SIFT-like u8 descriptors, 25% misplaced keypoints)",
        "config": {
            "workload": ("cfg3: all unordered pairs of n_img synthetic images x 2048 128-D u8 "
                         "descriptors; L2 match (mutual cross check + ratio 4/5) + 8-point "
                         "RANSAC 4096 hyp/pair (seed 42, Sampson 1 px^2, min 15 inliers)"),
            "n_img": n_img, "pairs_total": int(len(pairs)), "pairs_per_gpu": int(len(shard)),
            "k": args.k, "n_hyp": args.n_hyp, "parallelism": f"pair-sharded dp{world}",
        },
        "verified_matches_per_step": verified_per_step,
        "roofline": {"kernel": "K1 L2 match, mutual rule (mfma_prep + mfma_mutual_kernel + mutual_finalize, HIP events)",
                     "bound": "mfma", "achieved": k1_tops, "peak": PEAK_I8_TOPS,
                     "unit": "TOP/s (i8)", "frac": k1_tops / PEAK_I8_TOPS,
                     "traffic": pmc_traffic("mfma_mutual_kernel", n_img, args.k, world),
                     "traffic_unit": "bytes per mfma_mutual_kernel launch (PMC, profiles/r01_traffic_cfg3.json)",
                     "ms": match_ms, "ops_per_launch": k1_ops},
        "stages": {"match_ms": match_ms, "ransac_ms": ransac_ms,
                   "graph_ms": elapsed / args.steps * 1e3 - match_ms - ransac_ms,
                   "ransac_roofline": {"bound": "f32 VALU", "achieved": r_tflops,
                                       "peak": PEAK_F32_VALU_TFLOPS, "unit": "TFLOP/s",
                                       "frac": r_tflops / PEAK_F32_VALU_TFLOPS,
                                       "flops_per_launch": r_flops}},
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(scene, pairs, shard, pair_base, count, rs,
                                              args.cpu_pairs, args.n_hyp)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(scene, pairs, shard, pair_base, count, rs, n_sample, n_hyp):
    import numpy as np
    import oracle as O
    threads = min(16, len(os.sched_getaffinity(0)))
    O.set_threads(threads)
    stride = max(1, len(shard) // max(1, n_sample))
    idx = np.arange(0, len(shard), stride)[:n_sample]
    sample = np.ascontiguousarray(shard[idx])
    t0 = time.perf_counter()
    tot, nm, ni = O.match_verify_batch(scene["desc"], scene["kps"], sample, ratio=(4, 5), H=n_hyp,
                                       seed=42, thr=1.0, min_inl=15)
    dt = time.perf_counter() - t0
    g_cnt = count.cpu().numpy()[idx]
    g_inl = rs["inl_count"].cpu().numpy()[idx]
    parity = bool((g_cnt == nm).all() and (np.maximum(g_inl, 0) == ni).all())
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if "model name" in l][0]
    except Exception:
        model = "unknown"
    return {"value": tot / dt, "unit": "verified matches/s", "cores": threads, "kind": "port",
            "sample": (f"{len(sample)} of {len(shard)} pairs (stride {stride}), full K1+K2 per "
                       f"pair, OpenMP over pairs, {dt:.1f} s wall on {model}"),
            "per_pair_ms": dt * 1e3 * threads / len(sample),
            "inlier_parity_with_gpu": parity}


if __name__ == "__main__":
    main()
