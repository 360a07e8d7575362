#!/usr/bin/env python3
"""bench.py — verified matches/sec (match + RANSAC) on MI355X, 1..8 GPUs (BASELINE.json metric).

Workload (default `--config cfg4`, BASELINE.json configs[3]): 500 synthetic images
x 4096 SIFT-like 128-D u8 descriptors, all 124 750 unordered pairs; per pair K1 (MFMA L2 match,
mutual cross check + Lowe ratio 4/5) then K2 (8-point RANSAC, 4096 hypotheses, seed 42, Sampson
1 px^2, min 15 inliers).  `--config cfg3` (configs[2]) is 50 x 2048, 1225 pairs.

A step = one pass of match + verify over this rank's pairs (launched in chunks of `--chunk`
pairs) with descriptors/keypoints already resident in HBM, producing the verified match graph:
rows (pair, queryIdx, trainIdx) of every verified pair's inliers.  For N > 1 the step ends with
the graph exchange (per-pair counts + 4-byte packed rows, RCCL all-gather, expanded on every
rank), the analogue of `pair_matches` (code/pipeline.py:36-47).

Scaling is strong: the pair list is fixed and cut into N contiguous cost-balanced shards (one
process per GPU, no collective on the data path, RANSAC keyed by (seed, a, b, h) so results do
not depend on the sharding).  value = verified matches of the whole graph per step * steps /
max-over-ranks wall time.

Also reported (rank 0): `roofline` of K1 (algorithmic 2*Ka*Kb*128 i8 ops per pair over the K1
time measured with HIP events on the launch stream, against the dense i8 MFMA peak), the RANSAC
stage against the f32 vector peak (algorithmic and executed evaluations), `cpu_baseline` (N = 1):
the CPU oracle (oracle/, OpenMP over pairs) timed on a bounded stride sample of the same pairs on
this host, with the sampled pairs' full results (match indices, inlier masks, winners, graph
rows) compared against the GPU's, and `cfg1_cpu`: the reference's own shape (2 images x 512,
code/feature_matching.py:48-58 + RANSAC) timed fully on one core.  `cfg3` (N = 1, cfg4 runs):
the north_star's 2048 x 128 K1 kernel and the cfg3 step, measured in the same run.

`--config cfg5` (BASELINE configs[4]): full incremental SfM on a 500 x 4096 synthetic scene
(incremental.reconstruct: match + verify sharded over the ranks with the graph all-gathered, tracks,
registration, triangulation, LM bundle adjustment with the camera blocks all-reduced and the PCG
sharded or replicated by reconstruction.pcg_rule); a step = one whole reconstruction.  Every N = 1
cfg4 line carries a `cfg5` object measured in the same run.

Launch: `--gpus N` with no external launcher (WORLD_SIZE unset) starts N fresh rank processes
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT, rank r on GPU
r), relays rank 0's JSON line and exits non-zero if any rank fails; it refuses (rc 2) when fewer
than N GPUs are visible.  The launcher never imports torch: it counts GPUs from the KFD topology
(visible_gpus) and prints a `launcher-selfcheck` line on stderr showing that no HIP runtime was
mapped into it.  `--ranks-per-gpu R --dist-backend gloo` rehearses the same count-then-spawn path
with R ranks per GPU on a smaller box.  Under torch.distributed.run, `--gpus` must equal
WORLD_SIZE (rc 2 otherwise).
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
# practical ceilings of this chip (tools/mfma_peak.hip, profiles/r02/mfma_peak_i8.json): i8
# MFMA-only loop on random register operands, every CU busy — the clock drops to 1.71-1.78 GHz,
# 3460-3514 TOP/s = 69-70 % of nominal; v_pk_fma_f32 loop 141 TFLOP/s = 90 % of 157.3
PRACTICAL_I8_TOPS = 3490.0
PRACTICAL_F32_VALU_TFLOPS = 141.0
PEAK_F32_VALU_TFLOPS = 157.3
PEAK_HBM = 8.0e12
RANSAC_FLOP_PER_EVAL = 33      # Sampson test: 16 fma + 1 mul (ransac.hip sampson_inlier)
RANSAC_FLOP_PER_FIT = 1400     # sample + fit_f8

CONFIGS = {
    "cfg3": dict(n_img=50, k=2048, name="BASELINE configs[2] (cfg3)"),
    "cfg4": dict(n_img=500, k=4096, name="BASELINE configs[3] (cfg4)"),
    "cfg5": dict(n_img=500, k=4096, name="BASELINE configs[4] (cfg5)"),
}
# cfg5 scene: the incremental tests' seed (k1 in +-0.02) with local visibility (synth.make_scene
# grid / window / track_len): every 3-D point is seen by ~5 of the 3 x 3 neighbouring views around
# its home position — the SURVEY 8d cfg5 shape (~10^5 points, ~5 observations per point; 286 700
# points at 500 x 4096), with baselines an image sequence on the 120-degree arc cannot give
CFG5_SEED = 21
CFG5_WINDOW = 1                       # 3 x 3 neighbouring views may observe a point ...
CFG5_TRACK = 5                        # ... about 5 of them do (~5 obs / point)
CFG5_GRID = (32, 16, 120.0, 40.0)     # 500 views on a 32 x 16 sphere-cap grid, 3.75 / 2.5 deg apart


def pmc_traffic(kernel, cfg, n_img, k, world):
    """HBM bytes per step (all launches of the step, like `achieved`) of `kernel` from the
    committed PMC summary of this exact workload (tools/pmc_traffic.sh: FETCH_SIZE x2 +
    WRITE_SIZE, separate passes, MI355X_MICROARCH.md corrections), or None when no summary of
    this workload is committed."""
    f = os.path.join(ROOT, "profiles", f"traffic_{cfg}.json")
    if not os.path.exists(f) or world != 1:
        return None
    try:
        d = json.load(open(f))
        if d.get("n_img") != n_img or d.get("k") != k:
            return None
        return float(d["kernels"][kernel]["hbm_bytes_per_step"])
    except (KeyError, ValueError):
        return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        return [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if "model name" in l][0]
    except Exception:
        return "unknown"


def workload_string(cfg, n_img, k, n_hyp, chunk):
    return (f"{cfg}: all {n_img * (n_img - 1) // 2} unordered pairs of {n_img} synthetic images x "
            f"{k} 128-D u8 SIFT-like descriptors; L2 match (mutual cross check + ratio 4/5) + "
            f"8-point RANSAC {n_hyp} hyp/pair (seed 42, Sampson 1 px^2, min 15 inliers); "
            f"launches of <= {chunk} pairs")


class Runner:
    """One image set resident on this GPU and this rank's pair shard, cut into launch chunks."""

    def __init__(self, scene, pairs, lo, hi, chunk, n_hyp, local):
        import numpy as np
        import torch
        import match_graph
        self.torch, self.np = torch, np
        self.gb = match_graph.GraphBuilder(scene["desc"], scene["kps"], scene["n_kp"],
                                           device=local, ratio=(4, 5), n_hyp=n_hyp, seed=42,
                                           thr=1.0, min_inliers=15)
        self.ctx = self.gb.ctx
        self.lo, self.hi = lo, hi
        shard = pairs[lo:hi]
        self.chunks = []
        for c0 in range(0, len(shard), chunk):
            part = np.ascontiguousarray(shard[c0:c0 + chunk])
            self.chunks.append((lo + c0, torch.from_numpy(part).cuda()))
        n_kp = scene["n_kp"].astype(np.float64)
        self.k1_ops = 2.0 * 128 * float(np.sum(n_kp[shard[:, 0]] * n_kp[shard[:, 1]]))

    def step(self, ranges=None, ev=None):
        """One pass over the shard; returns the graph rows [n,3] (whole graph when `ranges`)."""
        import match_graph
        torch = self.torch
        rows_l, cnt_l, pk_l = [], [], []
        for ci, (base, pt) in enumerate(self.chunks):
            if ev is not None:
                ev[ci][0].record()
            count, match, _ = self.gb.match(pt)
            if ev is not None:
                ev[ci][1].record()
            rs = self.gb.verify(pt, count, match)
            if ev is not None:
                ev[ci][2].record()
            if ranges is None:
                rows_l.append(self.gb.graph_rows(base, count, match, rs))
            else:
                pk, offs = self.gb.graph_rows(base, count, match, rs, return_offsets=True,
                                              packed=True)
                c = (offs[1:] - offs[:-1]).to(torch.int32)
                cnt_l.append(c)
                pk_l.append(pk)
        if ranges is None:
            return rows_l[0] if len(rows_l) == 1 else torch.cat(rows_l)
        return match_graph.all_gather_graph(torch.cat(cnt_l), torch.cat(pk_l), ranges)

    def events(self):
        torch = self.torch
        return [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in self.chunks]

    @staticmethod
    def stage_ms(ev):
        m = sum(e[0].elapsed_time(e[1]) for e in ev)
        r = sum(e[1].elapsed_time(e[2]) for e in ev)
        return m, r


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg4")
    ap.add_argument("--n-img", type=int, default=0, help="override the config's image count")
    ap.add_argument("--k", type=int, default=0, help="override the config's keypoints/image")
    ap.add_argument("--n-pts", type=int, default=0,
                    help="cfg5: override the scene's 3-D point count (default n_img*n_in/5)")
    ap.add_argument("--n-hyp", type=int, default=4096)
    ap.add_argument("--chunk", type=int, default=131072,
                    help="pairs per K1/K2 launch (default: a cfg4 shard in one launch, ~90 GB of "
                         "buffers at N = 1; same graph checksum as 16384-pair chunks, 1.7-2.2 %% "
                         "faster, profiles/r02/bench_chunk_ab.txt)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU baseline budget (the sample is sized to about this much wall)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cfg3", action="store_true", help="skip the cfg3 side measurement")
    ap.add_argument("--no-cfg5", action="store_true", help="skip the cfg5 side measurement")
    ap.add_argument("--cfg5-n-img", type=int, default=0,
                    help="cfg4 line's cfg5 leg: override its image count (tests; default 500)")
    ap.add_argument("--cfg5-k", type=int, default=0,
                    help="cfg4 line's cfg5 leg: override its keypoints/image (tests; default 4096)")
    ap.add_argument("--no-fp64", action="store_true", help="skip the fp64-K2 side measurement")
    ap.add_argument("--no-local", action="store_true",
                    help="skip the cfg4_local side measurement (local-visibility scene)")
    ap.add_argument("--ba-pcg", default="auto", choices=("auto", "sharded", "replicated"),
                    help="cfg5: the sharded BA's PCG branch (reconstruction.pcg_rule)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="rehearsal only: 'gloo' lets N ranks share one GPU (RCCL cannot)")
    ap.add_argument("--device", type=int, default=-1, help="rehearsal only: force this GPU")
    ap.add_argument("--ranks-per-gpu", type=int, default=1,
                    help="rehearsal only (with --dist-backend gloo): the self-launcher puts rank r "
                         "on GPU r // R, going through the same count-then-spawn path as N GPUs")
    return ap.parse_args(argv)


# SFM_BENCH_KFD_NODES: tests point the launcher at a fake topology
KFD_NODES = os.environ.get("SFM_BENCH_KFD_NODES", "/sys/class/kfd/kfd/topology/nodes")


def visible_gpus(kfd_nodes=None, environ=None):
    """(number of GPUs this process could open, how it was counted) WITHOUT loading the HIP
    runtime: the KFD topology's GPU nodes (simd_count > 0; CPU nodes have none), cut down by
    ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (each an ordinal list
    into what the previous one left, read up to the first bad entry, as the runtimes do; ROCR
    also takes GPU-<uuid> entries).  Without a readable topology the count comes from a
    throwaway child process (it may initialise HIP; this process does not).  An empty variable
    is the runtimes' default (all devices), as HIP's and ROCr's flag parsing treat it."""
    import glob
    import re
    env = os.environ if environ is None else environ
    kfd_nodes = kfd_nodes or KFD_NODES
    n = None
    props = glob.glob(os.path.join(kfd_nodes, "*", "properties"))
    if props:
        n = 0
        for p in props:
            try:
                m = re.search(r"^simd_count\s+(\d+)", open(p).read(), re.M)
            except OSError:
                continue
            n += bool(m and int(m.group(1)) > 0)
        source = "kfd-topology"
    if n is None:
        import subprocess
        r = subprocess.run([sys.executable, "-c",
                            "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=300, env=dict(env))
        try:
            return int(r.stdout.strip().splitlines()[-1]), "child-process"
        except (ValueError, IndexError):
            return 0, "child-process (failed)"
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if not env.get(var, "").strip():   # unset or empty: the runtimes' default, all devices
            continue
        keep, seen = 0, set()
        for tok in (t.strip() for t in env[var].split(",")):
            ok = (tok.isdigit() and int(tok) < n and tok not in seen) or \
                 (var == "ROCR_VISIBLE_DEVICES" and tok.upper().startswith("GPU-"))
            if not ok:
                break
            seen.add(tok)
            keep += 1
        n = min(n, keep)
    return n, source


def launcher_selfcheck():
    """Proof that the launcher stayed GPU-free: torch never imported, no HIP / HSA runtime
    library mapped into this process."""
    try:
        maps = open("/proc/self/maps").read()
    except OSError:
        maps = ""
    return {"torch_imported": "torch" in sys.modules,
            "hip_runtime_mapped": "libamdhip64" in maps or "libhsa-runtime64" in maps}


def die_with_launcher():
    """In a self-launched rank, first thing: SIGTERM when the launcher dies (PR_SET_PDEATHSIG set
    by the child itself, so the launcher needs no preexec_fn / plain fork)."""
    import ctypes
    import signal
    try:
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)
    except OSError:
        return
    ppid = os.environ.get("SFM_BENCH_PARENT_PID")
    if ppid and os.getppid() != int(ppid):   # the launcher died before the prctl
        sys.exit(1)


def launch_ranks(args, argv):
    """`--gpus N` without an external launcher: N fresh child processes, one per GPU (rank r on
    GPU r // --ranks-per-gpu), started by a launcher that never imports torch nor maps the HIP
    runtime (GPUs counted by visible_gpus; checked by launcher_selfcheck, printed on stderr).
    Rank 0's stdout (the JSON line) is relayed; the other ranks' stdout goes to stderr.  Any
    failing rank stops the others; returns the exit code."""
    import signal
    import socket
    import subprocess
    import tempfile
    n, rpg = args.gpus, args.ranks_per_gpu
    if rpg < 1:
        log("bench.py: --ranks-per-gpu must be >= 1")
        return 2
    if (args.device >= 0 or rpg > 1) and args.dist_backend == "nccl":
        log(f"bench.py: --gpus {n} with --device / --ranks-per-gpu > 1 puts several ranks on one "
            f"GPU, which RCCL cannot do; use --dist-backend gloo for a same-GPU rehearsal")
        return 2
    have, source = visible_gpus()
    need = 1 if args.device >= 0 else -(-n // rpg)
    if have < need:
        log(f"bench.py: --gpus {n} needs {need} visible GPUs, {have} visible ({source}; one rank "
            f"per GPU; --ranks-per-gpu R --dist-backend gloo rehearses R ranks per GPU)")
        return 2
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []

    def forward(signum, _frame):  # a signal to the launcher stops the ranks too
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        sys.exit(128 + signum)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SFM_BENCH_LAUNCHER="self",
                   SFM_BENCH_PARENT_PID=str(os.getpid()),
                   SFM_BENCH_DEVICE=str(args.device if args.device >= 0 else r // rpg))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv,
                                      env=env, stdout=out0 if r == 0 else sys.stderr))
    log("bench.py launcher-selfcheck " + json.dumps(dict(
        launcher_selfcheck(), stage="spawned", visible_gpus=have, count_source=source,
        ranks=n, ranks_per_gpu=rpg)))
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.remove(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                log(f"bench.py: rank {r} exited with {c}; stopping the other ranks")
                for q in live:
                    procs[q].send_signal(signal.SIGTERM)
        time.sleep(0.05)
    for p in procs:
        p.wait()
    log("bench.py launcher-selfcheck " + json.dumps(dict(launcher_selfcheck(), stage="exit")))
    out0.seek(0)
    for line in out0.read().splitlines():  # the JSON line to stdout; library chatter to stderr
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line + "\n")
    sys.stdout.flush()
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            return launch_ranks(args, argv)
        if args.gpus < 1:
            log("bench.py: --gpus must be >= 1")
            return 2
        world, launcher = 1, "none"
    else:
        world = int(env_world)
        launcher = os.environ.get("SFM_BENCH_LAUNCHER", "external")
        if launcher == "self":
            die_with_launcher()
        if world != args.gpus:
            log(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
            return 2

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if launcher == "self":
        local = int(os.environ.get("SFM_BENCH_DEVICE", local))
    if args.device >= 0:
        local = args.device
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    dist_info = {"launcher": launcher, "backend": args.dist_backend if world > 1 else None,
                 "rccl_world": (dist.get_world_size() if world > 1 and
                                dist.get_backend() == "nccl" else None),
                 "world": dist.get_world_size() if world > 1 else 1, "device": local}
    if args.config == "cfg5":
        result = cfg5_main(args, world, rank, local, dist_info)
    else:
        result = pairs_main(args, world, rank, local, dist_info)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import reconstruction
        dist.barrier()   # rank 0's side legs (fp64 K2) end before any rank tears the group down
        reconstruction.release_allreduce()
        dist.destroy_process_group()
    return 0


def gather_ranks(world, info):
    """Every rank's dict (rank order) on every rank; [info] at world size 1."""
    if world == 1:
        return [info]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, info)
    return out


def pairs_main(args, world, rank, local, dist_info):
    """cfg3 / cfg4: the verified-matches/s line (match + verify over the pair shard)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import match_graph
    import synth

    cfg = CONFIGS[args.config]
    n_img = args.n_img or cfg["n_img"]
    k = args.k or cfg["k"]
    t0 = time.time()
    scene = synth.make_scene(n_img, k, seed=0)
    pairs = synth.unordered_pairs(n_img)
    ranges = [match_graph.shard_range(pairs, r, world, scene["n_kp"]) for r in range(world)]
    lo, hi = ranges[rank]
    run = Runner(scene, pairs, lo, hi, args.chunk, args.n_hyp, local)
    log(f"[rank {rank}] {args.config}: {n_img} imgs x {k} kps, {len(pairs)} pairs, shard "
        f"[{lo},{hi}) in {len(run.chunks)} launches (gen {time.time() - t0:.1f}s)")
    xr = ranges if world > 1 else None

    # K2's executed share is measured in the timed steps themselves (sfm_ransac_stats: one u32
    # store per score wave + one small reduction kernel per launch, ~10 us at cfg4).  Enabled
    # before the warm-up so the workspace that holds the per-wave counts is sized there; the
    # read below resets the counters before the timed region.
    run.ctx.ransac_stats(enable=True)
    for _ in range(args.warmup):
        run.step(xr)
    torch.cuda.synchronize()
    run.ctx.ransac_stats(enable=True, read=True)
    # this box's i8 matrix ceiling, measured in the same run right before the
    # timed steps (an MFMA-only launch of ~200 ms on every CU), so K1's fraction can be read
    # against the box it ran on; not inside the timed region
    calib = run.ctx.calib_mfma_i8(200.0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [run.events() for _ in range(args.steps)]
    t_start = time.perf_counter()
    for s in range(args.steps):
        graph = run.step(xr, evs[s])
    torch.cuda.synchronize()
    t_own = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64,
                      device="cuda" if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    verified_per_step = int(graph.shape[0])
    checksum = graph_checksum(torch, graph)  # after the timed region
    r_alg, r_exec, r_evals = ransac_flops(run.ctx.ransac_stats(enable=False, read=True),
                                          args.n_hyp, args.steps)
    st = [Runner.stage_ms(e) for e in evs]
    match_ms = float(np.mean([s[0] for s in st]))
    ransac_ms = float(np.mean([s[1] for s in st]))
    per_rank = gather_ranks(world, {
        "rank": rank, "device": local, "pairs": int(hi - lo),
        "shard_ms_per_step": t_own / args.steps * 1e3, "match_ms": match_ms,
        "ransac_ms": ransac_ms, "calib_tops": calib["tops"], "calib_clock_ghz": calib["clock_ghz"]})
    k1_tops = run.k1_ops / (match_ms * 1e-3) / 1e12
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
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int8 MFMA -> exact int32 (K1), f32 (K2)",
        "data": "synthetic (seeded scene: SIFT-like u8 descriptors, 25% misplaced keypoints)",
        "config": {
            "workload": workload_string(args.config, n_img, k, args.n_hyp, args.chunk),
            "baseline_config": cfg["name"], "n_img": n_img, "k": k, "n_hyp": args.n_hyp,
            "pairs_total": int(len(pairs)), "pairs_rank0": int(ranges[0][1] - ranges[0][0]),
            "launches_rank0": len(run.chunks), "parallelism": f"pair-sharded dp{world}",
        },
        "distributed": dict(dist_info, per_rank=per_rank),
        "verified_matches_per_step": verified_per_step,
        "graph_checksum": checksum,
        "roofline": {"kernel": "K1 L2 match, mutual rule (mfma_prep + mfma_mutual_kernel + "
                               "mutual_finalize, HIP events on the launch stream, rank 0)",
                     "bound": "mfma", "achieved": k1_tops, "peak": PEAK_I8_TOPS,
                     "unit": "TOP/s (i8)", "frac": k1_tops / PEAK_I8_TOPS,
                     "traffic": pmc_traffic("mfma_mutual_kernel", args.config, n_img, k, world),
                     "traffic_unit": f"HBM bytes per step (all launches), PMC, "
                                     f"profiles/traffic_{args.config}.json",
                     "ms": match_ms, "ops_per_step": run.k1_ops,
                     "practical_peak": calib["tops"],
                     "frac_of_practical": k1_tops / calib["tops"],
                     "practical_peak_note": "this run's calib probe (below): an i8 MFMA-only launch "
                                            "on random operands on every CU of this box",
                     "practical_peak_recorded": PRACTICAL_I8_TOPS},
        "calib": dict(calib, probe="sfm_calib_mfma_i8: v_mfma_i32_32x32x32_i8 on register "
                                   "operands, random data, 2 waves per SIMD on every CU, ~200 ms, "
                                   "run right before the timed steps (rank 0's device)",
                      nominal_tops=PEAK_I8_TOPS),
        "stages": {"match_ms": match_ms, "ransac_ms": ransac_ms,
                   "graph_ms": elapsed / args.steps * 1e3 - match_ms - ransac_ms,
                   "ransac_roofline": {
                       "bound": "f32 VALU", "peak": PEAK_F32_VALU_TFLOPS, "unit": "TFLOP/s",
                       "achieved": r_alg * r_exec / (ransac_ms * 1e-3) / 1e12,
                       "frac": r_alg * r_exec / (ransac_ms * 1e-3) / 1e12 / PEAK_F32_VALU_TFLOPS,
                       "executed_flops_per_step": r_alg * r_exec,
                       "algorithmic_flops_per_step": r_alg,
                       "executed_frac": r_exec,
                       "evaluations_per_step": r_evals,
                       "executed_counts_masked_lanes": True,
                       "note": "achieved / frac count the EXECUTED work (the exact pruning skips "
                               "the rest): Sampson evaluations counted by the score waves in the "
                               "timed steps (sfm_ransac_stats) x 33 flop + 1400 flop per fitted "
                               "hypothesis; algorithmic = every hypothesis on every match "
                               "(pairs with >= 8 matches); executed_frac = executed / algorithmic. "
                               "executed = ISSUED lane-slots (a score wave runs until its last "
                               "live lane stops: lanes already pruned count as masked slots; plus "
                               "the final kernel's M per pair), so frac is an issue-slot figure, "
                               "an upper bound on useful-work utilisation",
                       "practical_peak": PRACTICAL_F32_VALU_TFLOPS,
                       "frac_of_practical":
                           r_alg * r_exec / (ransac_ms * 1e-3) / 1e12 / PRACTICAL_F32_VALU_TFLOPS}},
    }
    # step-level fraction = sum of the stages' roofline times / measured step time
    # (K1 at the dense-i8 peak; K2 at the f32 VALU peak on the executed share of the work)
    t_k1 = run.k1_ops / (PEAK_I8_TOPS * 1e12)
    t_k2 = r_alg * r_exec / (PEAK_F32_VALU_TFLOPS * 1e12)
    step_s = elapsed / args.steps
    result["step_roofline"] = {
        "frac": (t_k1 + t_k2) / step_s, "k1_ideal_ms": t_k1 * 1e3, "k2_ideal_ms": t_k2 * 1e3,
        "step_ms": step_s * 1e3,
        "note": "sum of stage roofline times / measured step; K2 ideal on the executed "
                "(pruned) share of the algorithmic flops (measured in the timed steps)"}

    if rank == 0 and not args.no_fp64:
        result["k2_fp64"] = fp64_side(run, args.n_hyp)
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(scene, pairs, lo, hi, graph, run.gb,
                                                  args.cpu_seconds, args.n_hyp)
            result["cfg1_cpu"] = cfg1_timing()
        del run, graph   # the side legs below build their own buffers
        torch.cuda.empty_cache()
        if args.config != "cfg3" and not args.no_cfg3:
            result["cfg3"] = cfg3_side(args.n_hyp, args.chunk, calib["tops"])
            try:   # a side leg: its failure is recorded, the line stands
                result["cfg2"] = cfg2_side(calib["tops"])
            except Exception as e:  # noqa: BLE001
                result["cfg2"] = {"error": f"{type(e).__name__}: {e}"}
        if args.config == "cfg4" and not args.no_local:
            torch.cuda.empty_cache()
            try:   # a side leg: its failure is recorded, the cfg4 line stands
                result["cfg4_local"] = cfg4_local_side(n_img, k, args.n_hyp, args.chunk)
            except Exception as e:  # noqa: BLE001
                result["cfg4_local"] = {"error": f"{type(e).__name__}: {e}"}
    if args.config == "cfg4" and not args.no_cfg5:
        # BASELINE configs[4] beside the cfg4 line: at N = 1 on rank 0, at N > 1 on every rank
        # (pair-sharded matching + graph all-gather, point-sharded BA over the group's all-reduce
        # with the PCG branch chosen by reconstruction.pcg_rule on probed latency / bandwidth)
        if world > 1:
            del run, graph
        torch.cuda.empty_cache()
        try:   # a side leg: its failure is recorded, the cfg4 line stands
            r5 = cfg5_run(args.cfg5_n_img or CONFIGS["cfg5"]["n_img"],
                          args.cfg5_k or CONFIGS["cfg5"]["k"], None,
                          2 if world == 1 else 1, 1, world, rank, local, "auto")
        except Exception as e:  # noqa: BLE001
            r5 = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            result["cfg5"] = r5
    return result


def local_scene(n_img, k, n_pts=None):
    """The cfg5 scene (seeded CFG5_SEED, k1 in +-0.02, local visibility on a sphere-cap view
    grid, ~CFG5_TRACK observations per point); returns (scene, grid)."""
    import synth
    n_el = max(1, int(round((n_img / 2) ** 0.5)))
    grid = (-(-n_img // n_el), n_el, CFG5_GRID[2], CFG5_GRID[3])
    return synth.make_scene(n_img, k, seed=CFG5_SEED, k1_range=0.02, n_pts=n_pts,
                            window=CFG5_WINDOW, grid=grid, track_len=CFG5_TRACK), grid


def cfg4_local_side(n_img, k, n_hyp, chunk, steps=3, warmup=1):
    """the cfg4 step (all pairs of n_img x k 128-D, L2 mutual + ratio 4/5,
    RANSAC n_hyp, seed 42) on the local-visibility scene of cfg5, where most pairs share no
    points and fail verification (code/pipeline.py:42 drops them) — the realistic-overlap
    counterpart of the headline's arc scene, on which every pair verifies."""
    import numpy as np
    import torch
    import synth
    scene, _ = local_scene(n_img, k)
    pairs = synth.unordered_pairs(n_img)
    run = Runner(scene, pairs, 0, len(pairs), chunk, n_hyp, torch.cuda.current_device())
    run.ctx.ransac_stats(enable=True)
    for _ in range(warmup):
        run.step()
    torch.cuda.synchronize()
    run.ctx.ransac_stats(enable=True, read=True)
    evs = [run.events() for _ in range(steps)]
    t0 = time.perf_counter()
    for s_ in range(steps):
        graph = run.step(None, evs[s_])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    r_alg, r_exec, r_evals = ransac_flops(run.ctx.ransac_stats(enable=False, read=True), n_hyp,
                                          steps)
    st = [Runner.stage_ms(e) for e in evs]
    m = float(np.mean([x[0] for x in st]))
    r = float(np.mean([x[1] for x in st]))
    # verified pairs of the last step: pairs with at least one graph row
    n_ver = int(torch.unique(graph[:, 0]).numel()) if graph.shape[0] else 0
    tops = run.k1_ops / (m * 1e-3) / 1e12
    return {"workload": (f"cfg4_local: all {len(pairs)} unordered pairs of the cfg5 local-"
                         f"visibility scene ({n_img} x {k} 128-D, seed {CFG5_SEED}, ~{CFG5_TRACK} "
                         f"views per point); same K1 / K2 settings as the headline"),
            "value": graph.shape[0] * steps / el, "unit": "verified matches/s",
            "ms_per_step": el / steps * 1e3, "steps": steps,
            "verified_matches_per_step": int(graph.shape[0]),
            "verified_pairs": n_ver, "pairs": int(len(pairs)),
            "match_ms": m, "ransac_ms": r,
            "k1_frac": tops / PEAK_I8_TOPS,
            "k2_executed_frac": r_exec, "k2_evaluations_per_step": r_evals,
            "graph_checksum": graph_checksum(torch, graph)}


def cfg5_run(n_img, k, n_pts, steps, warmup, world, rank, local, pcg):
    """BASELINE configs[4]: `steps` whole incremental reconstructions of the cfg5 scene (seeded:
    CFG5_SEED, k1 in +-0.02, visibility window CFG5_WINDOW, n_pts 3-D points or the window's
    default) timed between barriers (max over ranks), after `warmup` reconstructions of the first
    4 views.  Returns the measurement dict (rank 0's
    view; quality against the scene's truth, BA sizes / iterations / PCG branch, and the K3 and
    CG-iteration HBM fractions on the final bundle adjustment's problem)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import incremental
    import reconstruction as R
    import synth
    t0 = time.time()
    scene, grid = local_scene(n_img, k, n_pts)
    n_pts = len(scene["pts"])
    intr = np.c_[scene["cams"][:, 6:8], scene["pp"]]
    log(f"[rank {rank}] cfg5 scene {n_img} x {k}, {n_pts} points (gen {time.time() - t0:.1f}s)")
    kw = dict(device=local, shard_ba=world > 1, ba_pcg=pcg)
    w = np.array(sorted({0, 1, grid[1], grid[1] + 1} & set(range(n_img))))  # a 2 x 2 patch
    for _ in range(warmup):
        incremental.reconstruct(scene["desc"][w], scene["kps"][w], scene["n_kp"][w], intr[w], **kw)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    walls = []
    say = (lambda *m: log(f"[rank {rank}] cfg5:", *m)) if rank == 0 else None
    for _ in range(steps):
        t1 = time.perf_counter()
        rec = incremental.reconstruct(scene["desc"], scene["kps"], scene["n_kp"], intr, log=say,
                                      **kw)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t1)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        el = el.cpu() if dist.get_backend() != "nccl" else el
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())

    tptr, timg, tkp = rec.tracks
    obs_track = np.repeat(np.arange(len(tptr) - 1), np.diff(tptr))
    use = rec.has_point[obs_track] & rec.registered[timg]
    pts_ids, pt_idx = np.unique(obs_track[use], return_inverse=True)
    pt_idx = pt_idx.astype(np.int32)
    uv = scene["kps"][timg[use], tkp[use]].astype(np.float64)
    err = R.reprojection_errors(rec.cams, scene["pp"], rec.points[pts_ids], timg[use], pt_idx, uv,
                                device=local)
    reg = rec.registered
    c_est, c_true = synth.camera_centres(rec.cams[reg]), synth.camera_centres(scene["cams"][reg])
    s_, Rm, t_ = synth.similarity_align(c_est, c_true)
    al = (s_ * (Rm @ c_est.T)).T + t_
    out = {
        "workload": (f"cfg5: full incremental SfM on {n_img} synthetic images x {k} 128-D "
                     f"SIFT-like descriptors on a {grid[0]} x {grid[1]} view grid ({n_pts} "
                     f"scene points, each seen by ~{CFG5_TRACK} of the 3 x 3 views around it, "
                     f"seed {CFG5_SEED}): all "
                     f"{n_img * (n_img - 1) // 2} pairs matched + verified (RANSAC 1024 hyp), "
                     f"tracks, P3P registration, triangulation, LM bundle adjustment"),
        "value": rec.n_verified * steps / elapsed, "unit": "verified matches/s (end to end)",
        "s_per_reconstruction": elapsed / steps, "walls_s_rank": walls,
        "verified_matches": rec.n_verified, "registered": int(reg.sum()), "n_img": n_img,
        "n_pts": n_pts,
        "points": int(rec.has_point.sum()), "observations": int(use.sum()),
        "median_reproj_px": float(np.median(err)), "mean_reproj_px": float(err.mean()),
        "max_centre_err_rel_radius": float(np.abs(al - c_true).max() / 8.0),
        "stage_s": {kk: (round(v, 4) if isinstance(v, float) else v)
                    for kk, v in rec.timings.items()},
        "bundle_adjustments": rec.ba_log,
        "ba_phase_s": {k: round(float(sum(b.get(k, 0.0) for b in rec.ba_log)), 4)
                       for k in ("select_s", "entry_wait_s", "setup_s", "problem_s", "schur_s", "lm_s",
                                 "post_s", "s")},
        "lm_steps": int(sum(b["lm_steps"] for b in rec.ba_log)),
        "lm_rejected": int(sum(b.get("lm_rejected", 0) for b in rec.ba_log)),
        "cg_iters": int(sum(b["cg_iters"] for b in rec.ba_log)),
        "pcg_branches": sorted({b["pcg"] for b in rec.ba_log}),
        "shard_ba": world > 1, "n_gpus": world,
    }
    rules = [dict(b["rule"], n_cam=b["n_cam"]) for b in rec.ba_log if isinstance(b.get("rule"), dict)
             and "allreduce_us" in b["rule"]]
    if rules:   # pcg_rule's probed all-reduce latency / bus bandwidth and its verdicts
        out["pcg_rule"] = {"probes": len(rules), "allreduce_us_first": rules[0]["allreduce_us"],
                           "busbw_GBs_first": rules[0]["busbw_GBs"],
                           "allreduce_us_last": rules[-1]["allreduce_us"],
                           "busbw_GBs_last": rules[-1]["busbw_GBs"],
                           "branch_counts": {m: sum(b["pcg"] == m for b in rec.ba_log)
                                             for m in ("sharded", "replicated")}}
    if rank == 0:
        out["ba_rooflines"] = ba_rooflines(scene["pp"], rec.cams, rec.points[pts_ids],
                                           timg[use].astype(np.int32), pt_idx, uv, local)
    return out


def ba_rooflines(pp, cams, pts, cam_idx, pt_idx, uv, device, reps=20, cg=32):
    """K3 (sfm_ba_jtj) and one Schur-PCG iteration on the final bundle adjustment's problem,
    HIP events on the launch stream, against 8 TB/s on their algorithmic bytes
    (tests/perf/ba_bench.py / ba_solve_bench.py accounting)."""
    import numpy as np
    import torch
    import reconstruction as R
    n_cam, n_pt, n_obs = len(cams), len(pts), len(cam_idx)
    P = R.BAProblem(pp, cam_idx, pt_idx, uv, n_cam, n_pt, device)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float64)).to(P.dev)
    c, p = T(cams), T(pts)

    def timed(fn, n):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n
    def timed_graph(fn, n):
        """fn captured once in a HIP graph (torch.cuda.graph; the library launches on torch's
        current stream, which is the capturing one), then replayed n times between events: the
        GPU time of fn's kernels without the host's per-call launch path (a cross-check that the
        eager timing is not host-bound).  None if the capture fails."""
        try:
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()                      # warm on the side stream (sizes the workspace)
                with torch.cuda.graph(g, stream=s):
                    fn()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g.replay()
            e0.record()
            for _ in range(n):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / n
        except Exception:  # noqa: BLE001
            return None

    def measure(P):
        jtj = timed(lambda: P.linearize(c, p, 2.0), reps)
        lin = P.linearize(c, p, 2.0)
        s0 = timed(lambda: P.solve(lin, 1e-3, max_iter=0, tol=0.0), reps)
        sn = timed(lambda: P.solve(lin, 1e-3, max_iter=cg, tol=0.0, poll=-1), max(reps // 4, 2))
        return jtj, (sn - s0) / cg
    jtj_ms, it_ms = measure(P)
    jtj_graph = timed_graph(lambda: P.linearize(c, p, 2.0), reps)
    # the production forms: bundle_adjust's sharding-invariant chunk sums (reconstruction.BAChunks)
    # and, where schur_rule takes it, the explicit reduced camera system on top
    nck = R.ba_chunk_count()
    Pck = R.BAProblem(pp, cam_idx, pt_idx, uv, n_cam, n_pt, device, chunks=nck) if nck else None
    jtj_ck, it_ck = measure(Pck) if nck else (None, None)
    jtj_ck_graph = timed_graph(lambda: Pck.linearize(c, p, 2.0), reps) if nck else None
    explicit = None
    if nck:
        Pe = R.BAProblem(pp, cam_idx, pt_idx, uv, n_cam, n_pt, device, chunks=nck)
        Pe.set_schur()
        sp = Pe.schur
        lin = Pe.linearize(c, p, 2.0)
        s0e = timed(lambda: Pe.solve(lin, 1e-3, max_iter=0, tol=0.0), reps)
        # the same set-up with the group list emptied: no products are formed (the tree and the
        # rest run as before), so the difference is the product kernel alone
        full_n_seg = sp.n_seg
        sp.n_seg = 0
        s0z = timed(lambda: Pe.solve(lin, 1e-3, max_iter=0, tol=0.0), reps)
        sp.n_seg = full_n_seg
        sne = timed(lambda: Pe.solve(lin, 1e-3, max_iter=cg, tol=0.0, poll=-1), max(reps // 4, 2))
        build_ms = s0e - s0z            # T's products (bas_schur_build), once per solve
        tb = sp.n_inst * (192 + 192 + 72)
        gsz = (sp.seg[3] - sp.seg[2]).cpu().numpy()   # products per (chunk, slot) group
        explicit = {"rule": R.schur_rule(sp.n_inst, sp.n_seg, sp.n_slot, n_obs),
                    "n_inst": sp.n_inst, "n_slot": sp.n_slot, "n_seg": sp.n_seg,
                    "group_products": {"mean": float(gsz.mean()), "p50": float(np.median(gsz)),
                                       "p99": float(np.percentile(gsz, 99)),
                                       "max": int(gsz.max())} if len(gsz) else None,
                    "setup_backsub_ms": s0e,
                    "schur_build": {"ms": build_ms, "bytes": tb,
                                    "achieved_GBs": tb / (build_ms * 1e-3) / 1e9 if build_ms > 0 else None,
                                    "frac": tb / (build_ms * 1e-3) / PEAK_HBM if build_ms > 0 else None,
                                    "note": "per solve; algorithmic bytes = per camera-pair product "
                                            "W_a + W_b rows + V_d^-1 (456 B)"},
                    "cg_iteration": {"ms": (sne - s0e) / cg,
                                     "bytes": 1024 * sp.n_slot + 8 * 16 * n_cam,
                                     "note": "S blocks (both orientations, 1 KB per camera pair) "
                                             "+ camera vectors: latency-bound, 2 launches"}}
    idx_b = 4 * (2 * n_obs + (n_pt + 1) + (n_cam + 1) + n_obs)     # cam/pt idx, CSR ptrs, cam_obs
    k3_b = (8 * (8 * n_cam + 2 * n_cam + 3 * n_pt + 2 * n_obs) + idx_b
            + 8 * (64 * n_cam + 9 * n_pt + 24 * n_obs + 8 * n_cam + 3 * n_pt + 2 * n_obs + 1))
    cg_b = n_obs * (192 + 128 + 8) + n_pt * (72 + 4) + n_cam * (64 * 8 + 4 * 8 * 8)
    return {"n_cam": n_cam, "n_pt": n_pt, "n_obs": n_obs,
            "k3": {"ms": jtj_ms, "bytes": k3_b, "achieved_GBs": k3_b / (jtj_ms * 1e-3) / 1e9,
                   "frac": k3_b / (jtj_ms * 1e-3) / PEAK_HBM,
                   "graph_ms": jtj_graph,
                   "graph_frac": k3_b / (jtj_graph * 1e-3) / PEAK_HBM if jtj_graph else None},
            "cg_iteration": {"ms": it_ms, "bytes": cg_b,
                             "achieved_GBs": cg_b / (it_ms * 1e-3) / 1e9 if it_ms > 0 else None,
                             "frac": cg_b / (it_ms * 1e-3) / PEAK_HBM if it_ms > 0 else None},
            "chunked": None if jtj_ck is None else {
                "chunks": nck, "note": "bundle_adjust's form (sharding-invariant chunk sums); "
                                       "the same algorithmic bytes",
                "k3": {"ms": jtj_ck, "frac": k3_b / (jtj_ck * 1e-3) / PEAK_HBM,
                       "graph_ms": jtj_ck_graph,
                       "graph_frac": (k3_b / (jtj_ck_graph * 1e-3) / PEAK_HBM
                                      if jtj_ck_graph else None),
                       "note": "ms: eager calls; graph_ms: the same call replayed as a HIP "
                               "graph (its kernels' GPU time, no host launch path)"},
                "cg_iteration": {"ms": it_ck,
                                 "frac": cg_b / (it_ck * 1e-3) / PEAK_HBM if it_ck > 0 else None}},
            "explicit_schur": explicit,
            "peak_GBs": PEAK_HBM / 1e9}


def cfg5_main(args, world, rank, local, dist_info):
    """`--config cfg5`: the end-to-end line (a step = one whole reconstruction)."""
    cfg = CONFIGS["cfg5"]
    n_img = args.n_img or cfg["n_img"]
    k = args.k or cfg["k"]
    r = cfg5_run(n_img, k, args.n_pts or None, args.steps, args.warmup, world, rank, local,
                 args.ba_pcg)
    n_pts = r["n_pts"]
    per_rank = gather_ranks(world, {"rank": rank, "device": local, "walls_s": r["walls_s_rank"],
                                    "pcg_branches": r["pcg_branches"]})
    result = {
        "metric": "verified matches/sec through full incremental SfM (match+RANSAC+tracks+"
                  "registration+triangulation+BA)",
        "value": r["value"], "unit": "verified matches/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": r["s_per_reconstruction"] * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None,
        "dtype": "int8 MFMA -> exact int32 (K1), f32 (K2), f64 (BA, triangulation, registration)",
        "data": f"synthetic (seeded scene {CFG5_SEED}: SIFT-like u8 descriptors, 25% misplaced "
                f"keypoints, k1 in +-0.02, local visibility: each point seen by ~{CFG5_TRACK} "
                f"neighbouring views of a sphere-cap grid)",
        "config": {"workload": r["workload"], "baseline_config": cfg["name"], "n_img": n_img,
                   "k": k, "n_pts": n_pts,
                   "parallelism": f"pair-sharded dp{world} + point-sharded BA"},
        "distributed": dict(dist_info, per_rank=per_rank),
        "cfg5": r,
    }
    if "ba_rooflines" in r:
        k3 = r["ba_rooflines"]["k3"]
        result["roofline"] = {"kernel": "K3 sfm_ba_jtj on the final BA problem", "bound": "hbm",
                              "achieved": k3["achieved_GBs"], "peak": PEAK_HBM / 1e9,
                              "unit": "GB/s", "frac": k3["frac"], "traffic": None}
    return result


def fp64_side(run, n_hyp, reps=2):
    """Side measurement (after the timed region): K2 in the fp64 mode (sfm_ransac_f_batch_f64)
    against the f32 spec on the same tentative matches of this rank's shard, HIP events on the
    launch stream; plus how many pairs' results differ between the two specs."""
    import numpy as np
    torch = run.torch
    gb = run.gb
    kps64 = gb.kps.double().contiguous()
    t32 = t64 = 0.0
    n_diff = n_ver32 = n_ver64 = inl32 = inl64 = 0
    for _, pt in run.chunks:
        count, match, _ = gb.match(pt)
        out64 = None
        for impl in ("f32", "f64"):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            for r in range(reps + 1):      # first call untimed (workspace growth)
                if r == 1:
                    ev[0].record()
                if impl == "f32":
                    rs32 = gb.verify(pt, count, match)
                else:
                    out64 = gb.ctx.ransac_batch(kps64, pt, count, match, out=out64,
                                                **gb.ransac_kw)
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / reps
            if impl == "f32":
                t32 += ms
                c32 = rs32["inl_count"].cpu().numpy()
            else:
                t64 += ms
                c64 = out64["inl_count"].cpu().numpy()
        mi = gb.min_inliers
        n_diff += int((c32 != c64).sum())
        n_ver32 += int((c32 >= mi).sum())
        n_ver64 += int((c64 >= mi).sum())
        inl32 += int(c32[c32 >= mi].sum())
        inl64 += int(c64[c64 >= mi].sum())
    return {"ransac_ms_f32": t32, "ransac_ms_f64": t64, "f64_over_f32": t64 / t32 if t32 else None,
            "pairs": int(sum(pt.shape[0] for _, pt in run.chunks)),
            "pairs_with_different_count": n_diff, "verified_pairs_f32": n_ver32,
            "verified_pairs_f64": n_ver64, "verified_matches_f32": inl32,
            "verified_matches_f64": inl64,
            "note": "fp64 verification mode (same sampler, schedule and spec in double, bit-exact "
                    "vs the fp64 oracle); timed after the main steps on the same matches"}


def graph_checksum(torch, graph):
    """Order-sensitive checksum of the verified graph rows [n,3] (pair, queryIdx, trainIdx):
    sum over rows of ((pair * 1000003 + q * 1009 + t) mod P) * (row + 1) mod P, P = 2^31 - 1, in
    int64 on the device.  Equal checksums across launch chunkings / rank counts = the same graph."""
    if graph.shape[0] == 0:
        return 0
    P = 2147483647
    g = graph.long()
    v = (g[:, 0] * 1000003 + g[:, 1] * 1009 + g[:, 2]) % P
    w = torch.arange(1, g.shape[0] + 1, device=g.device, dtype=torch.int64) % P
    return int(((v * w) % P).sum().item() % P)


def ransac_flops(stats, n_hyp, steps):
    """K2 flops per step from the device counters of the timed steps (sfm_ransac_stats):
    stats = (executed Sampson evaluations, algorithmic evaluations = n_hyp x M over pairs with
    M >= 8, number of such pairs), summed over `steps`.  Returns (algorithmic flops per step,
    executed fraction, evaluation counts per step)."""
    ex, al, npairs = (v / steps for v in stats)
    fit = RANSAC_FLOP_PER_FIT * n_hyp * npairs
    alg = RANSAC_FLOP_PER_EVAL * al + fit
    exe = RANSAC_FLOP_PER_EVAL * ex + fit
    return alg, (exe / alg if alg > 0 else 0.0), {"executed": ex, "algorithmic": al,
                                                   "pairs_ge8": npairs}


def cpu_baseline(scene, pairs, lo, hi, graph, gb, seconds, n_hyp):
    """The oracle timed on a stride sample of this shard, sized to ~`seconds` of wall; the
    sampled pairs' full results are compared with the GPU's (graph rows of the timed step, and
    match indices / masks / winners of a separate batch of just the sampled pairs)."""
    import numpy as np
    import torch
    import oracle as O
    share = cpu_share()
    aff, threads = share["cpus_in_affinity"], share["threads"]
    O.set_threads(threads)
    shard = pairs[lo:hi]
    cal = np.ascontiguousarray(shard[:: max(1, len(shard) // threads)][:threads])
    t0 = time.perf_counter()
    O.match_verify_batch(scene["desc"], scene["kps"], cal, ratio=(4, 5), H=n_hyp, seed=42,
                         thr=1.0, min_inl=15)
    t_cal = time.perf_counter() - t0
    n_sample = int(max(threads, min(len(shard), seconds / max(t_cal, 1e-3) * len(cal))))
    stride = max(1, len(shard) // n_sample)
    idx = np.arange(0, len(shard), stride)[:n_sample]
    sample = np.ascontiguousarray(shard[idx])
    t0 = time.perf_counter()
    tot, nm, ni, full = O.match_verify_batch(scene["desc"], scene["kps"], sample, ratio=(4, 5),
                                             H=n_hyp, seed=42, thr=1.0, min_inl=15, full=True)
    dt = time.perf_counter() - t0

    # GPU: the sampled pairs as one batch (results are batch-composition invariant)
    pt = torch.from_numpy(sample).cuda()
    count, match, _, rs = gb.run(pt)
    g_cnt = count.cpu().numpy()
    g_match = match.cpu().numpy()
    g_inl = rs["inl_count"].cpu().numpy()
    g_bh = rs["best_h"].cpu().numpy()
    g_mask = rs["mask"].cpu().numpy()
    ok_cnt = bool((g_cnt == nm).all())
    ok_idx = ok_mask = True
    for p in range(len(sample)):
        m = nm[p]
        ok_idx &= bool((g_match[p, :m] == full["match"][p, :m]).all())
        if m >= 8:
            ok_mask &= bool((g_mask[p, :m] == full["mask"][p, :m]).all()
                            and g_bh[p] == full["best_h"][p] and g_inl[p] == ni[p])
    # the timed step's graph rows of the sampled pairs vs the oracle's verified inliers
    gr = graph.cpu().numpy()
    gpair = lo + idx
    sel = np.isin(gr[:, 0], gpair)
    got = gr[sel]
    exp = []
    for p in range(len(sample)):
        if ni[p] >= 15:
            mm = full["mask"][p, :nm[p]].astype(bool)
            q = full["match"][p, :nm[p]][mm]
            exp.append(np.column_stack([np.full(len(q), gpair[p], np.int32), q]))
    exp = np.concatenate(exp) if exp else np.zeros((0, 3), np.int32)
    got = got[np.lexsort((got[:, 1], got[:, 0]))] if len(got) else got
    ok_rows = bool(got.shape == exp.shape and (got == exp).all())
    return {"value": tot / dt, "unit": "verified matches/s", "cores": threads, "kind": "port",
            "sample": (f"{len(sample)} of {len(shard)} pairs (stride {stride}), full K1+K2 per "
                       f"pair, OpenMP over pairs, {dt:.1f} s wall on {model_str(aff)}"),
            "host_cpus_in_affinity": aff, "cpu_share": share, "cpu_model": cpu_model(),
            "per_pair_core_ms": dt * 1e3 * threads / len(sample),
            "parity": {"pairs": int(len(sample)), "match_counts": ok_cnt,
                       "match_indices": bool(ok_idx),
                       "inlier_masks_best_h_counts": bool(ok_mask),
                       "graph_rows_of_timed_step": ok_rows},
            "inlier_parity_with_gpu": bool(ok_cnt and ok_idx and ok_mask and ok_rows)}


def cpu_share():
    """The CPUs this process may use: the affinity mask, the cgroup CPU quota (v2 cpu.max or v1
    cpu.cfs_quota_us / cpu.cfs_period_us) and OMP_NUM_THREADS (the GPU box sets it to the one-GPU
    slot's 16-CPU share and asks that worker pools be sized to it).  threads = the smallest."""
    aff = len(os.sched_getaffinity(0))
    info = {"cpus_in_affinity": aff, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    quota = None
    for path, kind in (("/sys/fs/cgroup/cpu.max", "v2"),
                       ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "v1")):
        try:
            raw = open(path).read().strip()
        except OSError:
            continue
        info["cgroup_" + kind] = raw
        try:
            if kind == "v2":
                q, per = raw.split()
                if q != "max":
                    quota = float(q) / float(per)
            else:
                q = float(raw)
                per = float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                if q > 0:
                    quota = q / per
        except (OSError, ValueError):
            pass
        break
    info["cgroup_cpu_quota"] = quota
    lim = [aff]
    if quota:
        lim.append(max(1, int(math.ceil(quota))))
    if info["omp_num_threads"]:
        lim.append(int(info["omp_num_threads"]))
    info["threads"] = min(lim)
    info["limited_by"] = ("cgroup quota" if quota and info["threads"] == int(math.ceil(quota))
                          else "OMP_NUM_THREADS (the box's per-GPU CPU share)"
                          if info["omp_num_threads"] and info["threads"] == int(info["omp_num_threads"])
                          else "affinity mask")
    return info


def model_str(aff):
    return f"{cpu_model()} ({aff} CPUs in the affinity mask)"


def cfg1_timing():
    """cfg1 (BASELINE configs[0]): the reference's own shape, one 2-image pair x 512 keypoints,
    timed fully on ONE core with the oracle: (a) ORB-like 256-bit descriptors, Hamming,
    OpenCV cross-check rule, `distance < 26` (code/feature_matching.py:48-58) + RANSAC; (b) the
    north_star's SIFT-like L2 descriptors, mutual + ratio 4/5 + RANSAC.  H = 4096."""
    import numpy as np
    import oracle as O
    import synth
    O.set_threads(1)
    out = {"shape": "2 images x 512 keypoints, 1 pair, RANSAC 4096 hyp", "cores": 1,
           "kind": "port", "cpu_model": cpu_model()}
    for name, orb, kw in (("orb_hamming_opencv_lt26", True,
                           dict(metric=1, cross_check=O.XC_OPENCV, max_dist=26)),
                          ("sift_l2_mutual_ratio", False,
                           dict(metric=0, cross_check=O.XC_MUTUAL, ratio=(4, 5)))):
        s = synth.make_scene(2, 512, seed=1, orb=orb)
        reps, t_m, t_r, n = 0, 0.0, 0.0, 0
        t_end = time.perf_counter() + 1.5
        while time.perf_counter() < t_end or reps < 3:
            t0 = time.perf_counter()
            q, t, _ = O.match(s["desc"][0], s["desc"][1], **kw)
            t1 = time.perf_counter()
            r = O.ransac_f(s["kps"][0][q], s["kps"][1][t], H=4096, seed=42, pa=0, pb=1)
            t2 = time.perf_counter()
            t_m += t1 - t0
            t_r += t2 - t1
            n = r["count"]
            reps += 1
        out[name] = {"match_ms": t_m / reps * 1e3, "ransac_ms": t_r / reps * 1e3,
                     "pair_ms": (t_m + t_r) / reps * 1e3, "matches": int(len(q)),
                     "inliers": int(n), "reps": reps}
    return out


def cfg3_side(n_hyp, chunk, practical):
    """cfg3 (50 x 2048, 1225 pairs) on this GPU: the north_star's 2048 x 128 K1 kernel and the
    cfg3 step, 10 timed steps after 3 warmups."""
    import numpy as np
    import torch
    import synth
    scene = synth.make_scene(50, 2048, seed=0)
    pairs = synth.unordered_pairs(50)
    run = Runner(scene, pairs, 0, len(pairs), chunk, n_hyp, torch.cuda.current_device())
    for _ in range(3):
        run.step()
    torch.cuda.synchronize()
    evs = [run.events() for _ in range(10)]
    t0 = time.perf_counter()
    for s in range(10):
        graph = run.step(None, evs[s])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = [Runner.stage_ms(e) for e in evs]
    m = float(np.mean([s[0] for s in st]))
    r = float(np.mean([s[1] for s in st]))
    tops = run.k1_ops / (m * 1e-3) / 1e12
    return {"workload": workload_string("cfg3", 50, 2048, n_hyp, chunk),
            "value": graph.shape[0] * 10 / el, "unit": "verified matches/s",
            "ms_per_step": el / 10 * 1e3, "match_ms": m, "ransac_ms": r,
            "k1_roofline": {"achieved": tops, "peak": PEAK_I8_TOPS, "unit": "TOP/s (i8)",
                            "frac_of_practical": tops / practical, "practical_peak": practical,
                            "frac": tops / PEAK_I8_TOPS,
                            "traffic": pmc_traffic("mfma_mutual_kernel", "cfg3", 50, 2048, 1)}}


def cfg2_side(practical, reps=20):
    """BASELINE configs[1] (cfg2): the 1225 pairs of cfg3's scene, L2 match with the fused ratio
    test (4/5) and no cross check — the dispatcher's ratio path (forward MFMA scan + exact
    recovery) — per call on this GPU (HIP events on the launch stream, `reps` calls after one);
    frac_of_practical against this run's calib probe."""
    import numpy as np
    import torch
    import sfmcore
    import synth
    s = synth.make_scene(50, 2048, seed=0)
    pairs = synth.unordered_pairs(50)
    ctx = sfmcore.context(torch.cuda.current_device())
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, pr = T(s["desc"]), T(s["n_kp"]), T(pairs)
    ops = 2.0 * 128 * float(sum(int(s["n_kp"][a]) * int(s["n_kp"][b]) for a, b in pairs))
    out = ctx.match_batch(desc, n_kp, pr, cross_check=0, ratio=(4, 5))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out = ctx.match_batch(desc, n_kp, pr, cross_check=0, ratio=(4, 5), out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tops = ops / (ms * 1e-3) / 1e12
    return {"workload": "cfg2: all 1225 unordered pairs of 50 synthetic images x 2048 128-D u8 "
                        "descriptors; L2 match with the fused ratio test 4/5, no cross check "
                        "(ratio path: forward MFMA scan + exact recovery)",
            "ms_per_call": ms, "matches": int(out[0].sum().item()),
            "k1_roofline": {"achieved": tops, "peak": PEAK_I8_TOPS, "unit": "TOP/s (i8)",
                            "frac": tops / PEAK_I8_TOPS,
                            "frac_of_practical": tops / practical,
                            "practical_peak": practical}}


if __name__ == "__main__":
    sys.exit(main())
