"""Worker of tests/test_gpu_ba_sharded.py::test_ba_sharded_two_ranks: one rank of a
torch.distributed.run job (gloo, every rank on GPU 0 — RCCL cannot share a device).  Each rank runs
the point-sharded bundle adjustment (reconstruction.bundle_adjust(shard=True): camera-block
all-reduce, sfm_ba_solve_stage with one all-reduce per CG iteration, all-reduced trial cost,
gathered points) and one sharded solve from the initial linearisation; it writes OUT.rank<r>.npz.
A second argument `tiny` uses a 2-point problem (with 3 ranks one shard is empty); a third one
picks bundle_adjust's PCG branch (sharded | replicated | auto; default sharded); a fourth one
repeats the bundle adjustment that many times (sequential auto-mode calls).
Usage: python -m torch.distributed.run --nproc-per-node N ... dist_ba_worker.py OUT [tiny|std] [pcg] [repeat]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd"), os.path.join(ROOT, "tests")]

import numpy as np
import torch
import torch.distributed as dist

import reconstruction as R
import sfmcore
import synth
from test_gpu_ba_sharded import problem, shard_solve, tiny_problem


def main():
    out = sys.argv[1]
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    prob = tiny_problem() if len(sys.argv) > 2 and sys.argv[2] == "tiny" else problem()
    args = (prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"], prob["uv"])
    fixed = R.gauge_mask(prob["cams"], ref=0, fix_intrinsics=True)
    pcg = sys.argv[3] if len(sys.argv) > 3 else "sharded"
    repeat = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    branches, deferred = [], []
    for _ in range(repeat):   # sequential auto-mode calls probe / cache consistently
        binfo = {}
        cams, pts, hist = R.bundle_adjust(*args, loss_s=2.0, max_iter=30, fixed=fixed,
                                          shard=True, pcg=pcg, info=binfo)
        branches.append(binfo["pcg"])
        rule = binfo.get("rule")
        deferred.append(bool(isinstance(rule, dict) and rule.get("explicit_schur_rejected")))
    dc, dp, info, lo, hi = shard_solve(prob, rank, world, R.make_allreduce())
    np.savez(f"{out}.rank{rank}.npz", cams=cams, pts=pts, hist=np.array(hist, np.float64),
             dc=dc, dp=dp, info=info, lo=lo, hi=hi, pcg=np.array(binfo["pcg"]),
             branches=np.array(branches), deferred=np.array(deferred),
             nchunk_adj=np.array(binfo.get("chunks_adjusted", {}).get("nchunk", -1)))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
