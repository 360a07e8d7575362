"""Worker of tests/test_gpu_incremental.py::test_incremental_sharded_matching_two_ranks: one rank of
a torch.distributed.run job (gloo, every rank on GPU 0 — RCCL cannot share a device), incremental
SfM with the matching sharded across the ranks; every rank writes its reconstruction to
OUT.rank<r>.npz.  A third argument `shard_ba` also shards every bundle adjustment by point.
A fourth one picks the sharded BA's PCG branch (auto | sharded | replicated).
Usage: python -m torch.distributed.run --nproc-per-node N ... worker.py OUT [shard_ba] [pcg]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch
import torch.distributed as dist

import incremental
import synth


def main():
    out = sys.argv[1]
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    scene = synth.make_scene(10, 1024, seed=21, k1_range=0.02)
    intr = np.c_[scene["cams"][:, 6:8], scene["pp"]]
    shard_ba = len(sys.argv) > 2 and sys.argv[2] == "shard_ba"
    pcg = sys.argv[3] if len(sys.argv) > 3 else "auto"
    rec = incremental.reconstruct(scene["desc"], scene["kps"], scene["n_kp"], intr, device=0,
                                  shard_ba=shard_ba, ba_pcg=pcg)
    tptr, timg, tkp = rec.tracks
    np.savez(f"{out}.rank{dist.get_rank()}.npz", cams=rec.cams, registered=rec.registered,
             points=rec.points, has_point=rec.has_point, tptr=tptr, timg=timg, tkp=tkp)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
