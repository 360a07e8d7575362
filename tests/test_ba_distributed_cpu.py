"""CPU: BA J^TJ sharded by point over 2 ranks (gloo) + the packed camera-block all-reduce.

The per-rank linearisation is the CPU oracle here (test infrastructure standing in for the GPU
kernel); the sharding (shard_points) and the collective (allreduce_camera_blocks) are the product
functions that run over RCCL on the GPU box.  Sums are reassociated across ranks, so U / g_c / cost
agree with the single-process build to fp64 rounding, and V / W / g_p / res exactly.
"""
import os
import socket

import numpy as np

import oracle as O
import reconstruction
import sfmcore
import synth

N_CAM, N_PT = 7, 120


def _problem():
    return synth.make_ba_problem(N_CAM, N_PT, obs_per_pt=4, seed=3)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pr = _problem()
    pt_ptr, _ = sfmcore.csr_by(pr["pt_idx"], N_PT)
    lo, hi = reconstruction.shard_points(pt_ptr, rank, world)
    o0, o1 = int(pt_ptr[lo]), int(pt_ptr[hi])
    o = O.ba_jtj(pr["cams"], pr["pp"], pr["pts"][lo:hi], pr["cam_idx"][o0:o1],
                 pr["pt_idx"][o0:o1] - lo, pr["uv"][o0:o1], loss_s=2.0)
    U, gc = torch.from_numpy(o["U"]), torch.from_numpy(o["gc"])
    cost = torch.tensor([o["cost"]], dtype=torch.float64)
    reconstruction.allreduce_camera_blocks(U, gc, cost)
    ar = torch.arange(6, dtype=torch.float64) * (rank + 1)   # the sharded solve's hook (gloo path)
    reconstruction.make_allreduce()(ar[1:5])
    # the replicated PCG branch's gather of the point-side blocks (ragged shards, rank order)
    cuts = [reconstruction.shard_points(pt_ptr, r, world) for r in range(world)]
    c_obs = [int(pt_ptr[b] - pt_ptr[a]) for a, b in cuts]
    Wall = reconstruction._gather_rows(torch.from_numpy(o["W"]), c_obs, None).numpy()
    Vall = reconstruction._gather_rows(torch.from_numpy(o["V"]), [b - a for a, b in cuts],
                                       None).numpy()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), U=U.numpy(), gc=gc.numpy(), ar=ar.numpy(),
             cost=cost.numpy(), V=o["V"], W=o["W"], res=o["res"], lo=lo, hi=hi, o0=o0, o1=o1,
             Wall=Wall, Vall=Vall)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_points_balanced():
    ptr = np.concatenate([[0], np.cumsum(np.random.default_rng(1).integers(2, 9, 1000))])
    for world in (1, 2, 3, 8):
        cuts = [reconstruction.shard_points(ptr, r, world) for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == 1000
        assert all(a[1] == b[0] for a, b in zip(cuts, cuts[1:]))
        loads = [ptr[h] - ptr[l] for l, h in cuts]
        assert max(loads) <= ptr[-1] / world + 8


def test_ba_allreduce_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    pr = _problem()
    full = O.ba_jtj(pr["cams"], pr["pp"], pr["pts"], pr["cam_idx"], pr["pt_idx"], pr["uv"],
                    loss_s=2.0)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(2)]
    assert r[0]["hi"] == r[1]["lo"] and r[1]["hi"] == N_PT
    for k in range(2):
        np.testing.assert_allclose(r[k]["U"], full["U"], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(r[k]["gc"], full["gc"], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(r[k]["cost"][0], full["cost"], rtol=1e-12)
        lo, hi, o0, o1 = (int(r[k][n]) for n in ("lo", "hi", "o0", "o1"))
        np.testing.assert_array_equal(r[k]["V"], full["V"][lo:hi])
        np.testing.assert_array_equal(r[k]["W"], full["W"][o0:o1])
        np.testing.assert_array_equal(r[k]["res"], full["res"][o0:o1])
        np.testing.assert_array_equal(r[k]["ar"], [0, 3, 6, 9, 12, 5 * (k + 1)])
        # replicated branch: every rank holds the whole W / V after the ragged all-gather
        np.testing.assert_array_equal(r[k]["Wall"], full["W"])
        np.testing.assert_array_equal(r[k]["Vall"], full["V"])
