"""Host vs device time of the sharded BA CG loop (world-size-1 RCCL group) at cfg5 scale.

Prints one JSON line: per-iteration wall time and host enqueue time of the sharded loop (eager
launches, or windows of 8 iterations replayed as HIP graphs) and of the unsharded solve.  Run under rocprofv3
--kernel-trace --stats to split the device time by kernel."""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch
import torch.distributed as dist

import reconstruction as R
import synth


def main():
    n_cam, n_pt, k, cg = 500, 100_000, 5, 64
    prob = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=k, seed=0)
    P = R.BAProblem(prob["pp"], prob["cam_idx"], prob["pt_idx"], prob["uv"], n_cam, n_pt)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    lin = P.linearize(T(prob["cams"]), T(prob["pts"]))
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ar = R.make_allreduce()
    ar_torch = R.make_allreduce(direct=False)
    shs = lambda it, a=ar, **kw: P.ctx.ba_solve_sharded(lin, P.cam_idx, P.pt_idx, P.pt_ptr,
                                                        P.cam_ptr, P.cam_obs, 1e-3, a,
                                                        max_iter=it, tol=0.0, **kw)
    out = {}
    for name, fn in (("sharded_torch_pg_poll8", lambda it: shs(it, ar_torch, poll=8, graph=False)),
                     ("sharded_direct_poll0", lambda it: shs(it, poll=0)),
                     ("sharded_direct_poll8", lambda it: shs(it, poll=8, graph=False)),
                     ("sharded_direct_graph_poll8", lambda it: shs(it, poll=8, graph=True)),
                     ("unsharded_poll0", lambda it: P.solve(lin, 1e-3, max_iter=it, tol=0.0, poll=0)),
                     ("unsharded_poll8", lambda it: P.solve(lin, 1e-3, max_iter=it, tol=0.0, poll=8))):
        for _ in range(3):
            fn(cg)
        torch.cuda.synchronize()
        host, wall = [], []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(cg)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append(t1 - t0)
            wall.append(t2 - t0)
        out[name] = {"host_enqueue_us_per_iter": 1e6 * min(host) / cg,
                     "wall_us_per_iter": 1e6 * min(wall) / cg}
    # host cost of one all-reduce call alone
    c = torch.zeros(8 * n_cam, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        ar_torch(c)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["torch_allreduce_alone"] = {"host_us": 1e6 * (t1 - t0) / 200, "wall_us": 1e6 * (t2 - t0) / 200}
    R.release_allreduce()
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
