"""CPU: pair sharding + verified-match-graph all-gather across ranks (gloo, world_size 2).

The GPU compute is replaced by the CPU oracle (test infrastructure) so the collective logic of
match_graph (shard_range / all_gather_rows / rows_to_pairs) runs here; on the GPU box the same
functions run over RCCL with device tensors.  Shard invariance: the gathered graph must equal the
single-process graph row for row (RANSAC is keyed by (seed, a, b, h)).
"""
import os
import socket

import numpy as np

import match_graph
import oracle as O
import synth

N_IMG, K, H = 5, 256, 256


def _scene():
    return synth.make_scene(N_IMG, K, seed=31)


def _rows_for(scene, pairs, base):
    rows = []
    for p, (a, b) in enumerate(pairs):
        q, t, _ = O.match(scene["desc"][a], scene["desc"][b], 0, 1, (4, 5))
        r = O.ransac_f(scene["kps"][a][q], scene["kps"][b][t], H=H, seed=42, pa=int(a), pb=int(b))
        if r["count"] >= 15:
            idx = np.nonzero(r["mask"])[0]
            rows.extend([(base + p, int(q[i]), int(t[i])) for i in idx])
    return np.array(rows, np.int32).reshape(-1, 3)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = _scene()
    pairs = synth.unordered_pairs(N_IMG)
    lo, hi = match_graph.shard_range(pairs, rank, world, scene["n_kp"])
    rows = torch.from_numpy(_rows_for(scene, pairs[lo:hi], lo))
    graph = match_graph.all_gather_rows(rows)
    if rank == 0:
        np.save(out_path, graph.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_and_balances():
    pairs = synth.unordered_pairs(23)
    n_kp = np.random.default_rng(0).integers(100, 4000, size=23)
    for world in (1, 2, 3, 8):
        cuts = [match_graph.shard_range(pairs, r, world, n_kp) for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == len(pairs)
        for (a, b), (c, d) in zip(cuts, cuts[1:]):
            assert b == c and a <= b
        cost = n_kp[pairs[:, 0]] * n_kp[pairs[:, 1]]
        loads = [cost[a:b].sum() for a, b in cuts]
        assert max(loads) <= cost.sum() / world + cost.max()


def test_all_gather_graph_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "graph.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    gathered = np.load(out)
    scene = _scene()
    pairs = synth.unordered_pairs(N_IMG)
    full = _rows_for(scene, pairs, 0)
    assert len(full) > 0
    np.testing.assert_array_equal(gathered, full)
    graph = match_graph.rows_to_pairs(gathered, pairs)
    assert [(a, b) for a, b, _ in graph] == sorted({(int(pairs[p, 0]), int(pairs[p, 1]))
                                                    for p in full[:, 0]})


def test_all_gather_single_process_is_identity():
    import torch
    rows = torch.arange(12, dtype=torch.int32).reshape(4, 3)
    assert match_graph.all_gather_rows(rows) is rows


def _worker_packed(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = _scene()
    pairs = synth.unordered_pairs(N_IMG)
    ranges = [match_graph.shard_range(pairs, r, world, scene["n_kp"]) for r in range(world)]
    lo, hi = ranges[rank]
    rows = torch.from_numpy(_rows_for(scene, pairs[lo:hi], lo))
    counts = torch.bincount(rows[:, 0].long() - lo, minlength=hi - lo)
    offs = torch.zeros(hi - lo + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(counts, 0)
    c, pk = match_graph.pack_rows(rows, offs)
    graph = match_graph.all_gather_graph(c, pk, ranges)
    if rank == 0:
        np.save(out_path, graph.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_all_gather_packed_graph_gloo_world2(tmp_path):
    """Packed exchange (per-pair counts + 4 B rows) expands to exactly the single-process rows."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "graph.npy")
    mp.spawn(_worker_packed, args=(2, _free_port(), out), nprocs=2, join=True)
    scene = _scene()
    full = _rows_for(scene, synth.unordered_pairs(N_IMG), 0)
    np.testing.assert_array_equal(np.load(out), full)


def test_packed_graph_single_process_roundtrip():
    import torch
    rows = torch.tensor([[3, 5, 7], [3, 4095, 0], [5, 1, 2]], dtype=torch.int32)
    offs = torch.tensor([0, 0, 2, 2, 3], dtype=torch.int64)  # pairs 2..5 (base 2)
    c, pk = match_graph.pack_rows(rows, offs)
    assert c.tolist() == [0, 2, 0, 1]
    g = match_graph.all_gather_graph(c, pk, [(2, 6)])
    np.testing.assert_array_equal(g.numpy(), rows.numpy())


def test_all_gather_packed_graph_gloo_world3(tmp_path):
    """Three ranks, uneven shards (10 pairs): the exchange still yields the single-process rows."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "graph.npy")
    mp.spawn(_worker_packed, args=(3, _free_port(), out), nprocs=3, join=True)
    scene = _scene()
    full = _rows_for(scene, synth.unordered_pairs(N_IMG), 0)
    np.testing.assert_array_equal(np.load(out), full)
