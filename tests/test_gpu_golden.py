"""GPU vs the committed golden vectors (tests/golden/oracle_fixtures.npz): no oracle at run time."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def test_gpu_matches_golden_vectors(ctx):
    import torch
    f = dict(np.load(os.path.join(G, "oracle_fixtures.npz")))
    meta = json.loads(bytes(f["meta"]).decode())
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    pairs = f["scene_pairs"]
    cnt, mt, dist = ctx.match_batch(T(f["scene_desc"]), T(f["scene_n_kp"]), T(pairs),
                                    cross_check=meta["cross_check"], ratio=tuple(meta["ratio"]))
    rs = ctx.ransac_batch(T(f["scene_kps"]), T(pairs), cnt, mt, n_hyp=meta["n_hyp"],
                          seed=meta["seed"], thr=meta["thr"])
    torch.cuda.synchronize()
    cnt, mt, dist = cnt.cpu().numpy(), mt.cpu().numpy(), dist.cpu().numpy()
    rs = {k: v.cpu().numpy() for k, v in rs.items()}
    for p in range(len(pairs)):
        exp = f[f"pair{p}_match"]
        assert cnt[p] == len(exp)
        np.testing.assert_array_equal(mt[p, :cnt[p]], exp)
        np.testing.assert_array_equal(dist[p, :cnt[p]], f[f"pair{p}_dist"])
        assert rs["inl_count"][p] == f[f"pair{p}_count"]
        assert rs["best_h"][p] == f[f"pair{p}_best_h"]
        np.testing.assert_array_equal(rs["mask"][p, :cnt[p]], f[f"pair{p}_mask"])
        np.testing.assert_array_equal(rs["F"][p].view(np.uint32), f[f"pair{p}_F_bits"])
        np.testing.assert_array_equal(rs["norm"][p].view(np.uint32), f[f"pair{p}_norm_bits"])
    od = f["orb_desc"]
    c2, m2, d2 = ctx.match_batch(T(od), T(np.array([od.shape[1]] * 2, np.int32)),
                                 T(np.array([[0, 1]], np.int32)), metric=1, cross_check=2,
                                 max_dist=26)
    torch.cuda.synchronize()
    k = int(c2.cpu()[0])
    np.testing.assert_array_equal(m2.cpu().numpy()[0, :k], f["orb_match"])
    np.testing.assert_array_equal(d2.cpu().numpy()[0, :k], f["orb_dist"])
