"""CPU: the track / triangulation restatement (oracle/recon.py) against independent checks.

Tracks vs scipy.sparse.csgraph.connected_components (labels canonicalised to the smallest node id)
plus the one-keypoint-per-image rule, on random graphs with chains, repeated edges and conflicts.
"""
import numpy as np
import pytest

import recon


def random_graph(rng, n_img=6, k=40, n_rows=300):
    n_kp = rng.integers(k // 2, k, size=n_img)
    pairs = np.array([(a, b) for a in range(n_img) for b in range(a + 1, n_img)], np.int32)
    p = rng.integers(0, len(pairs), size=n_rows)
    q = rng.integers(0, n_kp[pairs[p, 0]])
    t = rng.integers(0, n_kp[pairs[p, 1]])
    rows = np.stack([p, q, t], 1).astype(np.int32)
    return n_kp, pairs, rows


def scipy_tracks(n_kp, pairs, rows, min_len):
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    base = np.r_[0, np.cumsum(n_kp)]
    n = int(base[-1])
    u = base[pairs[rows[:, 0], 0]] + rows[:, 1]
    v = base[pairs[rows[:, 0], 1]] + rows[:, 2]
    _, lab = connected_components(coo_matrix((np.ones(len(u)), (u, v)), shape=(n, n)),
                                  directed=False)
    canon = {}
    for node in range(n):                    # smallest node id of each component
        canon.setdefault(lab[node], node)
    tracks = {}
    for node in range(n):
        tracks.setdefault(canon[lab[node]], []).append(node)
    img = np.searchsorted(base, np.arange(n), side="right") - 1
    out = []
    for key in sorted(tracks):
        nodes = tracks[key]
        im = img[nodes]
        if len(nodes) >= min_len and len(set(im.tolist())) == len(im):
            out.append([(int(img[x]), int(x - base[img[x]])) for x in nodes])
    return out


@pytest.mark.parametrize("seed,min_len", [(0, 2), (1, 2), (2, 3), (3, 2)])
def test_tracks_match_scipy_components(seed, min_len):
    rng = np.random.default_rng(seed)
    n_kp, pairs, rows = random_graph(rng, n_rows=int(rng.integers(50, 400)))
    base = np.r_[0, np.cumsum(n_kp)].astype(np.int32)
    ptr, ti, tk = recon.tracks(base, pairs, rows, min_len)
    got = [list(zip(ti[a:b].tolist(), tk[a:b].tolist())) for a, b in zip(ptr[:-1], ptr[1:])]
    assert got == scipy_tracks(n_kp, pairs, rows, min_len)


def test_tracks_drop_same_image_conflicts():
    # image 0 kp 1 - image 1 kp 2 - image 2 kp 3 - image 0 kp 4: a component with image 0 twice
    n_kp = np.array([10, 10, 10])
    pairs = np.array([[0, 1], [1, 2], [0, 2]], np.int32)
    rows = np.array([[0, 1, 2], [1, 2, 3], [2, 4, 3], [0, 7, 7]], np.int32)
    base = np.r_[0, np.cumsum(n_kp)].astype(np.int32)
    ptr, ti, tk = recon.tracks(base, pairs, rows, 2)
    assert ptr.tolist() == [0, 2] and ti.tolist() == [0, 1] and tk.tolist() == [7, 7]


def _noise_free_problem(seed=0, n_cam=8, n_pt=200, k=4):
    import synth
    prob = synth.make_ba_problem(n_cam, n_pt, obs_per_pt=k, seed=seed, noise_px=0.0, perturb=0.0)
    ptr = np.r_[0, np.cumsum(np.bincount(prob["pt_idx"], minlength=n_pt))].astype(np.int32)
    return prob, ptr


def test_triangulation_recovers_exact_points():
    prob, ptr = _noise_free_problem()
    pts, st = recon.triangulate(prob["cams"], prob["pp"], ptr, prob["cam_idx"], prob["uv"])
    assert np.all(st[:, 3] == 0)
    np.testing.assert_allclose(pts, prob["pts"], rtol=0, atol=1e-7)
    assert st[:, 0].max() < 1e-6                         # px
    assert np.all(st[:, 1] > 0.1) and np.all(st[:, 2] > 0)


def test_triangulation_status_codes():
    prob, ptr = _noise_free_problem(seed=1, n_pt=20)
    ptr = ptr.copy()
    # point 0 keeps a single observation: status 1
    cam_idx, uv = prob["cam_idx"].copy(), prob["uv"].copy()
    ptr2 = np.r_[0, 1, ptr[2:] - 3].astype(np.int32)    # drop 3 of point 0's 4 observations
    keep = np.r_[0, np.arange(4, len(cam_idx))]
    pts, st = recon.triangulate(prob["cams"], prob["pp"], ptr2, cam_idx[keep], uv[keep])
    assert st[0, 3] == 1 and np.all(st[1:, 3] == 0)


# ---- next-view registration (oracle/sfm_oracle_reg.c) ---------------------------------------------

def _rand_pose(rng):
    from scipy.spatial.transform import Rotation
    R = Rotation.random(random_state=int(rng.integers(1 << 30))).as_matrix()
    return R, rng.normal(size=3)


def test_reg_p3p_recovers_pose():
    import oracle as O
    rng = np.random.default_rng(0)
    hits = 0
    for _ in range(200):
        R, t = _rand_pose(rng)
        X = rng.normal(size=(3, 3))
        t = t + np.array([0, 0, 5 - (X @ R.T + t)[:, 2].min()])
        Pc = X @ R.T + t
        b = Pc / np.linalg.norm(Pc, axis=1, keepdims=True)
        sols = [s for s in O.reg_p3p(b, X) if s is not None]
        err = min((np.abs(Rs - R).max() + np.abs(ts - t).max() for Rs, ts in sols), default=1e9)
        hits += err < 1e-6
    assert hits >= 198                       # (near-)degenerate triangles may lose the root


def test_reg_bearing_inverts_projection():
    import oracle as O
    rng = np.random.default_rng(1)
    intr = np.array([1000.0, 0.04, 960.0, 540.0])
    q = rng.uniform(-0.8, 0.8, size=(50, 2))
    xy = intr[0] * (1 + intr[1] * (q * q).sum(1, keepdims=True)) * q + intr[2:]
    b = O.reg_bearing(xy, intr)
    ref = np.c_[q, np.ones(50)]
    ref /= np.linalg.norm(ref, axis=1, keepdims=True)
    np.testing.assert_allclose(b, ref, atol=1e-9)


def test_reg_ransac_finds_pose_with_outliers():
    import oracle as O
    rng = np.random.default_rng(2)
    R, t = _rand_pose(rng)
    X = rng.uniform(-2, 2, size=(300, 3))
    t = t + np.array([0, 0, 8 - (X @ R.T + t)[:, 2].min()])
    intr = np.array([1000.0, 0.02, 960.0, 540.0])
    Pc = X @ R.T + t
    q = Pc[:, :2] / Pc[:, 2:]
    xy = intr[0] * (1 + intr[1] * (q * q).sum(1, keepdims=True)) * q + intr[2:]
    xy += rng.normal(0, 0.5, size=xy.shape)
    out = rng.random(300) < 0.4
    xy[out] = rng.uniform([0, 0], [1920, 1080], size=(int(out.sum()), 2))
    r = O.reg_ransac(xy, X, intr, img=5, n_hyp=512, seed=42, thr=3.0)
    assert r["count"] >= 0.9 * (~out).sum()
    np.testing.assert_allclose(r["R"], R, atol=5e-3)
    assert np.abs(r["t"] - t).max() < 0.05 * np.linalg.norm(t)
    assert r["mask"][~out].mean() > 0.95 and r["mask"][out].mean() < 0.05


def test_reconstruction_host_copies_are_cached_until_the_model_changes():
    """Reconstruction.points / has_point copy the device model once per change, not
    once per read; a replaced tensor or an in-place write gives a fresh copy."""
    import torch
    import incremental
    rec = incremental.Reconstruction(3)
    assert rec.points is None and rec.has_point is None
    rec.pts_d = torch.zeros(4, 3, dtype=torch.float64)
    rec.has_d = torch.zeros(4, dtype=torch.bool)
    p1, p2 = rec.points, rec.points
    assert p1 is p2 and not p1.flags.writeable
    rec.pts_d[1, 2] = 5.0                      # in place
    p3 = rec.points
    assert p3 is not p1 and p3[1, 2] == 5.0   # (a CPU tensor's copy is a view; on the GPU a copy)
    rec.has_d[2] = True
    assert rec.has_point[2] and rec.has_point is rec.has_point
    rec.pts_d = torch.ones(2, 3, dtype=torch.float64)   # replaced
    assert rec.points.shape == (2, 3) and rec.points[0, 0] == 1.0
