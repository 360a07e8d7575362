"""CPU: the oracle (oracle/sfm_oracle*.c) against independent restatements.

* matching vs a numpy brute-force restatement of the same spec (exact integers);
* Philox against the Random123 known-answer vectors, Floyd sampling vs a pure-Python restatement;
* the 8-point fit vs numpy's SVD null space and exact two-view geometry;
* RANSAC vs the synthetic scene's ground truth;
* BA Jacobians vs central finite differences of an independent numpy projection.
"""
import numpy as np
import pytest

import oracle as O
import synth


def np_match(A, B, metric=0, xc=1, ratio=None, max_dist=-1):
    """numpy restatement of DESIGN.md §3.1 (independent of the C oracle)."""
    A = A.astype(np.int64)
    B = B.astype(np.int64)
    if metric == 0:
        D = (A * A).sum(1)[:, None] + (B * B).sum(1)[None, :] - 2 * A @ B.T
    else:
        ab = np.unpackbits(A.astype(np.uint8), axis=1).astype(np.int64)
        bb = np.unpackbits(B.astype(np.uint8), axis=1).astype(np.int64)
        D = ab.sum(1)[:, None] + bb.sum(1)[None, :] - 2 * ab @ bb.T
    nn = D.argmin(1)                      # first index of the minimum
    d1 = D[np.arange(len(A)), nn]
    if D.shape[1] >= 2:
        d2 = np.partition(D, 1, axis=1)[:, 1]
    else:
        d2 = np.full(len(A), np.iinfo(np.int64).max)
    rnn = D.argmin(0)
    out = []
    if xc == 2:
        best = {}
        for j in range(D.shape[1]):
            q = rnn[j]
            if q not in best or D[q, j] < best[q][0]:
                best[q] = (D[q, j], j)
        for i in range(len(A)):
            if i in best and (max_dist < 0 or best[i][0] < max_dist):
                out.append((i, best[i][1], best[i][0]))
        return out
    for i in range(len(A)):
        j = nn[i]
        if xc == 1 and rnn[j] != i:
            continue
        if ratio is not None and d2[i] != np.iinfo(np.int64).max:
            n, d = ratio
            if metric == 0 and not (d * d * d1[i] < n * n * d2[i]):
                continue
            if metric == 1 and not (d * d1[i] < n * d2[i]):
                continue
        if max_dist >= 0 and not d1[i] < max_dist:
            continue
        out.append((i, j, d1[i]))
    return out


@pytest.mark.parametrize("xc,ratio,md", [(1, (4, 5), -1), (0, None, -1), (2, None, -1),
                                         (1, None, 30000), (0, (7, 10), 50000)])
def test_l2_match_vs_numpy(xc, ratio, md):
    s = synth.make_scene(2, 300, seed=1)
    A, B = s["desc"][0], s["desc"][1][:257]
    B[10] = B[11]  # exact ties
    q, t, d = O.match(A, B, 0, xc, ratio, md)
    ref = np_match(A, B, 0, xc, ratio, md)
    assert list(zip(q.tolist(), t.tolist(), d.tolist())) == [(int(a), int(b), int(c))
                                                              for a, b, c in ref]


@pytest.mark.parametrize("xc,md", [(2, 26), (1, 26), (0, -1)])
def test_hamming_match_vs_numpy(xc, md):
    s = synth.make_scene(2, 200, seed=2, orb=True)
    A, B = s["desc"][0], s["desc"][1]
    q, t, d = O.match(A, B, 1, xc, None, md)
    ref = np_match(A, B, 1, xc, None, md)
    assert list(zip(q.tolist(), t.tolist(), d.tolist())) == [(int(a), int(b), int(c))
                                                              for a, b, c in ref]


def test_opencv_rule_differs_from_mutual_when_expected():
    # query 0's nearest train is 0, but train 0 prefers query 1; train 1's nearest query is 0.
    A = np.array([[10] * 128, [12] * 128], np.uint8)
    B = np.array([[12] * 128, [0] * 128], np.uint8)
    q, t, _ = O.match(A, B, 0, 2)
    assert list(zip(q, t)) == [(0, 1), (1, 0)]     # OpenCV keeps (0 -> 1): not mutual
    q, t, _ = O.match(A, B, 0, 1)
    assert list(zip(q, t)) == [(1, 0)]


KAT = [([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
       ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
       ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1])]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox_known_answers(ctr, key, expect):
    assert O.philox(ctr, key).tolist() == expect


def py_philox(ctr, key):
    c = list(ctr)
    k0, k1 = key
    M = 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & M
            k1 = (k1 + 0xBB67AE85) & M
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & M, p1 & M, ((p0 >> 32) ^ c[3] ^ k1) & M, p0 & M]
    return c


def py_sample8(seed, pa, pb, h, M):
    key = (seed & 0xFFFFFFFF, seed >> 32)
    r = py_philox((h, 0, pa, pb), key) + py_philox((h, 1, pa, pb), key)
    out = []
    for k in range(8):
        jmax = M - 8 + k
        t = (r[k] * (jmax + 1)) >> 32
        if t in out:
            t = jmax
        out.append(t)
    return out


@pytest.mark.parametrize("M", [8, 9, 50, 1000, 4096])
def test_sample8_floyd(M):
    for h in range(0, 300, 7):
        s = O.sample8(0x1234567890ABCDEF, 3, 17, h, M).tolist()
        assert s == py_sample8(0x1234567890ABCDEF, 3, 17, h, M)
        assert len(set(s)) == 8 and min(s) >= 0 and max(s) < M


def _two_view(n=40, noise=0.0, seed=0):
    s = synth.make_scene(2, 200, seed=seed, noise_px=noise, misplace_frac=0.0, inlier_frac=1.0)
    pid = s["point_ids"]
    common = np.intersect1d(pid[0][pid[0] >= 0], pid[1][pid[1] >= 0])[:n]
    i0 = np.array([np.nonzero(pid[0] == c)[0][0] for c in common])
    i1 = np.array([np.nonzero(pid[1] == c)[0][0] for c in common])
    return s["kps"][0][i0].astype(np.float64), s["kps"][1][i1].astype(np.float64)


def test_fit_f8_vs_svd_and_geometry():
    x1, x2 = _two_view(40)
    n1, cx1, cy1, s1 = O.normalize(x1)
    n2, cx2, cy2, s2 = O.normalize(x2)
    ok, F = O.fit_f8(n1[:8], n2[:8])
    assert ok == 0
    F = F.astype(np.float64).reshape(3, 3)
    # numpy null space of the same 8x9 system (before rank-2), for comparison
    a = n1[:8].astype(np.float64)
    b = n2[:8].astype(np.float64)
    A = np.stack([b[:, 0] * a[:, 0], b[:, 0] * a[:, 1], b[:, 0], b[:, 1] * a[:, 0],
                  b[:, 1] * a[:, 1], b[:, 1], a[:, 0], a[:, 1], np.ones(8)], 1)
    f = np.linalg.svd(A)[2][-1].reshape(3, 3)
    U, S, Vt = np.linalg.svd(f)
    f2 = U @ np.diag([S[0], S[1], 0]) @ Vt
    f2 /= np.linalg.norm(f2)
    Fn = F / np.linalg.norm(F)
    assert min(np.abs(Fn - f2).max(), np.abs(Fn + f2).max()) < 2e-3
    assert np.linalg.svd(F)[1][2] < 1e-5 * np.linalg.svd(F)[1][0]
    # every exact correspondence satisfies the epipolar constraint
    h1 = np.c_[n1, np.ones(len(n1))]
    h2 = np.c_[n2, np.ones(len(n2))]
    assert np.abs(np.einsum("ij,jk,ik->i", h2, Fn, h1)).max() < 1e-3


def test_ransac_oracle_recovers_ground_truth():
    s = synth.make_scene(2, 1024, seed=9)
    q, t, _ = O.match(s["desc"][0], s["desc"][1], 0, 1, (4, 5))
    r = O.ransac_f(s["kps"][0][q], s["kps"][1][t], H=1024, seed=42, pa=0, pb=1, thr=1.0)
    pid = s["point_ids"]
    true = (pid[0][q] == pid[1][t]) & (pid[0][q] >= 0)
    inl = r["mask"].astype(bool)
    # misplaced keypoints keep their point id but not their position: geometric truth is
    # "same point AND both keypoints on their projection"; count precision on geometry
    x1, x2 = s["kps"][0][q], s["kps"][1][t]
    assert r["count"] == inl.sum()
    assert inl.sum() >= 15
    assert (true & inl).sum() / inl.sum() > 0.97
    del x1, x2


def _project(cam, pp, X):
    R = synth.angle_axis_to_rotmat(cam[:3])
    uv, _ = synth.project(R, cam[3:6], cam[6], cam[7], pp[0], pp[1], X[None])
    return uv[0]


def test_ba_obs_vs_finite_differences():
    prob = synth.make_ba_problem(4, 10, obs_per_pt=3, seed=5)
    import ctypes as C
    for o in range(0, 30, 7):
        c, p = prob["cam_idx"][o], prob["pt_idx"][o]
        cam, pp, X, uv = prob["cams"][c].copy(), prob["pp"][c], prob["pts"][p].copy(), prob["uv"][o]
        r = np.zeros(2); Jc = np.zeros(16); Jp = np.zeros(6); w = np.zeros(1); rho = np.zeros(1)
        O.lib().oracle_ba_obs(*(O._p(np.ascontiguousarray(v)) for v in (cam, pp, X, uv)),
                              C.c_double(0.0), O._p(r), O._p(Jc), O._p(Jp), O._p(w), O._p(rho))
        np.testing.assert_allclose(r, _project(cam, pp, X) - uv, atol=1e-9)
        eps = 1e-6
        R = synth.angle_axis_to_rotmat(cam[:3])
        num = np.zeros((2, 8))
        for k in range(8):
            cp, cm = cam.copy(), cam.copy()
            if k < 3:  # left-multiplied rotation increment
                d = np.zeros(3); d[k] = eps
                cp[:3] = synth.rotmat_to_angle_axis(synth.angle_axis_to_rotmat(d) @ R)
                d[k] = -eps
                cm[:3] = synth.rotmat_to_angle_axis(synth.angle_axis_to_rotmat(d) @ R)
            else:
                cp[k] += eps; cm[k] -= eps
            num[:, k] = (_project(cp, pp, X) - _project(cm, pp, X)) / (2 * eps)
        np.testing.assert_allclose(Jc.reshape(2, 8), num, rtol=2e-5, atol=2e-4)
        nump = np.zeros((2, 3))
        for k in range(3):
            Xp, Xm = X.copy(), X.copy()
            Xp[k] += eps; Xm[k] -= eps
            nump[:, k] = (_project(cam, pp, Xp) - _project(cam, pp, Xm)) / (2 * eps)
        np.testing.assert_allclose(Jp.reshape(2, 3), nump, rtol=2e-5, atol=2e-4)


def test_ba_jtj_assembly_vs_dense():
    prob = synth.make_ba_problem(3, 8, obs_per_pt=2, seed=3)
    o = O.ba_jtj(prob["cams"], prob["pp"], prob["pts"], prob["cam_idx"], prob["pt_idx"],
                 prob["uv"])
    # dense J from the per-observation blocks, then J^T J blocks must match the accumulators
    import ctypes as C
    nc, npt, no = 3, 8, len(prob["cam_idx"])
    J = np.zeros((2 * no, 8 * nc + 3 * npt))
    rv = np.zeros(2 * no)
    for k in range(no):
        c, p = prob["cam_idx"][k], prob["pt_idx"][k]
        r = np.zeros(2); Jc = np.zeros(16); Jp = np.zeros(6); w = np.zeros(1); rho = np.zeros(1)
        O.lib().oracle_ba_obs(*(O._p(np.ascontiguousarray(v)) for v in
                                (prob["cams"][c], prob["pp"][c], prob["pts"][p], prob["uv"][k])),
                              C.c_double(0.0), O._p(r), O._p(Jc), O._p(Jp), O._p(w), O._p(rho))
        J[2 * k:2 * k + 2, 8 * c:8 * c + 8] = Jc.reshape(2, 8)
        J[2 * k:2 * k + 2, 8 * nc + 3 * p:8 * nc + 3 * p + 3] = Jp.reshape(2, 3)
        rv[2 * k:2 * k + 2] = r
    H = J.T @ J
    g = J.T @ rv
    for c in range(nc):
        np.testing.assert_allclose(o["U"][c], H[8 * c:8 * c + 8, 8 * c:8 * c + 8], rtol=1e-10,
                                   atol=1e-6)
        np.testing.assert_allclose(o["gc"][c], g[8 * c:8 * c + 8], rtol=1e-10, atol=1e-6)
    for p in range(npt):
        s = 8 * nc + 3 * p
        np.testing.assert_allclose(o["V"][p], H[s:s + 3, s:s + 3], rtol=1e-10, atol=1e-6)
    np.testing.assert_allclose(o["cost"], 0.5 * rv @ rv, rtol=1e-12)
