"""CPU: the explicit reduced camera system's structure (reconstruction.schur_instances /
schur_spec, include/sfmcore.h sfm_ba_set_schur) against a brute-force construction, and a numpy
restatement of the GPU product (bas_schur_build + bas_pcg_spmv) against the dense Schur complement.
The kernels themselves are checked on the GPU (tests/test_gpu_ba_lm.py::test_explicit_schur_*)."""
import numpy as np
import pytest
import torch

import reconstruction as R


def _problem(seed=0, n_cam=7, n_pt=40, dup=True):
    rng = np.random.default_rng(seed)
    cams, pts = [], []
    for p in range(n_pt):
        m = int(rng.integers(1, 7))
        cs = rng.choice(n_cam, size=min(m, n_cam), replace=False)
        if dup and p == 5:              # one point seen twice by one camera
            cs = np.array([3, 1, 3])
        cams += list(cs)
        pts += [p] * len(cs)
    return np.array(cams, np.int32), np.array(pts, np.int32), n_cam, n_pt


def _brute(cam, pt, n_cam, chunk_pt):
    ptr = np.searchsorted(pt, np.arange(len(np.unique(pt)) + 1))
    ptr = np.r_[np.searchsorted(pt, np.arange(pt.max() + 1)), len(pt)]
    gen, dups = [], []
    for p in range(len(ptr) - 1):
        k = int(np.searchsorted(np.asarray(chunk_pt[1:]), p, side="right"))
        for a in range(ptr[p], ptr[p + 1]):
            for b in range(a + 1, ptr[p + 1]):
                x, y = (a, b) if cam[a] <= cam[b] else (b, a)
                gen.append((k, cam[x], cam[y], x, y))
                if cam[a] == cam[b]:
                    dups.append((k, cam[y], cam[x], y, x))
    inst = gen + dups
    order = sorted(range(len(inst)), key=lambda i: ((inst[i][0] * n_cam + inst[i][1]) * n_cam + inst[i][2], i))
    return [inst[i] for i in order]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_schur_structure_matches_brute_force(seed):
    cam, pt, n_cam, n_pt = _problem(seed)
    chunk_pt = [0, 13, 13, 27, n_pt]          # an empty chunk included
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    ptr = np.r_[np.searchsorted(pt, np.arange(n_pt)), len(pt)].astype(np.int32)
    key, a, b = R.schur_instances(T(cam), T(pt), T(ptr), n_cam, chunk_pt)
    ref = _brute(cam, pt, n_cam, chunk_pt)
    np.testing.assert_array_equal(a.numpy(), [r[3] for r in ref])
    np.testing.assert_array_equal(b.numpy(), [r[4] for r in ref])
    comp, cnt = R.schur_groups(key)
    spec = R.schur_spec(comp, cnt, a, b, n_cam, comp)
    sk = sorted({r[1] * n_cam + r[2] for r in ref})
    np.testing.assert_array_equal(spec.slot_cam.numpy(), [[k // n_cam, k % n_cam] for k in sk])
    # groups: (chunk, slot) runs in order
    groups = []
    for i, r in enumerate(ref):
        g = (r[0], sk.index(r[1] * n_cam + r[2]))
        if not groups or tuple(groups[-1][:2]) != g:
            groups.append([g[0], g[1], i, i + 1])
        else:
            groups[-1][3] = i + 1
    np.testing.assert_array_equal(spec.seg.numpy().T, np.array(groups))
    # the whole problem's groups (one process: its own): chunk of each, each slot's in chunk order
    assert spec.n_group == len(groups) and spec.g0 == 0
    np.testing.assert_array_equal(spec.gk.numpy(), [g[0] for g in groups])
    for si in range(len(sk)):
        mine = [gi for gi, g in enumerate(groups) if g[1] == si]
        np.testing.assert_array_equal(spec.sg.numpy()[spec.sg_ptr[si]:spec.sg_ptr[si + 1]], mine)
    # rows: every slot once in its first camera's row, transposed in its second camera's row
    for c in range(n_cam):
        ents = spec.row_ent.numpy()[spec.row_ptr[c]:spec.row_ptr[c + 1]]
        want = []
        for s, k in enumerate(sk):
            ci, cj = k // n_cam, k % n_cam
            if ci == c:
                want.append((cj, 2 * s))
            if cj == c and ci != cj:
                want.append((ci, 2 * s + 1))
        assert list(ents) == [e for _, e in sorted(want)]


def test_schur_product_restatement_equals_dense():
    """T per slot (Σ Y_a W_bᵀ over its instances, all chunks), S_cc from the camera blocks, then the
    block-row product exactly as bas_pcg_spmv walks row_ent — against the dense Schur complement."""
    rng = np.random.default_rng(5)
    cam, pt, n_cam, n_pt = _problem(3)
    n_obs = len(cam)
    W = rng.standard_normal((n_obs, 8, 3))
    A = rng.standard_normal((n_pt, 3, 3))
    V = np.einsum("pij,pkj->pik", A, A) + 3 * np.eye(3)
    Vi = np.linalg.inv(V)
    U = np.stack([np.eye(8) * 50 for _ in range(n_cam)])
    ptr = np.r_[np.searchsorted(pt, np.arange(n_pt)), n_obs].astype(np.int32)
    T_ = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    key, a, b = R.schur_instances(T_(cam), T_(pt), T_(ptr), n_cam, [0, 20, n_pt])
    comp, cnt = R.schur_groups(key)
    spec = R.schur_spec(comp, cnt, a, b, n_cam, comp)
    Tb = np.zeros((spec.n_slot, 8, 8))
    seg, inst = spec.seg.numpy(), spec.inst.numpy()
    for g in range(spec.n_seg):
        for i in range(seg[2, g], seg[3, g]):
            x, y = inst[0, i], inst[1, i]
            Tb[seg[1, g]] += W[x] @ Vi[pt[x]] @ W[y].T
    Scc = U.copy()
    for o in range(n_obs):
        Scc[cam[o]] -= W[o] @ Vi[pt[o]] @ W[o].T
    # dense reference
    S = np.zeros((8 * n_cam, 8 * n_cam))
    for c in range(n_cam):
        S[8 * c:8 * c + 8, 8 * c:8 * c + 8] = U[c]
    for p in range(n_pt):
        for x in range(ptr[p], ptr[p + 1]):
            for y in range(ptr[p], ptr[p + 1]):
                S[8 * cam[x]:8 * cam[x] + 8, 8 * cam[y]:8 * cam[y] + 8] -= W[x] @ Vi[p] @ W[y].T
    pvec = rng.standard_normal(8 * n_cam)
    q = np.zeros(8 * n_cam)
    sc, rp, re = spec.slot_cam.numpy(), spec.row_ptr.numpy(), spec.row_ent.numpy()
    for c in range(n_cam):
        acc = np.zeros(8)
        for e in range(rp[c], rp[c + 1]):
            s, t = re[e] >> 1, re[e] & 1
            j = sc[s, 0] if t else sc[s, 1]
            acc += (Tb[s].T if t else Tb[s]) @ pvec[8 * j:8 * j + 8]
        q[8 * c:8 * c + 8] = Scc[c] @ pvec[8 * c:8 * c + 8] - acc
    np.testing.assert_allclose(q, S @ pvec, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("cuts", [[0, 2, 6], [0, 1, 3, 6], [0, 3, 3, 6]])
def test_schur_structure_of_shards_equals_whole(cuts):
    """The sharded form: each rank builds its groups from its run of chunks, the group keys are
    gathered (rank order = chunk order), and every shard then holds the whole problem's slots,
    groups and rows; its own groups are the whole problem's rows g0 .. g0 + n_seg, with the same
    instances (as global observations)."""
    cam, pt, n_cam, n_pt = _problem(7, n_pt=60)
    chunk_pt = [0, 9, 20, 20, 33, 47, n_pt]        # 6 chunks, one empty
    ptr = np.r_[np.searchsorted(pt, np.arange(n_pt)), len(pt)].astype(np.int32)
    T_ = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    nn = n_cam * n_cam
    key, a, b = R.schur_instances(T_(cam), T_(pt), T_(ptr), n_cam, chunk_pt)
    comp, cnt = R.schur_groups(key)
    whole = R.schur_spec(comp, cnt, a, b, n_cam, comp)
    parts = []
    for r in range(len(cuts) - 1):
        k0, k1 = cuts[r], cuts[r + 1]
        lo, hi = chunk_pt[k0], chunk_pt[k1]
        o0, o1 = ptr[lo], ptr[hi]
        lcpt = [c - lo for c in chunk_pt[k0:k1 + 1]]
        lk, la, lb = R.schur_instances(T_(cam[o0:o1]), T_(pt[o0:o1] - lo), T_(ptr[lo:hi + 1] - o0),
                                       n_cam, lcpt)
        lc, ln = R.schur_groups(lk)
        parts.append((k0, o0, lc, ln, la, lb))
    all_groups = torch.sort(torch.cat([p[2] + p[0] * nn for p in parts])).values
    np.testing.assert_array_equal(all_groups.numpy(), comp.numpy())
    for k0, o0, lc, ln, la, lb in parts:
        sp = R.schur_spec(lc, ln, la, lb, n_cam, all_groups, k0)
        for name in ("slot_cam", "row_ptr", "row_ent", "sg_ptr", "sg", "gk"):
            np.testing.assert_array_equal(getattr(sp, name).numpy(), getattr(whole, name).numpy())
        g = slice(sp.g0, sp.g0 + sp.n_seg)
        np.testing.assert_array_equal(sp.seg.numpy()[1], whole.seg.numpy()[1][g])       # slots
        np.testing.assert_array_equal(sp.seg.numpy()[0] + k0, whole.seg.numpy()[0][g])  # chunks
        wi0, wi1 = whole.seg.numpy()[2][g][0] if sp.n_seg else 0, whole.seg.numpy()[3][g][-1] if sp.n_seg else 0
        np.testing.assert_array_equal(sp.inst.numpy() + o0, whole.inst.numpy()[:, wi0:wi1])
