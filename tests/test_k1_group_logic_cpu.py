"""CPU: the decision logic of round 5's K1 (mfma_mutual_grp_kernel + mutual_grp_finalize_kernel,
sfm-project_amd/csrc/match_mfma.hip) restated in numpy and checked against the CPU oracle's mutual
+ ratio rule (oracle/sfm_oracle.c) on tie-heavy, duplicated and ragged descriptor sets.

What is restated: the row record the kernel keeps per query — per lane half (the 16 trains of a
32-train tile the MFMA layout gives one lane), the group maximum of e = x'.y' - ceil(|y'|^2/2) per
tile, (best, second-best group maximum, tile of the best) — merged over the two halves as the
kernel does; the exact column winners; and the finalize's classification: the mutual test on the
best proposal, the ratio bound, the tie and group rechecks, the exact row scan.  The GPU runs the
same rules (tests/test_gpu_match.py::test_group_kernel_equals_top2_kernel_and_oracle); this test
pins the rules themselves without a GPU.
"""
import numpy as np
import pytest

import oracle as O

INF = np.iinfo(np.int64).max
PAD = -(1 << 23)          # MU_PAD_ROW: e of a padded train row
E_VALID = -(1 << 22)      # MU_E_VALID


def _ratio_ok(d1, d2, ratio):
    if ratio is None or d2 == INF:
        return True
    num, den = ratio
    return den * den * d1 < num * num * d2


def group_kernel_match(A, B, ratio):
    """Restatement of the group kernel + its finalize for one pair (L2, mutual rule)."""
    xa = A.astype(np.int64) - 128
    yb = B.astype(np.int64) - 128
    na, nb = len(xa), len(yb)
    if na == 0 or nb == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int64)
    nx = (xa * xa).sum(1)
    ny = (yb * yb).sum(1)
    dot = xa @ yb.T
    e = dot - ((ny + 1) >> 1)[None, :]
    d = nx[:, None] + ny[None, :] - 2 * dot
    # --- rows: group maxima per (tile, lane half), tiles in order, halves merged
    n_t = -(-nb // 32)
    ep = np.full((na, n_t * 32), PAD, np.int64)
    ep[:, :nb] = e
    half = (np.arange(n_t * 32) % 32 >> 2) & 1          # row 8(r/4) + 4h + r%4 of a tile
    tb = np.full((2, na), np.iinfo(np.int64).min)
    ts = tb.copy()
    pos = np.zeros((2, na), np.int64)
    for t in range(n_t):
        cols = np.arange(32 * t, 32 * t + 32)
        for h in range(2):
            m = ep[:, cols[half[cols] == h]].max(1)
            pos[h] = np.where(m > tb[h], t, pos[h])
            ts[h] = np.median(np.stack([ts[h], tb[h], m]), 0).astype(np.int64)
            tb[h] = np.maximum(tb[h], m)
    e1 = np.maximum(tb[0], tb[1])
    e2 = np.maximum(np.minimum(tb[0], tb[1]), np.maximum(ts[0], ts[1]))
    gt = np.where(tb[0] >= tb[1], pos[0], pos[1])
    gh = np.where(tb[0] >= tb[1], 0, 1)
    # --- columns: every train's nearest query (lowest index on ties) proposes (d, j)
    cw = np.argmin(d, 0)                                 # first minimum = lowest query
    Dp = np.full(na, INF)
    Jp = np.zeros(na, np.int64)
    for j in range(nb):                                  # smallest d, then lowest j
        i = cw[j]
        if d[i, j] < Dp[i]:
            Dp[i], Jp[i] = d[i, j], j
    # --- finalize
    out = []

    def row_scan(i):
        o = np.lexsort((np.arange(nb), d[i]))
        j1 = o[0]
        b1 = d[i, j1]
        b2 = d[i, o[1]] if nb > 1 else INF
        if cw[j1] == i and _ratio_ok(b1, b2, ratio):
            out.append((i, j1, b1))

    for i in range(na):
        A_ = nx[i]
        d1lo = max(A_ - 2 * e1[i] - 1, 0)
        d2hi = A_ - 2 * e2[i] if e2[i] > E_VALID else INF
        if not (Dp[i] <= A_ - 2 * e1[i] and _ratio_ok(d1lo, d2hi, ratio)):
            continue
        if e1[i] == e2[i]:
            row_scan(i)
            continue
        g = [32 * gt[i] + 8 * (k >> 2) + 4 * gh[i] + (k & 3) for k in range(16)]
        g = [j for j in g if j < nb]
        ek = np.array([e[i, j] for j in g])
        if int((ek == e1[i]).sum()) != 1:
            row_scan(i)
            continue
        d2g = min([d[i, j] for j, v in zip(g, ek) if v != e1[i]], default=INF)
        o2lo = A_ - 2 * e2[i] - 1 if e2[i] > E_VALID else INF
        o2hi = A_ - 2 * e2[i] if e2[i] > E_VALID else INF
        d1 = Dp[i]
        if _ratio_ok(d1, min(d2g, o2lo), ratio):
            out.append((i, Jp[i], d1))
        elif _ratio_ok(d1, min(d2g, o2hi), ratio):
            row_scan(i)
    out.sort()
    q = np.array([o[0] for o in out], np.int32)
    t = np.array([o[1] for o in out], np.int32)
    dd = np.array([o[2] for o in out], np.int64)
    return q, t, dd


def _sets():
    rng = np.random.default_rng(2024)
    yield "random", rng.integers(0, 256, (180, 128), np.uint8), rng.integers(0, 256, (230, 128), np.uint8)
    lv = lambda n, L: (rng.integers(0, L, (n, 128)) * (255 // (L - 1))).astype(np.uint8)
    yield "ties2", lv(150, 2), lv(200, 2)
    yield "ties3", lv(120, 3), lv(97, 3)
    B = rng.integers(0, 256, (300, 128), np.uint8)
    B[1] = B[0]                     # nearest tie inside one group (same tile, same half)
    B[9] = B[8]
    B[34] = B[2]                    # tie across tiles
    B[3] = B[0] ^ 1                 # runner-up in the best group
    A = rng.integers(0, 256, (64, 128), np.uint8)
    A[:40] = B[:40]
    A[40:50] = B[100:110] ^ 3
    yield "planted", A, B
    yield "ragged33", A, B[:33]
    yield "one_train", A, B[:1]
    near = (B[:60].astype(np.int32) + rng.integers(-3, 4, (60, 128))).clip(0, 255).astype(np.uint8)
    yield "near", near, B
    import synth
    s = synth.make_scene(2, 700, seed=3)
    yield "sift_like", s["desc"][0, :s["n_kp"][0]], s["desc"][1, :s["n_kp"][1] - 5]


@pytest.mark.parametrize("ratio", [(4, 5), (1, 1), (3, 2), (65535, 1), None])
def test_group_rule_equals_oracle(ratio):
    for name, A, B in _sets():
        q, t, d = group_kernel_match(A, B, ratio)
        oq, ot, od = O.match(A, B, metric=0, cross_check=O.XC_MUTUAL, ratio=ratio)
        assert len(q) == len(oq), (name, ratio)
        np.testing.assert_array_equal(q, oq, err_msg=name)
        np.testing.assert_array_equal(t, ot, err_msg=name)
        np.testing.assert_array_equal(d, od, err_msg=name)
