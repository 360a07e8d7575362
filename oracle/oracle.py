"""ctypes front-end of the CPU oracle (oracle/sfm_oracle*.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, and only as the checker / timed CPU baseline — never by the product path under
sfm-project_amd/.  Parity status: "parity unpinned" (see sfm_oracle.c header and DESIGN.md §5).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SFM_ORACLE_LIB: the ASan/UBSan build (oracle/Makefile `sanitize`, tools/oracle_sanitize.sh)
_LIB_PATH = os.environ.get("SFM_ORACLE_LIB") or os.path.join(_HERE, "lib", "liboracle.so")
_lib = None

XC_NONE, XC_MUTUAL, XC_OPENCV = 0, 1, 2
INT64_MAX = np.iinfo(np.int64).max


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _bind(_lib)
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _bind(L):
    vp, i32, i64, u32, u64, f32, f64 = (C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64,
                                        C.c_float, C.c_double)
    L.oracle_match.argtypes = [vp, i32, vp, i32, i32, i32, i32, i32, i32, i64, vp, vp, vp]
    L.oracle_match.restype = i32
    L.oracle_nn_tables.argtypes = [vp, i32, vp, i32, i32, i32, vp, vp, vp, vp, vp]
    L.oracle_philox4x32_10.argtypes = [vp, vp, vp]
    L.oracle_sample8.argtypes = [u64, u32, u32, u32, i32, vp]
    L.oracle_normalize.argtypes = [vp, i32, vp, vp, vp, vp]
    L.oracle_fit_f8.argtypes = [vp, vp, vp]
    L.oracle_fit_f8.restype = i32
    L.oracle_ransac_f.argtypes = [vp, vp, i32, i32, u64, u32, u32, f32, vp, vp, vp, vp]
    L.oracle_ransac_f.restype = i32
    L.oracle_ransac_counts.argtypes = [vp, vp, i32, i32, u64, u32, u32, f32, vp]
    L.oracle_ransac_masks.argtypes = [vp, vp, i32, i32, u64, u32, u32, f32, vp, vp, vp]
    L.oracle_match_verify_batch.argtypes = [vp, vp, i32, i32, i32, vp, i32, i32, i32, i64, i32,
                                            u64, f32, i32, vp, vp, vp, vp, vp, vp, vp]
    L.oracle_match_verify_batch.restype = C.c_longlong
    # fp64 mode of the same spec (sfm_oracle_ransac.inc with R = double)
    L.oracle_normalize_f64.argtypes = [vp, i32, vp, vp, vp, vp]
    L.oracle_fit_f8_f64.argtypes = [vp, vp, vp]
    L.oracle_fit_f8_f64.restype = i32
    L.oracle_ransac_f_f64.argtypes = [vp, vp, i32, i32, u64, u32, u32, f32, vp, vp, vp, vp]
    L.oracle_ransac_f_f64.restype = i32
    L.oracle_ransac_counts_f64.argtypes = [vp, vp, i32, i32, u64, u32, u32, f32, vp]
    L.oracle_ransac_masks_f64.argtypes = [vp, vp, i32, i32, u64, u32, u32, f32, vp, vp, vp]
    L.oracle_match_verify_batch_f64.argtypes = L.oracle_match_verify_batch.argtypes
    L.oracle_match_verify_batch_f64.restype = C.c_longlong
    L.oracle_set_threads.argtypes = [i32]
    L.oracle_get_threads.restype = i32
    L.oracle_ba_obs.argtypes = [vp, vp, vp, vp, f64, vp, vp, vp, vp, vp]
    L.oracle_ba_jtj.argtypes = [i32, vp, vp, i32, vp, i32, vp, vp, vp, f64, vp, vp, vp, vp, vp,
                                vp]
    L.oracle_ba_jtj.restype = f64
    L.oracle_reg_bearing.argtypes = [f64, f64, vp, vp]
    L.oracle_reg_sample3.argtypes = [u64, u32, u32, i32, vp]
    L.oracle_reg_p3p.argtypes = [vp, vp, vp, vp, vp]
    L.oracle_reg_p3p.restype = i32
    L.oracle_reg_ransac.argtypes = [i32, vp, vp, vp, u32, i32, u64, f64, vp, vp, vp, vp]
    L.oracle_reg_ransac.restype = i32
    L.oracle_orb_levels.argtypes = [i32, i32, i32, f64, i32, vp, vp, vp, vp]
    L.oracle_orb_pattern.argtypes = [vp]
    L.oracle_orb_resize.argtypes = [vp, i32, i32, i32, i32, vp]
    L.oracle_orb_blur.argtypes = [vp, i32, i32, vp]
    L.oracle_orb_fast_score.argtypes = [vp, i32, i32, i32]
    L.oracle_orb_fast_score.restype = i32
    L.oracle_orb_harris.argtypes = [vp, i32, i32, i32]
    L.oracle_orb_harris.restype = i64
    L.oracle_orb_moments.argtypes = [vp, i32, i32, i32, vp, vp]
    L.oracle_orb_round_div.argtypes = [i64, i64]
    L.oracle_orb_round_div.restype = i64
    L.oracle_orb.argtypes = [vp, i32, i32, i32, i32, f64, i32, vp, vp, vp]
    L.oracle_orb.restype = i32


def match(A, B, metric=0, cross_check=XC_MUTUAL, ratio=None, max_dist=-1):
    """Returns (query_idx, train_idx, dist) arrays in ascending query order."""
    A = np.ascontiguousarray(A, np.uint8)
    B = np.ascontiguousarray(B, np.uint8)
    num, den = (0, 0) if ratio is None else ratio
    n = max(A.shape[0], 1)
    q = np.zeros(n, np.int32)
    t = np.zeros(n, np.int32)
    d = np.zeros(n, np.int64)
    k = lib().oracle_match(_p(A), A.shape[0], _p(B), B.shape[0], A.shape[1], metric, cross_check,
                           num, den, max_dist, _p(q), _p(t), _p(d))
    return q[:k], t[:k], d[:k]


def nn_tables(A, B, metric=0):
    A = np.ascontiguousarray(A, np.uint8)
    B = np.ascontiguousarray(B, np.uint8)
    Ka, Kb = A.shape[0], B.shape[0]
    nn = np.zeros(Ka, np.int32); d1 = np.zeros(Ka, np.int64); d2 = np.zeros(Ka, np.int64)
    rnn = np.zeros(Kb, np.int32); rd = np.zeros(Kb, np.int64)
    lib().oracle_nn_tables(_p(A), Ka, _p(B), Kb, A.shape[1], metric, _p(nn), _p(d1), _p(d2),
                           _p(rnn), _p(rd))
    return nn, d1, d2, rnn, rd


def philox(ctr, key):
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(o))
    return o


def sample8(seed, pa, pb, h, M):
    o = np.zeros(8, np.int32)
    lib().oracle_sample8(seed, pa, pb, h, M, _p(o))
    return o


def normalize(xy):
    xy = np.ascontiguousarray(xy, np.float32)
    out = np.zeros_like(xy)
    cx, cy, s = C.c_float(), C.c_float(), C.c_float()
    lib().oracle_normalize(_p(xy), xy.shape[0], _p(out), C.byref(cx), C.byref(cy), C.byref(s))
    return out, cx.value, cy.value, s.value


def fit_f8(p1, p2):
    p1 = np.ascontiguousarray(p1, np.float32)
    p2 = np.ascontiguousarray(p2, np.float32)
    F = np.zeros(9, np.float32)
    ok = lib().oracle_fit_f8(_p(p1), _p(p2), _p(F))
    return ok, F


def _rt(f64):
    return (np.float64, "_f64") if f64 else (np.float32, "")


def ransac_f(xy1, xy2, H=4096, seed=42, pa=0, pb=1, thr=1.0, f64=False):
    """Returns dict(count, best_h, F (normalised, 9), norm (6), mask (u8 [M])); f32 spec, or the
    fp64 mode of the same spec with f64=True (coordinates, F and norm in float64)."""
    dt, sfx = _rt(f64)
    xy1 = np.ascontiguousarray(xy1, dt)
    xy2 = np.ascontiguousarray(xy2, dt)
    M = xy1.shape[0]
    bh = np.zeros(1, np.int32)
    F = np.zeros(9, dt)
    nrm = np.zeros(6, dt)
    mask = np.zeros(max(M, 1), np.uint8)
    c = getattr(lib(), "oracle_ransac_f" + sfx)(_p(xy1), _p(xy2), M, H, seed, pa, pb, thr, _p(bh),
                                               _p(F), _p(nrm), _p(mask))
    return dict(count=c, best_h=int(bh[0]), F=F, norm=nrm, mask=mask[:M])


def ransac_counts(xy1, xy2, H=4096, seed=42, pa=0, pb=1, thr=1.0, f64=False):
    dt, sfx = _rt(f64)
    xy1 = np.ascontiguousarray(xy1, dt)
    xy2 = np.ascontiguousarray(xy2, dt)
    counts = np.zeros(H, np.int32)
    getattr(lib(), "oracle_ransac_counts" + sfx)(_p(xy1), _p(xy2), xy1.shape[0], H, seed, pa, pb,
                                                 thr, _p(counts))
    return counts


def ransac_masks(xy1, xy2, H=4096, seed=42, pa=0, pb=1, thr=1.0, f64=False):
    """Per-hypothesis decisions: (masks [H,M] u8, idx [H,8] i32, ok [H] bool)."""
    dt, sfx = _rt(f64)
    xy1 = np.ascontiguousarray(xy1, dt)
    xy2 = np.ascontiguousarray(xy2, dt)
    M = xy1.shape[0]
    masks = np.zeros((H, max(M, 1)), np.uint8)
    idx = np.zeros((H, 8), np.int32)
    ok = np.zeros(H, np.int32)
    getattr(lib(), "oracle_ransac_masks" + sfx)(_p(xy1), _p(xy2), M, H, seed, pa, pb, thr,
                                                _p(masks), _p(idx), _p(ok))
    return masks[:, :M], idx, ok.astype(bool)


def match_verify_batch(desc, kps, pairs, ratio=(4, 5), max_dist=-1, H=4096, seed=42, thr=1.0,
                       min_inl=15, full=False, f64=False):
    """K1 (mutual + ratio) + K2 per pair, OpenMP over pairs.  Returns (total verified inliers,
    n_match [P], n_inl [P]); full=True adds a dict with match [P,K,2] (queryIdx, trainIdx),
    mask [P,K] u8, dist [P,K] i32 (d^2), best_h [P] and F [P,9] f32 (entries past n_match[p]
    are zero; F and best_h are meaningful for pairs with >= 8 matches)."""
    dt, sfx = _rt(f64)
    desc = np.ascontiguousarray(desc, np.uint8)
    kps = np.ascontiguousarray(kps, dt)
    pairs = np.ascontiguousarray(pairs, np.int32)
    P, K = pairs.shape[0], desc.shape[1]
    nm = np.zeros(P, np.int32)
    ni = np.zeros(P, np.int32)
    mt = np.zeros((P, K, 2), np.int32) if full else None
    mk = np.zeros((P, K), np.uint8) if full else None
    bh = np.zeros(P, np.int32) if full else None
    dd = np.zeros((P, K), np.int32) if full else None
    FF = np.zeros((P, 9), dt) if full else None
    nul = C.c_void_p(None)
    tot = getattr(lib(), "oracle_match_verify_batch" + sfx)(_p(desc), _p(kps), desc.shape[0], desc.shape[1],
                                          desc.shape[2], _p(pairs), P, ratio[0], ratio[1],
                                          max_dist, H, seed, thr, min_inl, _p(nm), _p(ni),
                                          _p(mt) if full else nul, _p(mk) if full else nul,
                                          _p(bh) if full else nul, _p(dd) if full else nul,
                                          _p(FF) if full else nul)
    if full:
        return int(tot), nm, ni, dict(match=mt, mask=mk, best_h=bh, dist=dd, F=FF)
    return int(tot), nm, ni


def set_threads(n: int) -> int:
    lib().oracle_set_threads(int(n))
    return lib().oracle_get_threads()


def ba_jtj(cams, pp, pts, cam_idx, pt_idx, uv, loss_s=0.0):
    cams = np.ascontiguousarray(cams, np.float64)
    pp = np.ascontiguousarray(pp, np.float64)
    pts = np.ascontiguousarray(pts, np.float64)
    cam_idx = np.ascontiguousarray(cam_idx, np.int32)
    pt_idx = np.ascontiguousarray(pt_idx, np.int32)
    uv = np.ascontiguousarray(uv, np.float64)
    nc, npt, no = cams.shape[0], pts.shape[0], cam_idx.shape[0]
    U = np.zeros((nc, 8, 8)); V = np.zeros((npt, 3, 3)); W = np.zeros((no, 8, 3))
    gc = np.zeros((nc, 8)); gp = np.zeros((npt, 3)); res = np.zeros((no, 2))
    cost = lib().oracle_ba_jtj(nc, _p(cams), _p(pp), npt, _p(pts), no, _p(cam_idx), _p(pt_idx),
                               _p(uv), loss_s, _p(U), _p(V), _p(W), _p(gc), _p(gp), _p(res))
    return dict(U=U, V=V, W=W, gc=gc, gp=gp, res=res, cost=cost)


# ---- next-view registration (oracle/sfm_oracle_reg.c) ---------------------------------------------

def reg_bearing(xy, intr):
    intr = np.ascontiguousarray(intr, np.float64)
    out = np.zeros((len(xy), 3))
    b = np.zeros(3)
    for i, (x, y) in enumerate(np.asarray(xy, np.float64)):
        lib().oracle_reg_bearing(float(x), float(y), _p(intr), _p(b))
        out[i] = b
    return out


def reg_sample3(seed, img, h, n):
    out = np.zeros(3, np.int32)
    lib().oracle_reg_sample3(seed, img, h, n, _p(out))
    return out


def reg_p3p(b, X):
    b = np.ascontiguousarray(b, np.float64)
    X = np.ascontiguousarray(X, np.float64)
    Rs = np.zeros((4, 9)); ts = np.zeros((4, 3)); ok = np.zeros(4, np.int32)
    lib().oracle_reg_p3p(_p(b), _p(X), _p(Rs), _p(ts), _p(ok))
    return [(Rs[k].reshape(3, 3), ts[k]) if ok[k] else None for k in range(4)]


def reg_ransac(xy, X, intr, img=0, n_hyp=1024, seed=42, thr=4.0):
    """Returns dict(count, key, R [3,3], t [3], mask [n])."""
    xy = np.ascontiguousarray(xy, np.float64)
    X = np.ascontiguousarray(X, np.float64)
    intr = np.ascontiguousarray(intr, np.float64)
    n = len(xy)
    key = np.zeros(1, np.int32)
    R = np.zeros(9); t = np.zeros(3); mask = np.zeros(max(n, 1), np.uint8)
    cnt = lib().oracle_reg_ransac(n, _p(xy), _p(X), _p(intr), img, n_hyp, seed, thr, _p(key),
                                  _p(R), _p(t), _p(mask))
    return dict(count=int(cnt), key=int(key[0]), R=R.reshape(3, 3), t=t, mask=mask[:n])


# ---- ORB extraction spec (oracle/sfm_oracle_orb.c) ----------------------------------------------

def orb(img, nfeat=500, nlevels=8, scale=1.2, fast_thr=20):
    """Returns (kp [n,6] f32 (x, y, size, angle, response, octave), desc [n,32] u8,
    level counts [nlevels])."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    kp = np.zeros((max(nfeat, 1), 6), np.float32)
    desc = np.zeros((max(nfeat, 1), 32), np.uint8)
    lc = np.zeros(nlevels, np.int32)
    n = lib().oracle_orb(_p(img), H, W, nfeat, nlevels, scale, fast_thr, _p(kp), _p(desc), _p(lc))
    return kp[:n], desc[:n], lc


def orb_levels(W, H, nlevels=8, scale=1.2, nfeat=500):
    Wl = np.zeros(nlevels, np.int32); Hl = np.zeros(nlevels, np.int32)
    sc = np.zeros(nlevels); nl = np.zeros(nlevels, np.int32)
    lib().oracle_orb_levels(W, H, nlevels, scale, nfeat, _p(Wl), _p(Hl), _p(sc), _p(nl))
    return Wl, Hl, sc, nl


def orb_pattern():
    pat = np.zeros((256, 4), np.int32)
    lib().oracle_orb_pattern(_p(pat))
    return pat


def orb_resize(img, Hl, Wl):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros((Hl, Wl), np.uint8)
    lib().oracle_orb_resize(_p(img), img.shape[0], img.shape[1], Hl, Wl, _p(out))
    return out


def orb_blur(L):
    L = np.ascontiguousarray(L, np.uint8)
    out = np.zeros_like(L)
    lib().oracle_orb_blur(_p(L), L.shape[0], L.shape[1], _p(out))
    return out


def orb_fast_score(L, x, y):
    L = np.ascontiguousarray(L, np.uint8)
    return int(lib().oracle_orb_fast_score(_p(L), L.shape[1], x, y))


def orb_harris(L, x, y):
    L = np.ascontiguousarray(L, np.uint8)
    return int(lib().oracle_orb_harris(_p(L), L.shape[1], x, y))


def orb_moments(L, x, y):
    L = np.ascontiguousarray(L, np.uint8)
    a, b = C.c_int64(), C.c_int64()
    lib().oracle_orb_moments(_p(L), L.shape[1], x, y, C.byref(a), C.byref(b))
    return a.value, b.value


def orb_round_div(n, R2):
    return int(lib().oracle_orb_round_div(int(n), int(R2)))
