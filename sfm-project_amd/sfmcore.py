"""ctypes binding of libsfmcore.so (include/sfmcore.h) — the only way Python reaches the kernels.

Device memory and streams come from PyTorch-ROCm (plumbing only): arrays are passed as
`tensor.data_ptr()` and every call is enqueued on torch's current HIP stream, so kernels order
correctly with torch copies.  There is no CPU fallback: if the library is missing or the device is
not gfx950 the calls raise `SfmCoreError`.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SFMCORE_LIB: an alternative build of the same library (A/B timing of kernel variants only).
LIB_PATH = os.environ.get("SFMCORE_LIB") or os.path.join(_HERE, "lib", "libsfmcore.so")

METRIC_L2, METRIC_HAMMING = 0, 1
XC_NONE, XC_MUTUAL, XC_OPENCV = 0, 1, 2

EXPORTED = ["sfm_ctx_create", "sfm_ctx_destroy", "sfm_ctx_set_stream", "sfm_ctx_sync",
            "sfm_last_error", "sfm_version", "sfm_match_batch", "sfm_ransac_f_batch",
            "sfm_ba_jtj", "sfm_graph_offsets", "sfm_graph_rows", "sfm_ba_solve", "sfm_ba_cost",
            "sfm_ba_update", "sfm_tracks", "sfm_triangulate", "sfm_register_batch",
            "sfm_ba_fix_params", "sfm_orb_batch", "sfm_ransac_counts", "sfm_ba_solve_stage",
            "sfm_ransac_stats", "sfm_ransac_f_batch_f64", "sfm_graph_rows_packed",
            "sfm_graph_expand", "sfm_match_batch_both", "sfm_ransac_wave_stops",
            "sfm_ba_set_chunks", "sfm_ba_chunk_tree", "sfm_ba_set_schur", "sfm_calib_mfma_i8"]


class SfmCoreError(RuntimeError):
    pass


class MatchParams(C.Structure):
    _fields_ = [("metric", C.c_int32), ("cross_check", C.c_int32), ("ratio_num", C.c_int32),
                ("ratio_den", C.c_int32), ("max_dist", C.c_int64)]


class BaSolveParams(C.Structure):
    _fields_ = [("lam", C.c_double), ("tol", C.c_double), ("max_iter", C.c_int32),
                ("poll", C.c_int32), ("poll_first", C.c_int32)]


class RegisterParams(C.Structure):
    _fields_ = [("n_hyp", C.c_int32), ("refine", C.c_int32), ("thr", C.c_double),
                ("seed", C.c_uint64)]


class OrbParams(C.Structure):
    _fields_ = [("n_features", C.c_int32), ("n_levels", C.c_int32), ("scale_factor", C.c_double),
                ("fast_threshold", C.c_int32), ("_pad", C.c_int32)]


class RansacParams(C.Structure):
    _fields_ = [("n_hyp", C.c_int32), ("min_inliers", C.c_int32), ("thr", C.c_float),
                ("_pad", C.c_int32), ("seed", C.c_uint64)]


# stages of sfm_ba_solve_stage (include/sfmcore.h)
(BA_STAGE_SETUP, BA_STAGE_SETUP_FINISH, BA_STAGE_ITER, BA_STAGE_ITER_FINISH, BA_STAGE_BACKSUB,
 BA_STAGE_MODEL, BA_STAGE_POLL, BA_STAGE_SCHUR) = range(8)
# up to this many cameras ITER_FINISH is one k-free launch (ba_solve.hip FINISH_VEC_MAX_CAM)
BA_FINISH_VEC_MAX_CAM = 1024

_lib = None
_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Loads (building it first if hipcc is present and the .so is missing) libsfmcore.so."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # torch-ROCm ships its own libamdhip64.so.7: load it first so the process has ONE HIP
        # runtime (the dynamic loader then resolves libsfmcore's dependency to it).
        import torch  # noqa: F401
        if not os.path.exists(path):
            if os.path.exists("/opt/rocm/bin/hipcc"):
                from build_lib import build
                build()
            if not os.path.exists(path):
                raise SfmCoreError(f"libsfmcore.so not found at {path}; run __graft_entry__.build()")
        L = C.CDLL(path)
        vp, i32, i64, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_double
        L.sfm_ctx_create.argtypes = [i32, C.POINTER(vp)]
        L.sfm_ctx_destroy.argtypes = [vp]
        L.sfm_ctx_set_stream.argtypes = [vp, vp]
        L.sfm_ctx_sync.argtypes = [vp]
        L.sfm_last_error.restype = C.c_char_p
        L.sfm_version.restype = i32
        L.sfm_match_batch.argtypes = [vp, vp, vp, i32, i32, i32, vp, i32, C.POINTER(MatchParams),
                                      vp, vp, vp]
        L.sfm_match_batch_both.argtypes = L.sfm_match_batch.argtypes
        L.sfm_ransac_f_batch.argtypes = [vp, vp, i32, i32, vp, i32, vp, vp,
                                         C.POINTER(RansacParams), vp, vp, vp, vp, vp]
        L.sfm_ransac_f_batch_f64.argtypes = L.sfm_ransac_f_batch.argtypes
        L.sfm_ransac_counts.argtypes = [vp, vp, i32, i32, vp, i32, vp, vp,
                                        C.POINTER(RansacParams), vp, vp, vp, vp]
        L.sfm_ransac_stats.argtypes = [vp, i32, vp]
        L.sfm_ransac_wave_stops.argtypes = [vp, i32, i32, vp]
        L.sfm_calib_mfma_i8.argtypes = [vp, C.c_float, vp]
        L.sfm_ba_jtj.argtypes = [vp, i32, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, f64, vp,
                                 vp, vp, vp, vp, vp, vp]
        L.sfm_ba_solve.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                   C.POINTER(BaSolveParams), vp, vp, vp]
        L.sfm_ba_solve_stage.argtypes = [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp,
                                         vp, vp, vp, C.POINTER(BaSolveParams), vp, vp, vp, vp, vp]
        L.sfm_ba_cost.argtypes = [vp, i32, vp, vp, i32, vp, i32, vp, vp, vp, f64, vp]
        L.sfm_ba_update.argtypes = [vp, i32, vp, vp, i32, vp, vp, vp, vp]
        L.sfm_ba_fix_params.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp]
        L.sfm_ba_set_chunks.argtypes = [vp, i32, vp, vp, i32, vp]
        L.sfm_ba_set_schur.argtypes = [vp, i32, vp, i32, vp, i32, vp, vp, i32, vp, i32, vp, vp, vp]
        L.sfm_ba_chunk_tree.argtypes = [vp, i32, i64, vp, vp]
        L.sfm_orb_batch.argtypes = [vp, vp, i32, i32, i32, C.POINTER(OrbParams), vp, vp, vp]
        L.sfm_register_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, C.POINTER(RegisterParams),
                                         vp, vp, vp, vp]
        L.sfm_triangulate.argtypes = [vp, i32, vp, vp, i32, vp, vp, vp, vp, vp]
        L.sfm_tracks.argtypes = [vp, i32, vp, i32, vp, i64, vp, i32, vp, vp, vp, vp]
        L.sfm_graph_offsets.argtypes = [vp, i32, vp, i32, vp]
        L.sfm_graph_rows.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, i32, vp, vp]
        L.sfm_graph_rows_packed.argtypes = [vp, i32, i32, vp, vp, vp, vp, i32, vp, vp]
        L.sfm_graph_expand.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp]
        for name in EXPORTED:
            getattr(L, name).restype = getattr(L, name).restype or C.c_int
        _lib = L
        return L


def _check(rc: int):
    if rc != 0:
        msg = load_library().sfm_last_error().decode(errors="replace")
        raise SfmCoreError(f"libsfmcore error {rc}: {msg}")


def _ptr(t) -> int:
    return t.data_ptr()


def _expect(fn: str, *specs):
    """Raise SfmCoreError unless every (name, tensor, dtype, trailing shape) is a contiguous device
    tensor of that dtype whose trailing dimensions match (the kernels index raw pointers)."""
    for name, t, dt, tail in specs:
        ok = t.dtype == dt and t.is_cuda and t.is_contiguous()
        ok = ok and tuple(t.shape[t.dim() - len(tail):]) == tuple(tail) and t.dim() == len(tail) + 1
        if not ok:
            raise SfmCoreError(f"{fn}: {name} must be a contiguous device {dt} tensor of shape "
                               f"[n, {', '.join(map(str, tail))}]" if tail else
                               f"{fn}: {name} must be a contiguous device {dt} vector")


class Context:
    """One per device (not thread-safe).  Calls run on torch's current stream of that device."""

    def __init__(self, device: int = 0):
        import torch
        self.torch = torch
        if not torch.cuda.is_available():
            raise SfmCoreError("no HIP device visible: the sfm core has no CPU fallback")
        self.lib = load_library()
        self.device = device
        h = C.c_void_p()
        _check(self.lib.sfm_ctx_create(device, C.byref(h)))
        self.handle = h
        self._stream = None   # the torch stream last set on the context (_bind_stream)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.sfm_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind_stream(self):
        # only this wrapper sets the context's stream, so an unchanged torch stream is a no-op
        # (sfm_ctx_set_stream returns at once for it) and skips the ctypes call
        s = self.torch.cuda.current_stream(self.device).cuda_stream
        if s != self._stream:
            _check(self.lib.sfm_ctx_set_stream(self.handle, C.c_void_p(s)))
            self._stream = s

    def sync(self):
        _check(self.lib.sfm_ctx_sync(self.handle))

    # ---- matching --------------------------------------------------------------------------
    def match_batch(self, desc, n_kp, pairs, metric=METRIC_L2, cross_check=XC_MUTUAL,
                    ratio=None, max_dist=-1, out=None):
        """desc [n_img,k_max,dim] u8, n_kp [n_img] i32, pairs [P,2] i32 (device tensors).

        Returns (count [P] i32, match [P,k_max,2] i32, dist [P,k_max] i32)."""
        torch = self.torch
        n_img, k_max, dim = desc.shape
        P = pairs.shape[0]
        for t, dt in ((desc, torch.uint8), (n_kp, torch.int32), (pairs, torch.int32)):
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
                raise SfmCoreError("match_batch: expected contiguous device tensors "
                                   "(desc u8, n_kp i32, pairs i32)")
        dev = desc.device
        if out is None:
            out = (torch.empty(P, dtype=torch.int32, device=dev),
                   torch.empty((P, k_max, 2), dtype=torch.int32, device=dev),
                   torch.empty((P, k_max), dtype=torch.int32, device=dev))
        num, den = (0, 0) if ratio is None else ratio
        prm = MatchParams(metric, cross_check, int(num), int(den), int(max_dist))
        self._bind_stream()
        _check(self.lib.sfm_match_batch(self.handle, _ptr(desc), _ptr(n_kp), n_img, k_max, dim,
                                        _ptr(pairs), P, C.byref(prm), _ptr(out[0]), _ptr(out[1]),
                                        _ptr(out[2])))
        return out

    def match_batch_both(self, desc, n_kp, pairs, metric=METRIC_HAMMING, cross_check=XC_OPENCV,
                         max_dist=-1, out=None):
        """Both orders of every pair from one distance tile (sfm_match_batch_both): pairs [P,2]
        (a, b).  Returns (count [2P], match [2P,k_max,2], dist [2P,k_max]): rows p = match_batch
        on (a, b), rows P + p = match_batch on (b, a), bit for bit.  No ratio test."""
        torch = self.torch
        n_img, k_max, dim = desc.shape
        P = pairs.shape[0]
        for t, dt in ((desc, torch.uint8), (n_kp, torch.int32), (pairs, torch.int32)):
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
                raise SfmCoreError("match_batch_both: expected contiguous device tensors "
                                   "(desc u8, n_kp i32, pairs i32)")
        dev = desc.device
        if out is None:
            out = (torch.empty(2 * P, dtype=torch.int32, device=dev),
                   torch.empty((2 * P, k_max, 2), dtype=torch.int32, device=dev),
                   torch.empty((2 * P, k_max), dtype=torch.int32, device=dev))
        prm = MatchParams(metric, cross_check, 0, 0, int(max_dist))
        self._bind_stream()
        _check(self.lib.sfm_match_batch_both(self.handle, _ptr(desc), _ptr(n_kp), n_img, k_max,
                                             dim, _ptr(pairs), P, C.byref(prm), _ptr(out[0]),
                                             _ptr(out[1]), _ptr(out[2])))
        return out

    # ---- feature extraction ----------------------------------------------------------------
    def orb_batch(self, images, n_features=500, n_levels=8, scale_factor=1.2, fast_threshold=20,
                  out=None):
        """images [n_img,H,W] u8 device tensor.  Returns (kp [n_img,n_features,6] f32,
        desc [n_img,n_features,32] u8, count [n_img] i32) device tensors (see sfmcore.h)."""
        torch = self.torch
        if images.dtype != torch.uint8 or not images.is_cuda or not images.is_contiguous():
            raise SfmCoreError("orb_batch: expected a contiguous u8 device tensor [n_img,H,W]")
        n_img, H, W = images.shape
        dev = images.device
        if out is None:
            out = (torch.empty((n_img, n_features, 6), dtype=torch.float32, device=dev),
                   torch.empty((n_img, n_features, 32), dtype=torch.uint8, device=dev),
                   torch.empty(n_img, dtype=torch.int32, device=dev))
        prm = OrbParams(int(n_features), int(n_levels), float(scale_factor), int(fast_threshold), 0)
        self._bind_stream()
        _check(self.lib.sfm_orb_batch(self.handle, _ptr(images), n_img, H, W, C.byref(prm),
                                      _ptr(out[0]), _ptr(out[1]), _ptr(out[2])))
        return out

    # ---- geometric verification ------------------------------------------------------------
    def ransac_batch(self, kps, pairs, count, match, n_hyp=4096, seed=42, thr=1.0,
                     min_inliers=15, out=None):
        """kps [n_img,k_max,2] f32 (the spec) or f64 (the fp64 mode, sfm_ransac_f_batch_f64) +
        the outputs of match_batch.  Returns dict of device tensors: inl_count [P] (-1: fewer
        than 8 matches), best_h [P], mask [P,k_max] u8, F [P,9] (normalised coordinates),
        norm [P,6] (cx1,cy1,s1,cx2,cy2,s2); F and norm in the dtype of kps."""
        torch = self.torch
        n_img, k_max, _ = kps.shape
        P = pairs.shape[0]
        dev = kps.device
        if kps.dtype not in (torch.float32, torch.float64) or not kps.is_contiguous():
            raise SfmCoreError("ransac_batch: kps must be contiguous float32 or float64")
        f64 = kps.dtype == torch.float64
        if out is None:
            out = dict(inl_count=torch.empty(P, dtype=torch.int32, device=dev),
                       best_h=torch.empty(P, dtype=torch.int32, device=dev),
                       mask=torch.empty((P, k_max), dtype=torch.uint8, device=dev),
                       F=torch.empty((P, 9), dtype=kps.dtype, device=dev),
                       norm=torch.empty((P, 6), dtype=kps.dtype, device=dev))
        prm = RansacParams(int(n_hyp), int(min_inliers), float(thr), 0, int(seed))
        self._bind_stream()
        fn = self.lib.sfm_ransac_f_batch_f64 if f64 else self.lib.sfm_ransac_f_batch
        _check(fn(self.handle, _ptr(kps), n_img, k_max, _ptr(pairs), P,
                                           _ptr(count), _ptr(match), C.byref(prm),
                                           _ptr(out["inl_count"]), _ptr(out["best_h"]),
                                           _ptr(out["mask"]), _ptr(out["F"]), _ptr(out["norm"])))
        return out

    def ransac_counts(self, kps, pairs, count, match, n_hyp=4096, seed=42, thr=1.0,
                      hyp_F=False, hyp_mask=False):
        """Diagnostic: the inlier count of every hypothesis ([P, n_hyp] i32 device tensor, -1 for
        degenerate samples / pairs with < 8 matches) and norm [P,6], by the same score path as
        ransac_batch (sfm_ransac_counts); with hyp_F also every hypothesis's F [P, n_hyp, 9] f32
        (normalised coordinates), with hyp_mask every hypothesis's decisions [P, n_hyp, k_max] u8.
        Returns (counts, norm) or (counts, norm, F, mask) (None for what was not asked)."""
        torch = self.torch
        n_img, k_max, _ = kps.shape
        P = pairs.shape[0]
        dev = kps.device
        if kps.dtype != torch.float32 or not kps.is_contiguous():
            raise SfmCoreError("ransac_counts: kps must be contiguous float32")
        counts = torch.empty((P, n_hyp), dtype=torch.int32, device=dev)
        norm = torch.empty((P, 6), dtype=torch.float32, device=dev)
        F = torch.empty((P, n_hyp, 9), dtype=torch.float32, device=dev) if hyp_F else None
        mk = torch.zeros((P, n_hyp, k_max), dtype=torch.uint8, device=dev) if hyp_mask else None
        prm = RansacParams(int(n_hyp), 0, float(thr), 0, int(seed))
        self._bind_stream()
        _check(self.lib.sfm_ransac_counts(self.handle, _ptr(kps), n_img, k_max, _ptr(pairs), P,
                                          _ptr(count), _ptr(match), C.byref(prm), _ptr(counts),
                                          _ptr(norm), _ptr(F) if hyp_F else None,
                                          _ptr(mk) if hyp_mask else None))
        return (counts, norm, F, mk) if (hyp_F or hyp_mask) else (counts, norm)

    def ransac_stats(self, enable=True, read=False):
        """sfm_ransac_stats: enable / disable the execution counters of ransac_batch; with read,
        returns and resets (executed Sampson evaluations, algorithmic = n_hyp x M over pairs with
        M >= 8, number of such pairs) — synchronises the stream."""
        out = (C.c_uint64 * 3)()
        self._bind_stream()
        _check(self.lib.sfm_ransac_stats(self.handle, 1 if enable else 0, out if read else None))
        return (int(out[0]), int(out[1]), int(out[2])) if read else None

    def ransac_wave_stops(self, n_pairs, n_hyp):
        """sfm_ransac_wave_stops: [n_pairs, n_hyp / 64] u32 numpy array, the last counted batch's
        matches scored past the preview per score wave (synchronises the stream)."""
        out = np.zeros((n_pairs, n_hyp // 64), np.uint32)
        self._bind_stream()
        _check(self.lib.sfm_ransac_wave_stops(self.handle, int(n_pairs), int(n_hyp),
                                              out.ctypes.data_as(C.c_void_p)))
        return out

    def calib_mfma_i8(self, target_ms=200.0):
        """sfm_calib_mfma_i8: the device's i8 MFMA ceiling right now — dict(ms, tops, clock_ghz,
        frac_nominal) of an MFMA-only launch of about target_ms on every CU (synchronises)."""
        out = np.zeros(4, np.float64)
        self._bind_stream()
        _check(self.lib.sfm_calib_mfma_i8(self.handle, float(target_ms),
                                          out.ctypes.data_as(C.c_void_p)))
        return {"ms": float(out[0]), "tops": float(out[1]), "clock_ghz": float(out[2]),
                "frac_nominal": float(out[3])}

    # ---- verified match graph --------------------------------------------------------------
    def graph_rows(self, pair_base, count, match, inl_count, mask, min_inliers=15,
                   return_offsets=False, packed=False):
        """Rows [n,3] i32 (pair_base + pair, queryIdx, trainIdx) of the inliers of every verified
        pair (inl_count >= min_inliers), pair-major, ascending match index.  One device->host
        read of the row total sizes the output.  return_offsets: also the [P+1] i64 row offsets
        per pair.  packed: the exchange form instead, [n] i32 rows queryIdx << 16 | trainIdx
        (sfm_graph_rows_packed; pair_base is then implied by the caller's pair range)."""
        torch = self.torch
        P, k_max = mask.shape
        dev = mask.device
        offs = torch.empty(P + 1, dtype=torch.int64, device=dev)
        self._bind_stream()
        _check(self.lib.sfm_graph_offsets(self.handle, P, _ptr(inl_count), int(min_inliers),
                                          _ptr(offs)))
        n = int(offs[P].item())
        rows = torch.empty((n,) if packed else (n, 3), dtype=torch.int32, device=dev)
        if n and packed:
            _check(self.lib.sfm_graph_rows_packed(self.handle, P, k_max, _ptr(count),
                                                  _ptr(match), _ptr(mask), _ptr(inl_count),
                                                  int(min_inliers), _ptr(offs), _ptr(rows)))
        elif n:
            _check(self.lib.sfm_graph_rows(self.handle, P, k_max, int(pair_base), _ptr(count),
                                           _ptr(match), _ptr(mask), _ptr(inl_count),
                                           int(min_inliers), _ptr(offs), _ptr(rows)))
        return (rows, offs) if return_offsets else rows

    def graph_expand(self, pair_base, counts, src_offsets, dst_offsets, packed, n_rows):
        """[n_rows,3] i32 rows (pair_base + p, q, t) from packed rows (sfm_graph_expand): pair p's
        counts[p] rows start at packed[src_offsets[p]] and land at row dst_offsets[p]."""
        torch = self.torch
        dev = packed.device
        rows = torch.empty((n_rows, 3), dtype=torch.int32, device=dev)
        P = counts.shape[0]
        if P and n_rows:
            self._bind_stream()
            _check(self.lib.sfm_graph_expand(self.handle, P, int(pair_base), _ptr(counts),
                                             _ptr(src_offsets), _ptr(dst_offsets), _ptr(packed),
                                             _ptr(rows)))
        return rows

    # ---- bundle adjustment -----------------------------------------------------------------
    # ---- BA chunk mode (sfm_ba_set_chunks): sharding-invariant sums -----------------------------
    def ba_set_chunks(self, spec=None):
        """spec = BAChunks (reconstruction.py) or None (off).  Applies to the next BA calls."""
        if spec is None:
            _check(self.lib.sfm_ba_set_chunks(self.handle, 0, None, None, 0, None))
            return
        args = getattr(spec, "_cargs", None)   # the ctypes arrays, built once per spec
        if args is None:
            n = len(spec.chunk_pt) - 1
            args = spec._cargs = (n, (C.c_int32 * (n + 1))(*[int(v) for v in spec.chunk_pt]),
                                  (C.c_int32 * (n + 1))(*[int(v) for v in spec.chunk_obs]),
                                  int(spec.n_total), _ptr(spec.cam_bounds))
        _check(self.lib.sfm_ba_set_chunks(self.handle, *args))

    def ba_set_schur(self, spec=None):
        """spec = reconstruction.SchurSpec (the explicit reduced camera system's structure) or None
        (off).  Applies to the next BA solves (sfm_ba_set_schur; needs chunk mode)."""
        if spec is None:
            _check(self.lib.sfm_ba_set_schur(self.handle, 0, None, 0, None, 0, None, None, 0, None,
                                             0, None, None, None))
            return
        _check(self.lib.sfm_ba_set_schur(self.handle, spec.n_slot, _ptr(spec.slot_cam), spec.n_seg,
                                         _ptr(spec.seg), spec.n_inst, _ptr(spec.inst),
                                         _ptr(spec.row_ptr), spec.n_ent, _ptr(spec.row_ent),
                                         spec.n_group, _ptr(spec.sg_ptr), _ptr(spec.sg),
                                         _ptr(spec.gk)))

    def ba_chunk_tree(self, parts, out=None):
        """sfm_ba_chunk_tree: parts [n_total, ...] f64 device -> out [...] (the canonical tree)."""
        torch = self.torch
        parts = parts.contiguous()
        nt = parts.shape[0]
        if out is None:
            out = torch.empty(parts.shape[1:], dtype=torch.float64, device=parts.device)
        self._bind_stream()
        _check(self.lib.sfm_ba_chunk_tree(self.handle, nt, int(out.numel()), _ptr(parts),
                                          _ptr(out)))
        return out

    def ba_jtj(self, cams, pp, pts, cam_idx, pt_idx, uv, pt_ptr, cam_ptr, cam_obs, loss_s=0.0,
               n_slot=None):
        """n_slot: chunk mode of a shard (export form) — U [n_slot, n_cam, 8, 8], gc [n_slot, n_cam, 8],
        cost [n_slot] chunk partials (sfm_ba_set_chunks)."""
        torch = self.torch
        dev = cams.device
        nc, npt, no = cams.shape[0], pts.shape[0], cam_idx.shape[0]
        f64 = torch.float64
        lead = () if n_slot is None else (n_slot,)
        U = torch.empty(lead + (nc, 8, 8), dtype=f64, device=dev)
        V = torch.empty((npt, 3, 3), dtype=f64, device=dev)
        W = torch.empty((no, 8, 3), dtype=f64, device=dev)
        gc = torch.empty(lead + (nc, 8), dtype=f64, device=dev)
        gp = torch.empty((npt, 3), dtype=f64, device=dev)
        res = torch.empty((no, 2), dtype=f64, device=dev)
        cost = torch.empty(max(n_slot or 1, 1), dtype=f64, device=dev)
        self._bind_stream()
        _check(self.lib.sfm_ba_jtj(self.handle, nc, _ptr(cams), _ptr(pp), npt, _ptr(pts), no,
                                   _ptr(cam_idx), _ptr(pt_idx), _ptr(uv), _ptr(pt_ptr),
                                   _ptr(cam_ptr), _ptr(cam_obs), float(loss_s), _ptr(U), _ptr(V),
                                   _ptr(W), _ptr(gc), _ptr(gp), _ptr(res), _ptr(cost)))
        return dict(U=U, V=V, W=W, gc=gc, gp=gp, res=res, cost=cost)

    def tracks(self, img_base, pairs, rows, min_len=2):
        """Tracks of a verified match graph (device tensors): img_base [n_img+1] i32,
        pairs [P,2] i32, rows [n,3] i32.  Returns (track_ptr [T+1], track_img [n], track_kp [n])
        device i32 tensors, trimmed to the T tracks."""
        torch = self.torch
        dev = img_base.device
        n_img = img_base.shape[0] - 1
        n_nodes = int(img_base[-1].item()) if n_img > 0 else 0
        cap = max(n_nodes, 1)
        nt = torch.zeros(1, dtype=torch.int32, device=dev)
        ptr = torch.zeros(cap + 1, dtype=torch.int32, device=dev)
        ti = torch.empty(cap, dtype=torch.int32, device=dev)
        tk = torch.empty(cap, dtype=torch.int32, device=dev)
        self._bind_stream()
        _check(self.lib.sfm_tracks(self.handle, n_img, _ptr(img_base), pairs.shape[0],
                                   _ptr(pairs) if pairs.numel() else None, rows.shape[0],
                                   _ptr(rows) if rows.numel() else None, int(min_len), _ptr(nt),
                                   _ptr(ptr), _ptr(ti), _ptr(tk)))
        T = int(nt.item())
        total = int(ptr[T].item())
        return ptr[:T + 1], ti[:total], tk[:total]

    def register_batch(self, corr_ptr, xy, X, intr, img_id, n_hyp=1024, thr=4.0, seed=42,
                       refine=True):
        """P3P RANSAC + refinement for a batch of images (device tensors, see
        include/sfmcore.h).  Returns (cams [n_img,8] f64, count, key [n_img] i32, mask [n] u8)."""
        torch = self.torch
        dev = xy.device
        n_img = corr_ptr.shape[0] - 1
        n = xy.shape[0]
        _expect("register_batch", ("corr_ptr", corr_ptr, torch.int32, ()),
                ("xy", xy, torch.float64, (2,)), ("X", X, torch.float64, (3,)),
                ("intr", intr, torch.float64, (4,)), ("img_id", img_id, torch.int32, ()))
        if X.shape[0] != n or intr.shape[0] != n_img or img_id.shape[0] != n_img:
            raise SfmCoreError("register_batch: xy / X and intr / img_id / corr_ptr sizes differ")
        cams = torch.empty((max(n_img, 0), 8), dtype=torch.float64, device=dev)
        count = torch.empty(max(n_img, 0), dtype=torch.int32, device=dev)
        key = torch.empty(max(n_img, 0), dtype=torch.int32, device=dev)
        mask = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        prm = RegisterParams(int(n_hyp), 1 if refine else 0, float(thr), int(seed))
        self._bind_stream()
        _check(self.lib.sfm_register_batch(self.handle, n_img, _ptr(corr_ptr), _ptr(xy), _ptr(X),
                                           _ptr(intr), _ptr(img_id), C.byref(prm), _ptr(cams),
                                           _ptr(count), _ptr(key), _ptr(mask)))
        return cams, count, key, mask[:n]

    def triangulate(self, cams, pp, pt_ptr, cam_idx, uv):
        """(pts [n_pt,3], stats [n_pt,4]) f64 device tensors; see include/sfmcore.h."""
        torch = self.torch
        n_pt = pt_ptr.shape[0] - 1
        _expect("triangulate", ("cams", cams, torch.float64, (8,)), ("pp", pp, torch.float64, (2,)),
                ("pt_ptr", pt_ptr, torch.int32, ()), ("cam_idx", cam_idx, torch.int32, ()),
                ("uv", uv, torch.float64, (2,)))
        if pp.shape[0] != cams.shape[0] or uv.shape[0] != cam_idx.shape[0]:
            raise SfmCoreError("triangulate: cams / pp or cam_idx / uv sizes differ")
        pts = torch.empty((max(n_pt, 0), 3), dtype=torch.float64, device=cams.device)
        stats = torch.empty((max(n_pt, 0), 4), dtype=torch.float64, device=cams.device)
        self._bind_stream()
        _check(self.lib.sfm_triangulate(self.handle, cams.shape[0], _ptr(cams), _ptr(pp), n_pt,
                                        _ptr(pt_ptr), _ptr(cam_idx), _ptr(uv), _ptr(pts),
                                        _ptr(stats)))
        return pts, stats

    def ba_solve(self, lin, cam_idx, pt_idx, pt_ptr, cam_ptr, cam_obs, lam, max_iter=100,
                 tol=1e-10, out=None, poll=8, poll_first=0):
        """Damped Schur-complement PCG step from the ba_jtj blocks `lin`; returns
        (dc [n_cam,8], dp [n_pt,3], info [5] f64 device tensor).  poll: convergence poll period
        in CG iterations (one host sync each; <= 0 = none, fully asynchronous / graph-capturable);
        poll_first > 0: the first poll at that iteration; see include/sfmcore.h."""
        torch = self.torch
        U = lin["U"]
        dev = U.device
        nc, npt, no = U.shape[0], lin["V"].shape[0], cam_idx.shape[0]
        if out is None:
            f64 = torch.float64
            out = (torch.empty((nc, 8), dtype=f64, device=dev),
                   torch.empty((npt, 3), dtype=f64, device=dev),
                   torch.empty(5, dtype=f64, device=dev))
        dc, dp, info = out
        # C ABI: poll 0 = every SFM_BA_POLL_DEFAULT, < 0 = never; here poll <= 0 = never
        prm = BaSolveParams(float(lam), float(tol), int(max_iter), int(poll) if poll > 0 else -1,
                            max(int(poll_first), 0))
        self._bind_stream()
        _check(self.lib.sfm_ba_solve(self.handle, nc, npt, no, _ptr(cam_idx), _ptr(pt_idx),
                                     _ptr(pt_ptr), _ptr(cam_ptr), _ptr(cam_obs), _ptr(U),
                                     _ptr(lin["V"]), _ptr(lin["W"]), _ptr(lin["gc"]),
                                     _ptr(lin["gp"]), C.byref(prm), _ptr(dc), _ptr(dp),
                                     _ptr(info)))
        return dc, dp, info

    def ba_solve_sharded(self, lin, cam_idx, pt_idx, pt_ptr, cam_ptr, cam_obs, lam, allreduce,
                         max_iter=100, tol=1e-10, out=None, poll=8, graph=False, chunks=None,
                         schur=None, poll_first=0):
        """ba_solve on this rank's point shard (lin: ba_jtj of the shard with U / gc already
        all-reduced), driving sfm_ba_solve_stage: allreduce(t) sums the f64 device tensor t over
        all ranks in place, ordered on the current stream (reconstruction.make_allreduce).
        graph: replay the CG windows between polls as one HIP graph captured on the first
        window after k = 0 (needs allreduce.graph_safe, i.e. RCCL; the capture costs about as much
        as the launches it saves within one solve, profiles/r03/ba_sharded_ab.txt, so it is off
        by default).  poll_first > 0: the first poll at that iteration (ba_solve).  Returns
        (dc, dp, info) like ba_solve."""
        torch = self.torch
        U = lin["U"]
        dev = U.device
        nc, npt, no = U.shape[0], lin["V"].shape[0], cam_idx.shape[0]
        if out is None:
            f64 = torch.float64
            out = (torch.empty((nc, 8), dtype=f64, device=dev),
                   torch.empty((npt, 3), dtype=f64, device=dev),
                   torch.empty(5, dtype=f64, device=dev))
        dc, dp, info = out
        # chunk mode (chunks = reconstruction.BAChunks of a shard, set on this context): every
        # exchange is an all-reduce of a zero-filled [n_total] slot buffer in which this rank
        # fills only its own chunks' slots — an exact all-gather (x + 0 = x), so the stages after
        # it see every chunk's partial bit for bit, in chunk order
        nt = chunks.n_total if chunks is not None else 1
        k0 = chunks.k0 if chunks is not None else 0
        # explicit S (schur = reconstruction.SchurSpec, set on this context): SETUP's 44-sum
        # partials, then SCHUR's group partials of T [n_group][64] behind them, ONE exchange; the
        # CG iterations then run on every rank from the replicated S with no exchange
        ns = schur.n_slot if schur is not None else 0
        n_setup = nt * 44 * nc
        comm = torch.zeros(n_setup + (64 * schur.n_group if ns else 0), dtype=torch.float64,
                           device=dev)
        prm = BaSolveParams(float(lam), float(tol), int(max_iter), int(poll))
        done = C.c_int32(0)
        cptr = comm.data_ptr()

        def args(off=0):
            return (nc, npt, no, _ptr(cam_idx), _ptr(pt_idx), _ptr(pt_ptr), _ptr(cam_ptr),
                    _ptr(cam_obs), _ptr(U), _ptr(lin["V"]), _ptr(lin["W"]), _ptr(lin["gc"]),
                    _ptr(lin["gp"]), C.byref(prm), C.c_void_p(cptr + 8 * off), _ptr(dc), _ptr(dp),
                    _ptr(info), C.byref(done))
        a_base = args()
        a_setup, a_iter, a_back = args(k0 * 44 * nc), args(k0 * 8 * nc), args(k0 * 2)
        self._bind_stream()

        def stage(s, k=0, a=a_base):
            _check(self.lib.sfm_ba_solve_stage(self.handle, s, k, *a))

        def produce(s, n, a, k=0):   # a producing stage, then the exchange of its n doubles
            if chunks is not None:
                comm[:n].zero_()
            stage(s, k, a)
            allreduce(comm[:n])
        if ns:
            comm.zero_()
            stage(BA_STAGE_SETUP, 0, a_setup)
            stage(BA_STAGE_SCHUR, 0, args(n_setup + 64 * schur.g0))
            allreduce(comm)
        else:
            produce(BA_STAGE_SETUP, n_setup, a_setup)
        stage(BA_STAGE_SETUP_FINISH)
        every = poll
        # windows of `poll` iterations between host polls.  With a capturable collective (RCCL)
        # every window after the first replays one HIP graph of its launches and all-reduces:
        # the iteration kernels depend on k only through its parity and k > 0 (the one-launch
        # finish counts iterations itself), so a window captured at k = poll replays at any
        # k = m·poll, poll even.
        graph = (graph and not ns and getattr(allreduce, "graph_safe", False) and every > 0
                 and every % 2 == 0 and nc <= BA_FINISH_VEC_MAX_CAM)
        win = every if every > 0 else max(max_iter, 1)
        # the first window ends at poll_first (then every `win`: the windows after it start at
        # k = poll_first + m·win, one parity when win is even, so the graph replay holds)
        win0 = int(poll_first) if every > 0 and poll_first > 0 else win
        g = None
        k = 0
        while k < max_iter:
            if every > 0 and k > 0:
                stage(BA_STAGE_POLL)   # the same decision on every rank (replicated state)
                if done.value:
                    break
            n = min(win0 if k == 0 else win, max_iter - k)
            if graph and k > 0 and n == win:
                if g is None:
                    g = torch.cuda.CUDAGraph()
                    cap = torch.cuda.Stream(dev)
                    cap.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(cap):
                        self._bind_stream()
                        g.capture_begin()
                        try:
                            for j in range(n):
                                produce(BA_STAGE_ITER, nt * 8 * nc, a_iter, k + j)
                                stage(BA_STAGE_ITER_FINISH, k + j)
                        finally:
                            g.capture_end()
                    torch.cuda.current_stream(dev).wait_stream(cap)
                    self._bind_stream()
                g.replay()
            elif ns:
                for j in range(k, k + n):   # replicated S: nothing to exchange
                    stage(BA_STAGE_ITER, j)
            else:
                for j in range(k, k + n):
                    produce(BA_STAGE_ITER, nt * 8 * nc, a_iter, j)
                    stage(BA_STAGE_ITER_FINISH, j)
            k += n
        produce(BA_STAGE_BACKSUB, nt * 2, a_back)
        stage(BA_STAGE_MODEL)
        return dc, dp, info

    def ba_fix_params(self, lin, cam_idx, fixed):
        """In place on ba_jtj's blocks `lin` (U, W, gc): hold the parameters marked in fixed
        [n_cam,8] u8 device tensor (see include/sfmcore.h sfm_ba_fix_params).  Returns lin."""
        U = lin["U"]
        nc, no = U.shape[0], cam_idx.shape[0]
        self._bind_stream()
        _check(self.lib.sfm_ba_fix_params(self.handle, nc, no, _ptr(cam_idx), _ptr(fixed),
                                          _ptr(U), _ptr(lin["W"]), _ptr(lin["gc"])))
        return lin

    def ba_cost(self, cams, pp, pts, cam_idx, pt_idx, uv, loss_s=0.0, out=None, n_slot=None):
        torch = self.torch
        cost = out if out is not None else torch.empty(max(n_slot or 1, 1), dtype=torch.float64,
                                                       device=cams.device)
        self._bind_stream()
        _check(self.lib.sfm_ba_cost(self.handle, cams.shape[0], _ptr(cams), _ptr(pp),
                                    pts.shape[0], _ptr(pts), cam_idx.shape[0], _ptr(cam_idx),
                                    _ptr(pt_idx), _ptr(uv), float(loss_s), _ptr(cost)))
        return cost

    def ba_update(self, cams, dc, pts, dp, out=None):
        """(cams ⊕ dc, pts + dp), out of place."""
        torch = self.torch
        if out is None:
            out = (torch.empty_like(cams), torch.empty_like(pts))
        co, po = out
        self._bind_stream()
        _check(self.lib.sfm_ba_update(self.handle, cams.shape[0], _ptr(cams), _ptr(dc),
                                      pts.shape[0], _ptr(pts), _ptr(dp), _ptr(co), _ptr(po)))
        return co, po


_ctx_cache: dict = {}


def context(device: int = 0) -> Context:
    ctx = _ctx_cache.get(device)
    if ctx is None:
        ctx = Context(device)
        _ctx_cache[device] = ctx
    return ctx


def csr_by_device(index, n: int):
    """csr_by on a device tensor (torch's stable sort on the GPU): the same (ptr, order) as
    csr_by, int32 device tensors, without a host sort of every observation (and without a host
    sync: the counts are an index_add into n slots, not a bincount sized by the maximum)."""
    import torch
    idx = index.long()
    order = torch.argsort(idx, stable=True).to(torch.int32)
    return csr_ptr_device(idx, n), order


def csr_ptr_device(index, n: int, ascending: bool = False):
    """The CSR offsets [n + 1] (int32 device) of the values 0..n-1 of a device index tensor, with no
    host sync; ascending=True (index non-decreasing): a searchsorted instead of a count."""
    import torch
    idx = index.long()
    dev = index.device
    if ascending:
        return torch.searchsorted(idx, torch.arange(n + 1, dtype=torch.int64, device=dev)).to(torch.int32)
    cnt = torch.zeros(n, dtype=torch.int64, device=dev)
    cnt.index_add_(0, idx, torch.ones_like(idx))
    ptr = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    ptr[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    return ptr


def csr_by(index: np.ndarray, n: int):
    """CSR (ptr [n+1], order) grouping positions of `index` by value, stable."""
    order = np.argsort(index, kind="stable").astype(np.int32)
    ptr = np.zeros(n + 1, np.int32)
    np.cumsum(np.bincount(index, minlength=n), out=ptr[1:])
    return ptr, order
