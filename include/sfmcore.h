/*
 * sfmcore.h — C-ABI of the MI355X matching / geometric-verification / BA-J^TJ core.
 *
 * This is the drop-in boundary behind the reference's Python call signatures.
 * The reference has no FFI of its own: its arithmetic is OpenCV, reached by star-import
 * (code/pipeline.py:1-3).  Each entry point below names the reference interface it replaces;
 * INTEGRATION.md shows the ctypes binding (sfm-project_amd/sfmcore.py) that the reference-side
 * modules feature_matching / geometric_verification / 3d_reconstruction call through.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Every array argument is a DEVICE pointer (hipMalloc'd or a
 *     torch.cuda tensor's data_ptr), C-contiguous, caller-owned.
 *   - Work is enqueued on the context's stream: a non-blocking stream the context creates, until
 *     sfm_ctx_set_stream selects another (NULL selects the legacy default stream, which is what
 *     torch's default stream is).  Entry points return after enqueueing; sfm_ctx_sync waits.
 *   - Return 0 (SFM_OK) on success, < 0 on error; sfm_last_error() gives a thread-local message.
 *     No C++ exception crosses the ABI.  No callbacks.
 *   - A context is bound to one device and must not be used from two threads at once.
 */
#ifndef SFMCORE_H
#define SFMCORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFM_OK 0
#define SFM_ERR_INVALID (-1)     /* bad argument (shape, null pointer, unsupported combination) */
#define SFM_ERR_HIP (-2)         /* HIP runtime error (message in sfm_last_error) */
#define SFM_ERR_NOMEM (-3)       /* device workspace allocation failed */

#define SFM_METRIC_L2 0          /* u8 x 128 (SIFT-like), squared Euclidean distance */
#define SFM_METRIC_HAMMING 1     /* u8 x 32 (ORB 256-bit), Hamming distance */

#define SFM_XC_NONE 0            /* no cross check */
#define SFM_XC_MUTUAL 1          /* strict mutual nearest neighbours, lowest index on ties */
#define SFM_XC_OPENCV 2          /* OpenCV batchDistance cross-check rule (BFMatcher crossCheck) */

typedef struct sfm_ctx sfm_ctx;

typedef struct sfm_match_params {
    int32_t metric;        /* SFM_METRIC_* */
    int32_t cross_check;   /* SFM_XC_* */
    int32_t ratio_num;     /* Lowe ratio r = num/den on (unsquared) distances; den = 0: off */
    int32_t ratio_den;
    int64_t max_dist;      /* keep distance < max_dist (d^2 for L2, bits for Hamming); < 0: off */
} sfm_match_params;

typedef struct sfm_ransac_params {
    int32_t n_hyp;         /* hypotheses per pair (multiple of 256) */
    int32_t min_inliers;   /* pair verified iff best count >= min_inliers */
    float thr;             /* Sampson-error threshold in squared pixels */
    int32_t _pad;
    uint64_t seed;         /* RANSAC seed; hypothesis h of pair (a,b) uses Philox key=seed,
                              counter=(h, 0|1, a, b): results are shard-invariant */
} sfm_ransac_params;

/* ---- context ---------------------------------------------------------------------------- */
int sfm_ctx_create(int32_t device, sfm_ctx** out);
int sfm_ctx_destroy(sfm_ctx* ctx);
int sfm_ctx_set_stream(sfm_ctx* ctx, void* hip_stream);   /* hipStream_t; NULL = default stream */
int sfm_ctx_sync(sfm_ctx* ctx);
const char* sfm_last_error(void);
int32_t sfm_version(void);

/* ---- matching -----------------------------------------------------------------------------
 * Replaces cv2.BFMatcher(normType, crossCheck).match(des1, des2) + the distance filter of
 * code/feature_matching.py:48-58 (extract_and_match, called per ordered pair from
 * code/pipeline.py:41), batched over a pair list.
 *   desc      [n_img][k_max][dim] u8  (dim = 128 for L2, 32 for Hamming)
 *   n_kp      [n_img] i32             valid descriptors per image (<= k_max)
 *   pairs     [n_pairs][2] i32        (query image a, train image b)
 *   out_count [n_pairs] i32           matches per pair
 *   out_match [n_pairs][k_max][2] i32 (queryIdx, trainIdx), ascending queryIdx
 *   out_dist  [n_pairs][k_max] i32    d^2 (L2) or Hamming distance
 * Limits: k_max <= 8192.  L2 above 4096 needs a cross-check rule (SFM_XC_MUTUAL / SFM_XC_OPENCV:
 * the column-winner kernel); the ratio-only and no-rule L2 paths stop at 4096.  Hamming above
 * 4096 runs the VALU popcount kernel.
 */
int sfm_match_batch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                    int32_t k_max, int32_t dim, const int32_t* pairs, int32_t n_pairs,
                    const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                    int32_t* out_dist);
/* Both orders of every pair from one distance tile: the reference enumerates ORDERED pairs i != j
 * (code/pipeline.py:38-41) and matches each with BFMatcher(crossCheck=True)
 * (code/feature_matching.py:48-50); (a, b) and (b, a) share every distance.  pairs [n_pairs][2]
 * (a, b); outputs hold 2 * n_pairs results: slot p = sfm_match_batch on (a, b), slot n_pairs + p =
 * sfm_match_batch on (b, a), bit for bit (out_count [2 n_pairs], out_match [2 n_pairs][k_max][2],
 * out_dist [2 n_pairs][k_max]).  Any cross_check rule and max_dist; no ratio test (ratio_den
 * must be 0: the reverse direction's ratio needs its own second-best neighbour); k_max <= 4096. */
int sfm_match_batch_both(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                         int32_t k_max, int32_t dim, const int32_t* pairs, int32_t n_pairs,
                         const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                         int32_t* out_dist);

/* ---- geometric verification -----------------------------------------------------------------
 * Fills the empty code/geometric_verification.py (placeholder comment at code/pipeline.py:60):
 * 8-point fundamental-matrix RANSAC per pair on the tentative matches of sfm_match_batch.
 *   kps           [n_img][k_max][2] f32 pixel coordinates
 *   match_count / matches: as written by sfm_match_batch
 *   out_inl_count [n_pairs] i32  best inlier count (-1 if fewer than 8 matches)
 *   out_best_h    [n_pairs] i32  winning hypothesis id (lowest id among equal counts)
 *   out_mask      [n_pairs][k_max] u8  inlier flag per tentative match
 *   out_F         [n_pairs][9] f32  F in normalised coordinates (row-major)
 *   out_norm      [n_pairs][6] f32  (cx1, cy1, s1, cx2, cy2, s2) normalisation of each side
 */
int sfm_ransac_f_batch(sfm_ctx* ctx, const float* kps, int32_t n_img, int32_t k_max,
                       const int32_t* pairs, int32_t n_pairs, const int32_t* match_count,
                       const int32_t* matches, const sfm_ransac_params* prm,
                       int32_t* out_inl_count, int32_t* out_best_h, uint8_t* out_mask,
                       float* out_F, float* out_norm);

/* fp64 mode of sfm_ransac_f_batch (SURVEY.md §8b's f64 coordinates / F): the same spec, sampler,
 * schedule and outputs with every floating-point operation of normalisation, 8-point fit, rank-2
 * step and Sampson test in double (the oracle's *_f64 restatement is bit-identical).  kps
 * [n_img][k_max][2] f64; out_F [n_pairs][9] f64; out_norm [n_pairs][6] f64; the ordered schedule
 * only (SFM_RANSAC_MODE is ignored).
 */
int sfm_ransac_f_batch_f64(sfm_ctx* ctx, const double* kps, int32_t n_img, int32_t k_max,
                           const int32_t* pairs, int32_t n_pairs, const int32_t* match_count,
                           const int32_t* matches, const sfm_ransac_params* prm,
                           int32_t* out_inl_count, int32_t* out_best_h, uint8_t* out_mask,
                           double* out_F, double* out_norm);

/* Diagnostic companion of sfm_ransac_f_batch: the inlier count of EVERY hypothesis (no pruning),
 * out_counts [n_pairs][n_hyp] i32 (-1: degenerate sample or fewer than 8 matches), computed by the
 * score kernel of sfm_ransac_f_batch with pruning off; out_norm as above.  Optional (NULL: not
 * written): out_hyp_F [n_pairs][n_hyp][9] f32, every hypothesis's F in normalised coordinates;
 * out_hyp_mask [n_pairs][n_hyp][k_max] u8, every hypothesis's inlier decision per match.  The
 * exhaustive parity tests compare them with the oracle's and with scikit-image's estimates.
 */
int sfm_ransac_counts(sfm_ctx* ctx, const float* kps, int32_t n_img, int32_t k_max,
                      const int32_t* pairs, int32_t n_pairs, const int32_t* match_count,
                      const int32_t* matches, const sfm_ransac_params* prm, int32_t* out_counts,
                      float* out_norm, float* out_hyp_F, uint8_t* out_hyp_mask);

/* Execution statistics of sfm_ransac_f_batch (measurement, default off).  enable != 0: every later
 * batch on ctx adds its Sampson evaluations to device counters (one u32 store per score wave + a
 * small reduction kernel on the context's stream).  out != NULL: synchronises the stream, writes
 * (executed evaluations, algorithmic evaluations = n_hyp x M summed over pairs with M >= 8, number
 * of such pairs) and resets the counters.  executed / algorithmic is the share of the Sampson work
 * the exact pruning did not skip.
 */
int sfm_ransac_stats(sfm_ctx* ctx, int32_t enable, uint64_t* out);
/* Diagnostic companion of sfm_ransac_stats: the last counted sfm_ransac_f_batch{,_f64} batch's
 * per-wave counts (host out [n_pairs][n_hyp / 64] u32: matches the score wave scored past the
 * preview; entries of pairs with < 8 matches are undefined).  n_pairs / n_hyp must equal that
 * batch's; no other sfm_* call on ctx in between (the counts live in its workspace).
 * Synchronises the stream.  executed = Σ_{M>=8} n_hyp·min(128, M) + 64·Σ_w out[p][w] + M. */
int sfm_ransac_wave_stops(sfm_ctx* ctx, int32_t n_pairs, int32_t n_hyp, uint32_t* out);

/* ---- verified match graph -------------------------------------------------------------------
 * Replaces the pair_matches list of code/pipeline.py:42-47 (Pair(img_inx_1, img_inx_2, matches)
 * for every non-empty pair) for a batch: rows (pair_base + pair, queryIdx, trainIdx) of the RANSAC
 * inliers of every pair whose inl_count >= min_inliers, pair-major, ascending match index.
 *   sfm_graph_offsets: out_offsets [n_pairs + 1] i64, exclusive scan of the verified counts
 *                      (out_offsets[n_pairs] = total rows); size out_rows from it.
 *   sfm_graph_rows:    out_rows [total][3] i32; match_count / matches / mask / inl_count as
 *                      written by sfm_match_batch and sfm_ransac_f_batch.
 */
int sfm_graph_offsets(sfm_ctx* ctx, int32_t n_pairs, const int32_t* inl_count,
                      int32_t min_inliers, int64_t* out_offsets);
int sfm_graph_rows(sfm_ctx* ctx, int32_t n_pairs, int32_t k_max, int32_t pair_base,
                   const int32_t* match_count, const int32_t* matches, const uint8_t* mask,
                   const int32_t* inl_count, int32_t min_inliers, const int64_t* offsets,
                   int32_t* out_rows);
/* The multi-GPU exchange form of the same graph (the graph all-gather):
 *   sfm_graph_rows_packed: out_packed [total] u32 = queryIdx << 16 | trainIdx (k_max <= 65536),
 *                          same order and offsets as sfm_graph_rows.
 *   sfm_graph_expand:      rows of n_pairs consecutive pairs back to [total][3] i32: pair p's
 *                          counts[p] packed rows start at packed[src_offsets[p]] (e.g. inside
 *                          the padded per-rank slots of an all-gather) and are written at row
 *                          dst_offsets[p] as (pair_base + p, queryIdx, trainIdx).
 */
int sfm_graph_rows_packed(sfm_ctx* ctx, int32_t n_pairs, int32_t k_max,
                          const int32_t* match_count, const int32_t* matches, const uint8_t* mask,
                          const int32_t* inl_count, int32_t min_inliers, const int64_t* offsets,
                          uint32_t* out_packed);
int sfm_graph_expand(sfm_ctx* ctx, int32_t n_pairs, int32_t pair_base, const int32_t* counts,
                     const int64_t* src_offsets, const int64_t* dst_offsets,
                     const uint32_t* packed, int32_t* out_rows);

/* ---- bundle-adjustment linearisation ---------------------------------------------------------
 * Fills the empty code/3d_reconstruction.py (import commented out at code/pipeline.py:4) with the
 * J^TJ build of papers/schoenberger2016sfm.pdf eq. (1) / §4.4.  Observations must be grouped by
 * point (pt_ptr = CSR row pointer over points, n_pt + 1 entries); cam_ptr/cam_obs is the CSR
 * index of observations by camera.
 *   cams [n_cam][8] f64 (angle-axis, t, f, k1), pp [n_cam][2] f64, pts [n_pt][3] f64
 *   uv [n_obs][2] f64, cam_idx/pt_idx [n_obs] i32
 *   out: U [n_cam][8][8], V [n_pt][3][3], W [n_obs][8][3], gc [n_cam][8], gp [n_pt][3],
 *        res [n_obs][2], cost [1] (0.5 * sum rho)
 */
int sfm_ba_jtj(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* pp, int32_t n_pt,
               const double* pts, int32_t n_obs, const int32_t* cam_idx, const int32_t* pt_idx,
               const double* uv, const int32_t* pt_ptr, const int32_t* cam_ptr,
               const int32_t* cam_obs, double loss_s, double* U, double* V, double* W,
               double* gc, double* gp, double* res, double* cost);

/* ---- bundle-adjustment step (LM with Schur complement + PCG) ----------------------------------
 * SURVEY.md §8f item 3 ("rest of incremental SfM for cfg5"): the step of paper eq. (1) that the
 * empty code/3d_reconstruction.py would take after the J^TJ build above.  Spec: DESIGN.md §4.5,
 * restated by oracle/ba_lm.py.
 *
 * sfm_ba_solve: solves the Marquardt-damped normal equations of sfm_ba_jtj's blocks,
 *     [U + λ D_U   W ; Wᵀ   V + λ D_V] [dc; dp] = -[gc; gp],  D = clamp(diag, 1e-6, 1e32),
 *   by the Schur complement on the points and block-Jacobi preconditioned CG on the cameras
 *   (S is never formed), then back-substitutes dp.  Same CSR inputs as sfm_ba_jtj
 *   (observations point-major).  Stops when |r| <= tol |b| or after max_iter iterations.
 *   out (device): dc [n_cam][8], dp [n_pt][3],
 *   info [5] f64 = {CG iterations, |r|/|b|, gᵀδ, δᵀ JᵀJ δ (undamped), preconditioner fallback}
 *   — the LM predicted decrease is -(gᵀδ + ½ δᵀ JᵀJ δ).
 * sfm_ba_cost:   cost = 0.5 Σ ρ(|r|²) at the given parameters (no Jacobians).
 * sfm_ba_update: cams_out = cams ⊕ dc (R <- exp([δr]x) R, the tangent space of the Jacobians;
 *   t, f, k1 additive), pts_out = pts + dp.  Out-of-place.
 */
typedef struct sfm_ba_solve_params {
    double lambda;    /* Marquardt damping λ (>= 0) */
    double tol;       /* relative CG residual |r|/|b| */
    int32_t max_iter; /* CG iteration cap */
    int32_t poll;     /* convergence poll: every `poll` > 0 CG iterations the host reads the
                         device's convergence flag (one 4-byte copy + a hipStreamSynchronize) and
                         stops enqueueing once it is set; 0 (the zero-initialised struct) = every
                         SFM_BA_POLL_DEFAULT (8) iterations; < 0 = never: fully asynchronous,
                         capturable in a hip graph (all max_iter iterations are enqueued, the
                         converged ones exit at once).  Results are identical either way.
                         (sfm_version 1 read 0 as "never"; version 2 restores 0 = poll.) */
    int32_t poll_first; /* > 0: the first poll at iteration poll_first, then every `poll` (a
                         caller that expects about as many iterations as its previous solve took
                         polls once, there, instead of at every multiple of `poll`); 0 = at
                         `poll` (sfm_version 5; earlier versions had no such field) */
} sfm_ba_solve_params;
#define SFM_BA_POLL_DEFAULT 8

int sfm_ba_solve(sfm_ctx* ctx, int32_t n_cam, int32_t n_pt, int32_t n_obs,
                 const int32_t* cam_idx, const int32_t* pt_idx, const int32_t* pt_ptr,
                 const int32_t* cam_ptr, const int32_t* cam_obs, const double* U, const double* V,
                 const double* W, const double* gc, const double* gp,
                 const sfm_ba_solve_params* prm, double* dc, double* dp, double* info);
/* Multi-GPU form of sfm_ba_solve (observations sharded by point, one process per
 * GPU), as caller-driven stages so that no callback crosses the ABI: the caller all-reduces
 * (sums over all ranks, in place) the device buffer comm (>= 44 * n_cam doubles) between the
 * stage that fills it and the next one, ordered on the context's stream (e.g. an RCCL all-reduce
 * enqueued on it).  V, W, gp, dp, pt_ptr and the observation arrays are this rank's point shard
 * (indices local to it); U and gc are the GLOBAL camera blocks (sfm_ba_jtj on the shard, an
 * all-reduce of U / gc, then sfm_ba_fix_params).  Sequence (prm / arrays identical in every call;
 * no other sfm_* call on this context in between — the stages share its workspace):
 *   SETUP           -> all-reduce comm[0, 44 n_cam)  -> SETUP_FINISH
 *   for k = 0 .. max_iter-1:
 *     [every prm->poll > 0 iterations, k > 0 (from prm->poll_first when > 0): POLL -> *done
 *      (host int32); stop if 1]
 *     ITER(k)       -> all-reduce comm[0, 8 n_cam)   -> ITER_FINISH(k)
 *   BACKSUB         -> all-reduce comm[0, 2)         -> MODEL   (dc, dp, info as sfm_ba_solve)
 * After each all-reduce every camera-space value is replicated, so every rank takes the same CG
 * decisions (POLL included) and issues the same collectives; dc and info are the same on every
 * rank, dp is the shard's.  Equal to sfm_ba_solve on the whole problem up to the fp64 summation
 * order.  No counterpart in the reference (its BA module is empty). */
#define SFM_BA_STAGE_SETUP 0
#define SFM_BA_STAGE_SETUP_FINISH 1
#define SFM_BA_STAGE_ITER 2
#define SFM_BA_STAGE_ITER_FINISH 3
#define SFM_BA_STAGE_BACKSUB 4
#define SFM_BA_STAGE_MODEL 5
#define SFM_BA_STAGE_POLL 6
#define SFM_BA_STAGE_SCHUR 7   /* explicit S only (sfm_ba_set_schur): after SETUP, exports T's partials */
int sfm_ba_solve_stage(sfm_ctx* ctx, int32_t stage, int32_t k, int32_t n_cam, int32_t n_pt,
                       int32_t n_obs, const int32_t* cam_idx, const int32_t* pt_idx,
                       const int32_t* pt_ptr, const int32_t* cam_ptr, const int32_t* cam_obs,
                       const double* U, const double* V, const double* W, const double* gc,
                       const double* gp, const sfm_ba_solve_params* prm, double* comm, double* dc,
                       double* dp, double* info, int32_t* done);
/* Fixed parameters (the gauge: the reference camera's pose and one translation coordinate of a
 * second camera; known intrinsics f, k1): in place on sfm_ba_jtj's U [n_cam][8][8], W [n_obs][8][3]
 * and g_c [n_cam][8], the rows/columns of the parameters marked in fixed [n_cam][8] (u8, 1 =
 * fixed) become the identity's, their g_c entries and W rows 0 — sfm_ba_solve then returns
 * δ = 0 for them exactly.  Call after sfm_ba_jtj (and after any camera-block all-reduce). */
int sfm_ba_fix_params(sfm_ctx* ctx, int32_t n_cam, int32_t n_obs, const int32_t* cam_idx,
                      const uint8_t* fixed, double* U, double* W, double* gc);
int sfm_ba_cost(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* pp, int32_t n_pt,
                const double* pts, int32_t n_obs, const int32_t* cam_idx, const int32_t* pt_idx,
                const double* uv, double loss_s, double* cost);
int sfm_ba_update(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* dc, int32_t n_pt,
                  const double* pts, const double* dp, double* cams_out, double* pts_out);

/* Sharding-invariant sums (chunk mode, sfm_version 3).  The points of the WHOLE problem are cut
 * into n_total fixed chunks (contiguous point ranges; a rank's shard is a run of whole chunks), and
 * every sum that runs over points or observations into a camera-space or scalar value — U / g_c
 * and the cost of sfm_ba_jtj, sfm_ba_cost, the Schur diagonal blocks and b of the solve set-up,
 * the CG product Σ_o u_o, the LM model terms — is computed per chunk (an order that depends only
 * on the chunk's own observations) and the chunk partials are combined by ONE canonical pairwise
 * tree over all n_total chunks: while n > 1, a[i] = a[2i] + a[2i+1] (i < n/2), an odd last
 * element is carried, n = ceil(n/2).  Results are then bit-identical for every split of the
 * chunks over ranks, the single process included.
 *   sfm_ba_set_chunks(ctx, n_chunk, chunk_pt, chunk_obs, n_total, cam_bounds): the next BA calls
 *   on ctx work on a problem holding n_chunk of the chunks; chunk_pt / chunk_obs (host, n_chunk +
 *   1) are their LOCAL point offsets and the matching observation offsets (pt_ptr[chunk_pt[k]];
 *   chunk_pt[0] = 0, chunk_pt[n_chunk] = n_pt, non-decreasing; empty chunks allowed); cam_bounds
 *   (device, [n_cam][n_chunk + 1] i32, caller-owned) are the positions in cam_obs where each
 *   camera's observation list crosses those offsets (the list is ascending, so each chunk's part
 *   is contiguous): cam_bounds[c][0] = cam_ptr[c], cam_bounds[c][n_chunk] = cam_ptr[c + 1].
 *   n_total = 0: the problem is the whole one (n_chunk = n_total chunks), every result is final.
 *   n_total > 0: a shard (export form): sfm_ba_jtj writes U as [n_chunk][n_cam][8][8], gc as
 *   [n_chunk][n_cam][8] and cost as [n_chunk] (chunk partials, combined by the caller after
 *   gathering every rank's chunks in chunk order: sfm_ba_chunk_tree), sfm_ba_cost writes cost
 *   [n_chunk]; the sharded solve's stages write chunk partials to comm and the stages after the
 *   exchange read ALL n_total chunks' partials in chunk order: SETUP -> comm [n_chunk][n_cam][44],
 *   gathered [n_total][n_cam][44] -> SETUP_FINISH; ITER -> [n_chunk][n_cam][8], gathered ->
 *   ITER_FINISH; BACKSUB -> [n_chunk][2], gathered -> MODEL (an all-GATHER instead of the
 *   all-reduce; comm >= n_total * 44 * n_cam doubles).
 *   n_chunk = 0 switches chunk mode off (the default: the round-4 sums).  1 <= n_chunk <= 16.
 *   sfm_ba_chunk_tree(ctx, n_total, n, parts, out): out[i] = canonical tree over k of
 *   parts[k * n + i] (device arrays), i < n — the combine the library applies itself. */
#define SFM_BA_MAX_CHUNKS 16
int sfm_ba_set_chunks(sfm_ctx* ctx, int32_t n_chunk, const int32_t* chunk_pt,
                      const int32_t* chunk_obs, int32_t n_total, const int32_t* cam_bounds);
int sfm_ba_chunk_tree(sfm_ctx* ctx, int32_t n_total, int64_t n, const double* parts, double* out);

/* Explicit reduced camera system (sfm_version 4; needs chunk mode).  The solve forms the
 * off-diagonal Schur blocks T_ij = Σ_p W_pi V_d,p⁻¹ W_pjᵀ once per solve (S_ij = -T_ij, i != j) and
 * runs the CG on S directly — two launches per iteration over 64 B per camera-pair block instead of
 * streaming W (192 B per observation) every iteration.  It pays when the camera-pair products are
 * few against the CG iterations (short tracks); the caller decides (reconstruction.schur_rule).
 *   sfm_ba_set_schur(ctx, n_slot, slot_cam, n_seg, seg, n_inst, inst, row_ptr, n_ent, row_ent,
 *                    n_group, sg_ptr, sg, gk):
 *   slot_cam [n_slot][2] (ci <= cj): the camera pairs (slots) of the WHOLE problem, the same table
 *   on every rank; inst [2][n_inst] (observation a, observation b of one point, LOCAL observation
 *   indices; cam(a) = ci, cam(b) = cj of its slot; a pair within one camera appears as (a, b) and
 *   (b, a)); seg [4][n_seg] (local chunk, slot, first instance, end instance): this problem's
 *   instances grouped by (chunk, slot), each group in point order — a group's T partial is the
 *   fixed-order sum over it; row_ptr [n_cam + 1], row_ent [n_ent] = 2 slot + t: block row c of S
 *   (t = 1: the slot's transpose), in a fixed order.  The groups of the WHOLE problem (every rank's,
 *   in chunk order: a shard's n_seg groups are a contiguous run of them): n_group of them, gk
 *   [n_group] their chunk, sg_ptr [n_slot + 1] / sg [n_group] each slot's groups in chunk order.
 *   T_slot = the canonical chunk tree over the slot's group partials (missing chunks 0).  All
 *   device, caller-owned.  n_slot = 0 turns it off.  Sharded (n_total > 0): SCHUR (after SETUP)
 *   writes the shard's group partials [n_seg][64] at its comm pointer (the caller passes comm +
 *   n_total·44·n_cam + g0·64, g0 = the shard's first group); one exchange of n_total·44·n_cam +
 *   n_group·64 doubles (zero-filled: an exact all-gather); SETUP_FINISH; then ITER / ITER_FINISH
 *   need no exchange (S is replicated). */
int sfm_ba_set_schur(sfm_ctx* ctx, int32_t n_slot, const int32_t* slot_cam, int32_t n_seg,
                     const int32_t* seg, int32_t n_inst, const int32_t* inst, const int32_t* row_ptr,
                     int32_t n_ent, const int32_t* row_ent, int32_t n_group, const int32_t* sg_ptr,
                     const int32_t* sg, const int32_t* gk);

/* ---- feature tracks ----------------------------------------------------------------------------
 * the verified match graph (sfm_graph_rows) -> tracks, the input of
 * triangulation and bundle adjustment.  Nodes are (image, keypoint), node = img_base[image] +
 * keypoint (img_base [n_img + 1] i32, exclusive scan of the keypoint counts); each graph row
 * (pair, queryIdx, trainIdx) joins node(pairs[pair][0], q) and node(pairs[pair][1], t).
 * A track is a connected component with >= min_len nodes and at most one node per image;
 * tracks are ordered by their smallest node id, nodes ascending within a track (deterministic).
 *   out (device): n_tracks [1], track_ptr [n_tracks + 1] (capacity n_nodes + 1),
 *                 track_img, track_kp [track_ptr[n_tracks]] (capacity n_nodes).
 * Synchronises the stream (the component rounds are host-driven). */
int sfm_tracks(sfm_ctx* ctx, int32_t n_img, const int32_t* img_base, int32_t n_pairs,
               const int32_t* pairs, int64_t n_rows, const int32_t* rows, int32_t min_len,
               int32_t* out_n_tracks, int32_t* out_track_ptr, int32_t* out_track_img,
               int32_t* out_track_kp);

/* ---- triangulation ---------------------------------------------------------------------------
 * the points of the tracks (sfm_tracks) from posed cameras, the start of
 * bundle adjustment.  Multi-view DLT on undistorted normalised coordinates (spec in
 * csrc/triangulate.hip; restated by oracle/recon.py).  Observations point-major: pt_ptr [n_pt+1]
 * CSR, cam_idx [n_obs] i32, uv [n_obs][2] f64; cams [n_cam][8], pp [n_cam][2] as sfm_ba_jtj.
 *   out (device): pts [n_pt][3] f64; stats [n_pt][4] f64 = {mean reprojection error (px), largest
 *   ray angle (deg), smallest depth, status: 0 ok, 1 < 2 views, 2 at infinity, 3 behind a camera}.
 */
int sfm_triangulate(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* pp,
                    int32_t n_pt, const int32_t* pt_ptr, const int32_t* cam_idx, const double* uv,
                    double* out_pts, double* out_stats);

/* ---- next-view registration ---------------------------------------------------------------
 * registers a batch of images against triangulated points (P3P RANSAC +
 * Gauss-Newton refinement; spec in oracle/sfm_oracle_reg.c / csrc/register.hip).  Per image i:
 * correspondences corr_ptr[i]..corr_ptr[i+1] of xy [n][2] f64 (pixels) and X [n][3] f64 (world),
 * intrinsics intr [n_img][4] = (f, k1, cx, cy), img_id [n_img] (keys the hypothesis RNG).
 * Hypothesis h of image i depends only on (seed, img_id[i], h): batch-composition invariant.
 *   out (device): cams [n_img][8] (angle-axis, t, f, k1; zeros on failure), count [n_img]
 *   (RANSAC inliers, -1 = no pose), key [n_img] (4 h + root of the winner, -1), mask [n] u8. */
typedef struct sfm_register_params {
    int32_t n_hyp;   /* multiple of 256 */
    int32_t refine;  /* 1: Gauss-Newton on the inliers (10 steps) */
    double thr;      /* inlier threshold, pixels */
    uint64_t seed;
} sfm_register_params;

int sfm_register_batch(sfm_ctx* ctx, int32_t n_img, const int32_t* corr_ptr, const double* xy,
                       const double* X, const double* intr, const int32_t* img_id,
                       const sfm_register_params* prm, double* out_cams, int32_t* out_count,
                       int32_t* out_key, uint8_t* out_mask);

/* ---- ORB feature extraction -------------------------------------------------------------------
 * replaces cv2.ORB_create() + orb.detectAndCompute(gray, None) of
 * code/feature_matching.py:42-45 (OpenCV defaults: 500 features, scale 1.2, 8 levels, edge 31,
 * patch 31, FAST 20, Harris score), batched over images of one size.  The spec is the build's
 * integer-exact restatement of the published algorithm (oracle/sfm_oracle_orb.c header; parity
 * against OpenCV itself unpinned: no cv2 here).
 *   images    [n_img][H][W] u8 (device)
 *   out_kp    [n_img][n_features][6] f32: x, y (level-0 pixels), size, angle (deg), Harris
 *             response, octave — level order, best Harris first within a level
 *   out_desc  [n_img][n_features][32] u8 (256-bit rBRIEF, OpenCV bit order)
 *   out_count [n_img] i32 keypoints found (<= n_features)
 */
typedef struct sfm_orb_params {
    int32_t n_features;      /* 500 */
    int32_t n_levels;        /* 8 (<= 16) */
    double scale_factor;     /* 1.2 */
    int32_t fast_threshold;  /* 20 */
    int32_t _pad;
} sfm_orb_params;

int sfm_orb_batch(sfm_ctx* ctx, const uint8_t* images, int32_t n_img, int32_t H, int32_t W,
                  const sfm_orb_params* prm, float* out_kp, uint8_t* out_desc,
                  int32_t* out_count);

/* ---- measurement: the device's i8 matrix ceiling right now ------------------------------------
 * Not a reference interface: the bench line's calibration probe (bench.py "calib"), so that K1's
 * roofline fraction can be read against the ceiling of the box it ran on.  Every CU runs MFMA-only
 * waves (v_mfma_i32_32x32x32_i8, register operands, random data, 2 waves per SIMD) for about
 * target_ms (0 < target_ms <= 5000).  out[4]: wall ms of the measured launch, i8 TOP/s, median
 * in-kernel clock (GHz), fraction of the nominal dense-i8 peak.  Synchronises the stream. */
int sfm_calib_mfma_i8(sfm_ctx* ctx, float target_ms, double* out);

#ifdef __cplusplus
}
#endif
#endif /* SFMCORE_H */
