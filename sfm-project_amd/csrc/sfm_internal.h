// Internal helpers shared by the HIP translation units of libsfmcore (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/sfmcore.h"

struct sfm_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    void* ws = nullptr;          // growable device workspace (shared by every call on ctx)
    size_t ws_bytes = 0;
    hipEvent_t handoff = nullptr;  // orders the workspace across sfm_ctx_set_stream switches
    int32_t* pinned = nullptr;     // small pinned host buffer (device -> host flag reads)
    hipEvent_t poll_ev = nullptr;  // the BA solve's look-ahead convergence poll (lazily created)
    int n_cu = 256;
    // RANSAC execution statistics (sfm_ransac_stats): on/off and the accumulated (executed,
    // algorithmic, pairs) evaluation counters; the per-wave counts live in the batch workspace
    int ransac_stats = 0;
    unsigned long long* rs_acc = nullptr;
    // the last counted batch's per-wave counts (sfm_ransac_wave_stops): where, and its shape
    const uint32_t* rs_last_w = nullptr;
    int rs_last_pairs = 0, rs_last_hyp = 0;
    // BA chunk mode (sfm_ba_set_chunks): local chunk point offsets; n_total 0 = whole problem
    int ba_nchunk = 0, ba_ntotal = 0;
    int32_t ba_chunk_pt[17] = {0}, ba_chunk_obs[17] = {0};
    const int32_t* ba_cam_bounds = nullptr;
    // explicit reduced camera system (sfm_ba_set_schur): n_slot 0 = off
    int ba_nslot = 0, ba_nseg = 0, ba_ninst = 0, ba_nent = 0, ba_ngroup = 0;
    const int32_t *ba_slot_cam = nullptr, *ba_seg = nullptr, *ba_inst = nullptr,
                  *ba_row_ptr = nullptr, *ba_row_ent = nullptr, *ba_sg_ptr = nullptr,
                  *ba_sg = nullptr, *ba_gk = nullptr;
};

namespace sfm {

// BA chunk mode (sfm_ba_set_chunks): chunk offsets passed to kernels by value.
struct ChunkOff {
    int32_t v[17];
};
// Chunk of a (per-lane) index x in the monotone offsets off[0..nck] (off[k] <= x < off[k+1], the
// last chunk for x >= off[nck - 1]): fully unrolled compares against the kernel-argument offsets at
// compile-time positions (uniform scalar loads + selects) — a loop with a per-lane index into the
// argument struct would turn into dependent per-lane memory loads.  Returns k; *a / *b receive
// base[k] and base[k + 1] of a second offset table (may be the same).
__device__ __forceinline__ int chunk_of(int x, int nck, const ChunkOff& off, const ChunkOff& base,
                                        int& a, int& b) {
    int k = 0;
    a = base.v[0];
    b = base.v[1];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
        if (i < nck && x >= off.v[i]) {
            k = i;
            a = base.v[i];
            b = base.v[i + 1];
        }
    }
    return k;
}
// The canonical pairwise tree over the chunk partials a[0..n) (n <= 16): a fixed 16-leaf tree with
// the missing leaves 0 — the same as "a[i] = a[2i] + a[2i+1], an odd last one carried".
__device__ __forceinline__ double chunk_tree16(double (&a)[16]) {
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) a[i] = a[2 * i] + a[2 * i + 1];
    return a[0];
}

// Wave reduction of M <= 64 per-lane values by recursive halving: at the step with lane bit OFF,
// the lane keeps one half of its (zero-padded) values and adds the partner's copy of that half,
// so M values cost about M exchanges instead of the 6 M of M separate shuffle trees.  Afterwards
// a[0] of lane l is the wave sum of value `idx` (the sum of the kept-half offsets) when the call
// returns true; every value is held by exactly one such lane (a padding slot can carry an index
// that is real elsewhere, so `rs`, the real length of the lane's current slice, decides).  The
// association is fixed (a function of M).
template <int M, int OFF, int MINOFF = 1>
__device__ __forceinline__ void wave_halving_step(double* a, int lane, int& idx, int& rs) {
    if constexpr (OFF >= MINOFF) {
        constexpr int H = (M + 1) / 2;
        const bool up = (lane & OFF) != 0;
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const double lo = a[i], hi = (H + i < M) ? a[H + i] : 0.0;
            const double r = __shfl_xor(up ? lo : hi, OFF, 64);
            a[i] = (up ? hi : lo) + r;
        }
        if (up) {
            idx += H;
            rs -= H;
        } else if (rs > H) {
            rs = H;
        }
        wave_halving_step<H, OFF / 2, MINOFF>(a, lane, idx, rs);
    }
}
// The same over the lanes that share lane bits below MINOFF (e.g. MINOFF 2: even lanes with even
// lanes, odd with odd), M <= 64 / MINOFF values.
template <int M, int MINOFF>
__device__ __forceinline__ bool wave_halving_sum_strided(double* a, int lane, int& idx) {
    static_assert(M >= 1 && M <= 64 / MINOFF, "wave_halving_sum_strided: too many values");
    int rs = M;
    idx = 0;
    wave_halving_step<M, 32, MINOFF>(a, lane, idx, rs);
    return rs > 0;
}
// LANES < 64: the same over each aligned group of LANES lanes (a power of two, M <= LANES).
template <int M, int LANES = 64>
__device__ __forceinline__ bool wave_halving_sum(double* a, int lane, int& idx) {
    static_assert(LANES >= 2 && LANES <= 64 && (LANES & (LANES - 1)) == 0, "wave_halving_sum: lanes");
    static_assert(M >= 1 && M <= LANES, "wave_halving_sum: 1..LANES values");
    int rs = M;
    idx = 0;
    wave_halving_step<M, LANES / 2>(a, lane, idx, rs);
    return rs > 0;
}

void set_error(const std::string& msg);

// Returns a device pointer with at least `bytes` of workspace (grows, never shrinks).
void* workspace(sfm_ctx* ctx, size_t bytes);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

#define SFM_HIP_CHECK(expr)                                                                   \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            sfm::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                \
            return SFM_ERR_HIP;                                                               \
        }                                                                                     \
    } while (0)

#define SFM_REQUIRE(cond, msg)                                                                \
    do {                                                                                      \
        if (!(cond)) { sfm::set_error(msg); return SFM_ERR_INVALID; }                          \
    } while (0)

}  // namespace sfm

// Kernel-launch entry points implemented in the per-stage translation units.
int sfm_match_both_launch(sfm_ctx* ctx, int metric, const uint8_t* desc, const int32_t* n_kp,
                          int32_t n_img, int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                          const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                          int32_t* out_dist);
int sfm_match_l2_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                        int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                        const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                        int32_t* out_dist);
int sfm_match_l2fr_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                          int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                          const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                          int32_t* out_dist);
int sfm_match_hamming_mfma_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp,
                                  int32_t n_img, int32_t k_max, const int32_t* pairs,
                                  int32_t n_pairs, const sfm_match_params* prm,
                                  int32_t* out_count, int32_t* out_match, int32_t* out_dist);
int sfm_match_hamming_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp,
                             int32_t n_img, int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                             const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                             int32_t* out_dist);
