// ORB feature extraction on the GPU (the reference's
// cv2.ORB_create() + detectAndCompute at code/feature_matching.py:42-45, which the reference runs
// 2 x N(N-1) times in its pair loop, code/pipeline.py:38-41).  Batched over images of one size.
//
// The spec is integer-exact and restated on the CPU by oracle/sfm_oracle_orb.c (read its header:
// pyramid by 11-bit bilinear resampling of level 0, FAST-9 score = best arc's minimum contrast,
// 3x3 strict non-maximum suppression, 2 n_l best FAST scores then n_l best Harris responses
// R = 25 (ab - c^2) - (a+b)^2 with raster-order tie breaks, intensity-centroid orientation, 256
// rotated BRIEF tests on a 7x7 Gaussian blur with EXACT rounding of the rotated test points).
// Parity against OpenCV itself is unpinned (no cv2 here); against the oracle it is bit-exact.
//
// Kernels (grid y = image):
//   orb_pyr_kernel     thread per pyramid pixel: level 0 copied, level l >= 1 resampled
//   orb_blur_kernel    thread per pixel: 7x7 separable Gaussian, fixed point
//   orb_fast_kernel    thread per pixel: FAST-9 score inside the 31-pixel border (0 elsewhere)
//   orb_nms_kernel     thread per pixel: strict 3x3 maximum flag
//   orb_rows_kernel    wave per level row: survivors per row (ballot), and with the row offsets
//                      from orb_scan_kernel the raster-order candidate list (x, y, score packed)
//   orb_select_kernel  block per (image, level): FAST-score top 2 n_l by histogram threshold,
//                      Harris, LDS bitonic sort, orientation and descriptors of the n_l best
//   orb_pack_kernel    block per image: levels' slots -> one dense list per image
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "sfm_internal.h"

namespace {

constexpr int EDGE = 31;
constexpr int MAXC = 32768;      // candidates per level (raster order)
constexpr int MAXLEV = 16;
constexpr int SEL_MAX = 1024;    // 2 n_l per level handled by the select kernel
constexpr int RADIUS = 15;

struct OrbLevels {
    int32_t nlev;
    int32_t W[MAXLEV], H[MAXLEV], n[MAXLEV], slot[MAXLEV];  // slot: first output slot of level
    int64_t off[MAXLEV + 1];         // pixel offset of each level in an image's pyramid
    int64_t rowoff[MAXLEV + 1];      // row offset of each level (row-count arrays)
    int32_t mapx[MAXLEV], mapy[MAXLEV];  // offsets (entries of 3 ints) into the axis-map table
    double sc[MAXLEV];
};

__constant__ int c_fast_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int c_fast_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
__constant__ int c_blur_w[7] = {18, 34, 49, 54, 49, 34, 18};

__device__ __forceinline__ int find_level(const OrbLevels& L, int64_t i) {
    int l = 0;
    while (l + 1 < L.nlev && i >= L.off[l + 1]) ++l;
    return l;
}

__global__ __launch_bounds__(256) void orb_pyr_kernel(const uint8_t* __restrict__ imgs, int H,
                                                      int W, OrbLevels L,
                                                      const int32_t* __restrict__ maps,
                                                      uint8_t* __restrict__ pyr) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t tot = L.off[L.nlev];
    if (i >= tot) return;
    const uint8_t* img = imgs + (size_t)blockIdx.y * H * W;
    uint8_t* out = pyr + (size_t)blockIdx.y * tot;
    const int l = find_level(L, i);
    const int64_t p = i - L.off[l];
    const int w = L.W[l];
    const int y = (int)(p / w), x = (int)(p - (int64_t)y * w);
    if (l == 0) {
        out[i] = img[(size_t)y * W + x];
        return;
    }
    const int32_t* mx = maps + 3 * (L.mapx[l] + x);
    const int32_t* my = maps + 3 * (L.mapy[l] + y);
    const uint8_t* r0 = img + (size_t)my[0] * W;
    const uint8_t* r1 = img + (size_t)my[1] * W;
    const int wx = mx[2], wy = my[2];
    const int t0 = r0[mx[0]] * (2048 - wx) + r0[mx[1]] * wx;
    const int t1 = r1[mx[0]] * (2048 - wx) + r1[mx[1]] * wx;
    out[i] = (uint8_t)((t0 * (2048 - wy) + t1 * wy + (1 << 21)) >> 22);
}

__global__ __launch_bounds__(256) void orb_blur_kernel(const uint8_t* __restrict__ pyr, OrbLevels L,
                                                       uint8_t* __restrict__ blur) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t tot = L.off[L.nlev];
    if (i >= tot) return;
    const int l = find_level(L, i);
    const int64_t p = i - L.off[l];
    const int w = L.W[l], h = L.H[l];
    const int y = (int)(p / w), x = (int)(p - (int64_t)y * w);
    const uint8_t* lv = pyr + (size_t)blockIdx.y * tot + L.off[l];
    int acc = 0;
#pragma unroll
    for (int j = -3; j <= 3; ++j) {
        const uint8_t* row = lv + (size_t)min(max(y + j, 0), h - 1) * w;
        int s = 0;
#pragma unroll
        for (int q = -3; q <= 3; ++q) s += c_blur_w[q + 3] * row[min(max(x + q, 0), w - 1)];
        acc += c_blur_w[j + 3] * s;
    }
    blur[(size_t)blockIdx.y * tot + i] = (uint8_t)((acc + 32768) >> 16);
}

__global__ __launch_bounds__(256) void orb_fast_kernel(const uint8_t* __restrict__ pyr, OrbLevels L,
                                                       int thr, uint8_t* __restrict__ score) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t tot = L.off[L.nlev];
    if (i >= tot) return;
    const int l = find_level(L, i);
    const int64_t p = i - L.off[l];
    const int w = L.W[l], h = L.H[l];
    const int y = (int)(p / w), x = (int)(p - (int64_t)y * w);
    int s = 0;
    if (x >= EDGE && x < w - EDGE && y >= EDGE && y < h - EDGE) {
        const uint8_t* lv = pyr + (size_t)blockIdx.y * tot + L.off[l];
        const int c = lv[(size_t)y * w + x];
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = (int)lv[(size_t)(y + c_fast_dy[k]) * w + x + c_fast_dx[k]] - c;
        int best = 0;
#pragma unroll
        for (int st = 0; st < 16; ++st) {
            int b = 255, k = 255;
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const int v = d[(st + q) & 15];
                b = min(b, v);
                k = min(k, -v);
            }
            best = max(best, max(b, k));
        }
        s = best > thr ? best : 0;
    }
    score[(size_t)blockIdx.y * tot + i] = (uint8_t)s;
}

__global__ __launch_bounds__(256) void orb_nms_kernel(const uint8_t* __restrict__ score, OrbLevels L,
                                                      uint8_t* __restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t tot = L.off[L.nlev];
    if (i >= tot) return;
    const int l = find_level(L, i);
    const int64_t p = i - L.off[l];
    const int w = L.W[l], h = L.H[l];
    const int y = (int)(p / w), x = (int)(p - (int64_t)y * w);
    const uint8_t* sc = score + (size_t)blockIdx.y * tot + L.off[l];
    int keep = 0;
    const int s = sc[(size_t)y * w + x];
    if (s && x >= EDGE && x < w - EDGE && y >= EDGE && y < h - EDGE) {
        keep = 1;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx)
                if ((dx || dy) && sc[(size_t)(y + dy) * w + x + dx] >= s) keep = 0;
    }
    flag[(size_t)blockIdx.y * tot + i] = (uint8_t)keep;
}

// Wave per level row (grid x = global row / 4, 4 waves per block).  pass 0: survivors per row;
// pass 1: write them, packed (y << 20 | x << 8 | score), at the row's offset (raster order).
__global__ __launch_bounds__(256) void orb_rows_kernel(int pass, const uint8_t* __restrict__ flag,
                                                       const uint8_t* __restrict__ score,
                                                       OrbLevels L, int32_t* __restrict__ rowcnt,
                                                       const int32_t* __restrict__ rowpos,
                                                       int32_t* __restrict__ cand) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nrows = L.rowoff[L.nlev];
    if (r >= nrows) return;  // wave-uniform
    int l = 0;
    while (l + 1 < L.nlev && r >= L.rowoff[l + 1]) ++l;
    const int y = (int)(r - L.rowoff[l]);
    const int w = L.W[l], h = L.H[l];
    const size_t img = blockIdx.y;
    const int64_t tot = L.off[L.nlev];
    const size_t gr = img * (size_t)nrows + r;
    if (y < EDGE || y >= h - EDGE) {
        if (pass == 0 && lane == 0) rowcnt[gr] = 0;
        return;
    }
    const uint8_t* fl = flag + img * tot + L.off[l] + (size_t)y * w;
    const uint8_t* sc = score + img * tot + L.off[l] + (size_t)y * w;
    int n = 0;
    int pos = pass ? rowpos[gr] : 0;
    int32_t* out = cand + (img * L.nlev + l) * (size_t)MAXC;
    for (int x0 = EDGE; x0 < w - EDGE; x0 += 64) {
        const int x = x0 + lane;
        const bool f = x < w - EDGE && fl[x];
        const unsigned long long m = __ballot(f);
        if (pass && f) {
            const int k = pos + n + __popcll(m & ((1ull << lane) - 1ull));
            if (k < MAXC) out[k] = (int32_t)(((unsigned)y << 20) | ((unsigned)x << 8) | sc[x]);
        }
        n += __popcll(m);
    }
    if (pass == 0 && lane == 0) rowcnt[gr] = n;
}

// Block per (image, level): exclusive scan of the level's row counts (fixed order) -> row
// positions and the level's candidate count (capped at MAXC).
__global__ __launch_bounds__(256) void orb_scan_kernel(OrbLevels L, const int32_t* __restrict__ rowcnt,
                                                       int32_t* __restrict__ rowpos,
                                                       int32_t* __restrict__ ncand) {
    __shared__ int carry;
    __shared__ int wsum[4];
    const int l = blockIdx.x, tid = threadIdx.x;
    const size_t img = blockIdx.y;
    const int64_t nrows = L.rowoff[L.nlev];
    const int32_t* rc = rowcnt + img * nrows + L.rowoff[l];
    int32_t* rp = rowpos + img * nrows + L.rowoff[l];
    const int h = L.H[l];
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int y0 = 0; y0 < h; y0 += 256) {
        const int y = y0 + tid;
        const int v = y < h ? rc[y] : 0;
        int incl = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if ((tid & 63) >= off) incl += t;
        }
        if ((tid & 63) == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        int base = carry;
        for (int k = 0; k < (tid >> 6); ++k) base += wsum[k];
        if (y < h) rp[y] = base + incl - v;
        __syncthreads();
        if (tid == 255) carry = base + incl;
        __syncthreads();
    }
    if (tid == 0) ncand[img * L.nlev + l] = min(carry, MAXC);
}

__device__ __forceinline__ bool le_r(long long B, long long A, long long R2) {
    if (B <= 0 && A >= 0) return true;
    if (B > 0 && A < 0) return false;
    if (B >= 0) return B * B * R2 <= A * A;
    return B * B * R2 >= A * A;
}

// floor(n / sqrt(R2) + 1/2) exactly: a floating estimate, then integer comparisons decide
__device__ __forceinline__ int round_div(long long n, long long R2) {
    long long k = (long long)floor((double)n / sqrt((double)R2) + 0.5);
    while (!le_r(2 * k - 1, 2 * n, R2)) --k;
    while (le_r(2 * k + 1, 2 * n, R2)) ++k;
    return (int)k;
}

// Block per (image, level), 256 threads.
__global__ __launch_bounds__(256) void orb_select_kernel(
    const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur, OrbLevels L,
    const int32_t* __restrict__ cand, const int32_t* __restrict__ ncand,
    const int32_t* __restrict__ pattern, int nfeat, float* __restrict__ slot_kp,
    uint8_t* __restrict__ slot_desc, int32_t* __restrict__ lvl_count) {
    __shared__ int hist[256];
    __shared__ int s_T, s_above, s_sel, s_ties;
    __shared__ int wcnt[4][2];
    __shared__ unsigned sel_c[SEL_MAX];
    __shared__ long long sel_r[SEL_MAX];
    __shared__ int sel_i[SEL_MAX];
    __shared__ int s_pat[1024];
    const int l = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const size_t img = blockIdx.y;
    const int nl = L.n[l];
    const int w = L.W[l];
    if (tid == 0) lvl_count[img * L.nlev + l] = 0;
    if (nl <= 0) return;
    const int nc = ncand[img * L.nlev + l];
    const int32_t* cd = cand + (img * L.nlev + l) * (size_t)MAXC;
    const int64_t tot = L.off[L.nlev];
    const uint8_t* lv = pyr + img * tot + L.off[l];
    const uint8_t* bl = blur + img * tot + L.off[l];
    for (int k = tid; k < 1024; k += 256) s_pat[k] = pattern[k];
    // ---- the 2 n_l best FAST scores: histogram threshold, ties in raster order ----
    hist[tid] = 0;
    __syncthreads();
    for (int k = tid; k < nc; k += 256) atomicAdd(&hist[cd[k] & 255], 1);
    __syncthreads();
    const int a = 2 * nl;
    if (tid == 0) {
        int T = 0, above = 0;
        if (nc > a) {
            for (T = 255; T > 0; --T) {
                if (above + hist[T] >= a) break;
                above += hist[T];
            }
        }
        s_T = T; s_above = above; s_sel = 0; s_ties = 0;
    }
    __syncthreads();
    const int T = s_T, quota = a - s_above;
    const bool all = nc <= a;
    for (int k0 = 0; k0 < nc; k0 += 256) {
        const int k = k0 + tid;
        const int sc = k < nc ? (cd[k] & 255) : -1;
        const bool gt = k < nc && (all || sc > T);
        const bool eq = k < nc && !all && sc == T;
        // ordered ranks of this chunk: ties among equals, then selections
        const unsigned long long me = __ballot(eq);
        const int eq_before = __popcll(me & ((1ull << lane) - 1ull));
        if (lane == 0) wcnt[wv][0] = __popcll(me);
        __syncthreads();
        int eq_base = s_ties;
        for (int q = 0; q < wv; ++q) eq_base += wcnt[q][0];
        const bool take = gt || (eq && eq_base + eq_before < quota);
        const unsigned long long mt = __ballot(take);
        if (lane == 0) wcnt[wv][1] = __popcll(mt);
        __syncthreads();
        int sel_base = s_sel;
        for (int q = 0; q < wv; ++q) sel_base += wcnt[q][1];
        if (take) {
            const int pos = sel_base + __popcll(mt & ((1ull << lane) - 1ull));
            if (pos < SEL_MAX) sel_c[pos] = (unsigned)cd[k];
        }
        __syncthreads();
        if (tid == 0) {
            s_ties += wcnt[0][0] + wcnt[1][0] + wcnt[2][0] + wcnt[3][0];
            s_sel += wcnt[0][1] + wcnt[1][1] + wcnt[2][1] + wcnt[3][1];
        }
        __syncthreads();
    }
    const int n1 = min(s_sel, SEL_MAX);
    // ---- Harris response of the selected candidates ----
    int np2 = 1;
    while (np2 < n1) np2 <<= 1;
    for (int k = tid; k < np2; k += 256) {
        long long R = LLONG_MIN;
        if (k < n1) {
            const unsigned c = sel_c[k];
            const int y = (int)(c >> 20), x = (int)((c >> 8) & 4095u);
            long long A = 0, B = 0, C = 0;
            for (int v = -3; v <= 3; ++v)
                for (int u = -3; u <= 3; ++u) {
                    const uint8_t* m = lv + (size_t)(y + v) * w + (x + u);
                    const int ix = (m[-w + 1] + 2 * m[1] + m[w + 1]) - (m[-w - 1] + 2 * m[-1] + m[w - 1]);
                    const int iy = (m[w - 1] + 2 * m[w] + m[w + 1]) - (m[-w - 1] + 2 * m[-w] + m[-w + 1]);
                    A += (long long)ix * ix;
                    B += (long long)iy * iy;
                    C += (long long)ix * iy;
                }
            R = 25 * (A * B - C * C) - (A + B) * (A + B);
        }
        sel_r[k] = R;
        sel_i[k] = k;
    }
    __syncthreads();
    // ---- bitonic sort: R descending, raster index ascending ----
    for (int size = 2; size <= np2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int k = tid; k < np2; k += 256) {
                const int j = k ^ stride;
                if (j > k) {
                    const bool up = (k & size) == 0;  // first element should precede
                    const long long rk = sel_r[k], rj = sel_r[j];
                    const int ik = sel_i[k], ij = sel_i[j];
                    const bool k_first = rk > rj || (rk == rj && ik < ij);
                    if (k_first != up) {
                        sel_r[k] = rj; sel_r[j] = rk;
                        sel_i[k] = ij; sel_i[j] = ik;
                    }
                }
            }
            __syncthreads();
        }
    const int n2 = min(n1, nl);
    // ---- orientation and descriptor of the n_l best ----
    for (int k = tid; k < n2; k += 256) {
        const unsigned c = sel_c[sel_i[k]];
        const int y = (int)(c >> 20), x = (int)((c >> 8) & 4095u);
        long long m10 = 0, m01 = 0;
        for (int v = -RADIUS; v <= RADIUS; ++v) {
            const uint8_t* row = lv + (size_t)(y + v) * w + x;
            for (int u = -RADIUS; u <= RADIUS; ++u) {
                if (u * u + v * v > RADIUS * RADIUS) continue;
                const int I = row[u];
                m10 += (long long)u * I;
                m01 += (long long)v * I;
            }
        }
        const long long R2 = m10 * m10 + m01 * m01;
        double ang = atan2((double)m01, (double)m10) * (180.0 / 3.14159265358979323846);
        if (ang < 0.0) ang += 360.0;
        const size_t o = img * (size_t)nfeat + L.slot[l] + k;
        float* kp = slot_kp + 6 * o;
        kp[0] = (float)((double)x * L.sc[l]);
        kp[1] = (float)((double)y * L.sc[l]);
        kp[2] = (float)(31.0 * L.sc[l]);
        kp[3] = (float)ang;
        kp[4] = (float)((double)sel_r[k] / 25.0);
        kp[5] = (float)l;
        unsigned words[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int t = 0; t < 256; ++t) {
            int q[4];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const long long px = s_pat[4 * t + 2 * e], py = s_pat[4 * t + 2 * e + 1];
                if (R2 == 0) {
                    q[2 * e] = (int)px;
                    q[2 * e + 1] = (int)py;
                } else {
                    q[2 * e] = round_div(px * m10 - py * m01, R2);
                    q[2 * e + 1] = round_div(px * m01 + py * m10, R2);
                }
            }
            const int i1 = bl[(size_t)(y + q[1]) * w + x + q[0]];
            const int i2 = bl[(size_t)(y + q[3]) * w + x + q[2]];
            if (i1 < i2) words[t >> 5] |= 1u << (t & 31);
        }
        uint4* d = (uint4*)(slot_desc + 32 * o);
        d[0] = make_uint4(words[0], words[1], words[2], words[3]);
        d[1] = make_uint4(words[4], words[5], words[6], words[7]);
    }
    if (tid == 0) lvl_count[img * L.nlev + l] = n2;
}

// Block per image: the levels' slots -> one dense list (level order), count.
__global__ __launch_bounds__(256) void orb_pack_kernel(OrbLevels L, int nfeat,
                                                       const float* __restrict__ slot_kp,
                                                       const uint8_t* __restrict__ slot_desc,
                                                       const int32_t* __restrict__ lvl_count,
                                                       float* __restrict__ out_kp,
                                                       uint8_t* __restrict__ out_desc,
                                                       int32_t* __restrict__ out_count) {
    const size_t img = blockIdx.x;
    int base = 0;
    for (int l = 0; l < L.nlev; ++l) {
        const int n = lvl_count[img * L.nlev + l];
        for (int k = threadIdx.x; k < n; k += 256) {
            const size_t s = img * (size_t)nfeat + L.slot[l] + k, d = img * (size_t)nfeat + base + k;
#pragma unroll
            for (int q = 0; q < 6; ++q) out_kp[6 * d + q] = slot_kp[6 * s + q];
            const uint4* sd = (const uint4*)(slot_desc + 32 * s);
            uint4* dd = (uint4*)(out_desc + 32 * d);
            dd[0] = sd[0];
            dd[1] = sd[1];
        }
        base += n;
    }
    if (threadIdx.x == 0) out_count[img] = base;
}

// ---- host-side tables (mirrored by oracle/sfm_oracle_orb.c) ------------------------------------

uint64_t sm_next(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int pattern_coord(uint64_t& s) {
    double g = 0.0;
    for (int i = 0; i < 12; ++i) g += (double)(sm_next(s) >> 11) * (1.0 / 9007199254740992.0);
    g -= 6.0;
    const long v = lround(6.2 * g);
    return (int)std::min(13L, std::max(-13L, v));
}

void make_pattern(int32_t* pat) {
    uint64_t s = 0x5EED0B5EULL;
    for (int t = 0; t < 256; ++t) {
        const int x1 = pattern_coord(s), y1 = pattern_coord(s);
        int x2, y2;
        do {
            x2 = pattern_coord(s);
            y2 = pattern_coord(s);
        } while (x2 == x1 && y2 == y1);
        pat[4 * t] = x1; pat[4 * t + 1] = y1; pat[4 * t + 2] = x2; pat[4 * t + 3] = y2;
    }
}

void axis_map(int n_in, int n_out, int32_t* map) {
    const double r = (double)n_in / (double)n_out;
    for (int d = 0; d < n_out; ++d) {
        const double sx = ((double)d + 0.5) * r - 0.5;
        int x0 = (int)floor(sx);
        int w = (int)lround((sx - (double)x0) * 2048.0);
        if (x0 < 0) { x0 = 0; w = 0; }
        int x1 = x0 + 1;
        if (x0 >= n_in - 1) { x0 = n_in - 1; x1 = n_in - 1; w = 0; }
        map[3 * d] = x0; map[3 * d + 1] = x1; map[3 * d + 2] = w;
    }
}

}  // namespace

extern "C" int sfm_orb_batch(sfm_ctx* ctx, const uint8_t* images, int32_t n_img, int32_t H,
                             int32_t W, const sfm_orb_params* prm, float* out_kp,
                             uint8_t* out_desc, int32_t* out_count) {
    SFM_REQUIRE(ctx && prm, "sfm_orb_batch: ctx/prm is NULL");
    SFM_REQUIRE(n_img >= 0 && H >= 0 && W >= 0, "sfm_orb_batch: negative size");
    if (n_img == 0) return SFM_OK;
    SFM_REQUIRE(images && out_kp && out_desc && out_count, "sfm_orb_batch: NULL array");
    SFM_REQUIRE(H >= 1 && W >= 1 && H <= 4095 && W <= 4095,
                "sfm_orb_batch: image size must be 1..4095 x 1..4095");
    SFM_REQUIRE(prm->n_levels >= 1 && prm->n_levels <= MAXLEV,
                "sfm_orb_batch: n_levels must be 1..16");
    SFM_REQUIRE(prm->scale_factor > 1.0, "sfm_orb_batch: scale_factor must be > 1");
    SFM_REQUIRE(prm->n_features >= 1 && prm->fast_threshold >= 0 && prm->fast_threshold < 255,
                "sfm_orb_batch: bad n_features / fast_threshold");
    SFM_REQUIRE(n_img <= 65535, "sfm_orb_batch: at most 65535 images per call");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // levels, per-level budget (oracle_orb_levels), axis maps, pattern
    OrbLevels L{};
    L.nlev = prm->n_levels;
    const int nlev = prm->n_levels, nfeat = prm->n_features;
    double sc = 1.0;
    for (int l = 0; l < nlev; ++l) {
        L.sc[l] = sc;
        L.W[l] = (int32_t)lround((double)W / sc);
        L.H[l] = (int32_t)lround((double)H / sc);
        sc *= prm->scale_factor;
    }
    const double factor = 1.0 / prm->scale_factor;
    double fp = 1.0;
    for (int l = 0; l < nlev; ++l) fp *= factor;
    double nd = (double)nfeat * (1.0 - factor) / (1.0 - fp);
    int sum = 0;
    for (int l = 0; l < nlev - 1; ++l) {
        L.n[l] = (int32_t)lround(nd);
        sum += L.n[l];
        nd *= factor;
    }
    L.n[nlev - 1] = std::max(nfeat - sum, 0);
    int slot = 0, nmap = 0;
    L.off[0] = 0;
    L.rowoff[0] = 0;
    for (int l = 0; l < nlev; ++l) {
        SFM_REQUIRE(L.W[l] >= 1 && L.H[l] >= 1, "sfm_orb_batch: too many levels for the image size");
        // levels with no room inside the border or no budget detect nothing
        if (L.W[l] <= 2 * EDGE || L.H[l] <= 2 * EDGE) L.n[l] = 0;
        SFM_REQUIRE(2 * L.n[l] <= SEL_MAX, "sfm_orb_batch: n_features too large (per-level 2 n_l <= 1024)");
        L.slot[l] = slot;
        slot += L.n[l];
        L.off[l + 1] = L.off[l] + (int64_t)L.W[l] * L.H[l];
        L.rowoff[l + 1] = L.rowoff[l] + L.H[l];
        L.mapx[l] = nmap;
        nmap += L.W[l];
        L.mapy[l] = nmap;
        nmap += L.H[l];
    }
    std::vector<int32_t> host(3 * (size_t)nmap + 1024);
    for (int l = 1; l < nlev; ++l) {
        axis_map(W, L.W[l], host.data() + 3 * (size_t)L.mapx[l]);
        axis_map(H, L.H[l], host.data() + 3 * (size_t)L.mapy[l]);
    }
    make_pattern(host.data() + 3 * (size_t)nmap);
    // workspace: tables | pyramid | blur | score | flags | row counts, positions | candidates |
    // candidate counts | level counts | slots (kp, desc)
    const size_t tot = (size_t)L.off[nlev], nrows = (size_t)L.rowoff[nlev];
    const size_t b_tab = sfm::align_up(sizeof(int32_t) * host.size(), 256);
    const size_t b_img = sfm::align_up(tot * n_img, 256);
    const size_t b_rows = sfm::align_up(sizeof(int32_t) * nrows * n_img, 256);
    const size_t b_cand = sizeof(int32_t) * (size_t)MAXC * nlev * n_img;
    const size_t b_cnt = sfm::align_up(sizeof(int32_t) * (size_t)nlev * n_img, 256);
    const size_t b_skp = sfm::align_up(sizeof(float) * 6 * (size_t)nfeat * n_img, 256);
    const size_t b_sd = sfm::align_up((size_t)32 * nfeat * n_img, 256);
    char* ws = (char*)sfm::workspace(ctx, b_tab + 4 * b_img + 2 * b_rows + b_cand + 2 * b_cnt +
                                              b_skp + b_sd);
    if (!ws) return SFM_ERR_NOMEM;
    int32_t* tab = (int32_t*)ws;
    uint8_t* pyr = (uint8_t*)(ws + b_tab);
    uint8_t* blur = pyr + b_img;
    uint8_t* score = blur + b_img;
    uint8_t* flag = score + b_img;
    int32_t* rowcnt = (int32_t*)(flag + b_img);
    int32_t* rowpos = (int32_t*)((char*)rowcnt + b_rows);
    int32_t* cand = (int32_t*)((char*)rowpos + b_rows);
    int32_t* ncand = (int32_t*)((char*)cand + b_cand);
    int32_t* lvl = (int32_t*)((char*)ncand + b_cnt);
    float* skp = (float*)((char*)lvl + b_cnt);
    uint8_t* sdesc = (uint8_t*)((char*)skp + b_skp);
    SFM_HIP_CHECK(hipMemcpyAsync(tab, host.data(), sizeof(int32_t) * host.size(),
                                 hipMemcpyHostToDevice, st));
    const int32_t* maps = tab;
    const int32_t* pattern = tab + 3 * (size_t)nmap;
    const dim3 gpix((unsigned)((tot + 255) / 256), (unsigned)n_img);
    hipLaunchKernelGGL(orb_pyr_kernel, gpix, dim3(256), 0, st, images, H, W, L, maps, pyr);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_blur_kernel, gpix, dim3(256), 0, st, pyr, L, blur);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_fast_kernel, gpix, dim3(256), 0, st, pyr, L, prm->fast_threshold, score);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_nms_kernel, gpix, dim3(256), 0, st, score, L, flag);
    SFM_HIP_CHECK(hipGetLastError());
    const dim3 grow((unsigned)((nrows + 3) / 4), (unsigned)n_img);
    hipLaunchKernelGGL(orb_rows_kernel, grow, dim3(256), 0, st, 0, flag, score, L, rowcnt,
                       rowpos, cand);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_scan_kernel, dim3(nlev, n_img), dim3(256), 0, st, L, rowcnt, rowpos,
                       ncand);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_rows_kernel, grow, dim3(256), 0, st, 1, flag, score, L, rowcnt,
                       rowpos, cand);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_select_kernel, dim3(nlev, n_img), dim3(256), 0, st, pyr, blur, L,
                       cand, ncand, pattern, nfeat, skp, sdesc, lvl);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_pack_kernel, dim3(n_img), dim3(256), 0, st, L, nfeat, skp, sdesc, lvl,
                       out_kp, out_desc, out_count);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
