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
//   orb_tile_kernel    block per 64 x 32 level tile: pyramid pixels (level 0 copied, level l >= 1
//                      resampled) with a halo in LDS, 7x7 separable Gaussian (fixed point),
//                      FAST-9 score inside the 31-pixel border, strict 3x3 maximum -> pyramid,
//                      blur and the kept scores
//                      and the survivor count of every 64-pixel row segment
//   orb_scan_kernel    block per (image, level): row positions in raster order
//   orb_cand_kernel    wave per level row: the raster-order candidate list (x, y, score packed),
//                      every NMS survivor (round 3: no per-level cap)
//   orb_select_kernel  block per (image, level): FAST-score top 2 n_l by histogram threshold,
//                      Harris, LDS bitonic sort, orientation and descriptors of the n_l best
//   orb_pack_kernel    block per image: levels' slots -> one dense list per image
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "orb_bit_pattern_31.h"
#include "sfm_internal.h"

namespace {

constexpr int EDGE = 31;
constexpr int MAXLEV = 16;
constexpr int SEL_MAX = 1024;    // 2 n_l per level handled by the select kernel
constexpr int RADIUS = 15;

struct OrbLevels {
    int32_t nlev;
    int32_t W[MAXLEV], H[MAXLEV], n[MAXLEV], slot[MAXLEV];  // slot: first output slot of level
    int64_t off[MAXLEV + 1];         // pixel offset of each level in an image's pyramid
    int32_t mapx[MAXLEV], mapy[MAXLEV];  // offsets (entries of 3 ints) into the axis-map table
    int32_t ntx[MAXLEV];              // TW x TH tiles per level row
    int32_t pitch[MAXLEV];            // bytes per level row in pyr / blur / nms (multiple of 64)
    int32_t tileoff[MAXLEV + 1];      // first tile of each level (orb_tile_kernel grid x)
    int64_t segoff[MAXLEV + 1];       // first 64-pixel row segment (row-major: y * ntx + tile x)
    int64_t rowoff[MAXLEV + 1];       // first row of each level (row position arrays)
    int64_t candoff[MAXLEV + 1];      // first candidate slot of each level in an image's list:
                                      // room for every strict 3x3 maximum inside the border,
                                      // ceil((W - 62) / 2) x ceil((H - 62) / 2) (no cap)
    double sc[MAXLEV];
};

__constant__ int c_fast_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int c_fast_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

// ---- fused front end: pyramid, blur, FAST, NMS per 64 x 32 tile ------------------------------
//
// Block per (level tile, image).  The tile's pyramid pixels with a 4-pixel halo are computed once
// into LDS (level 0 copied, level l >= 1 resampled from the image through the axis maps; halo
// coordinates clamped to the level, which is exactly the blur's border rule) and written out for
// the select kernel; the 7x7 blur runs as a horizontal pass into LDS and a vertical pass
// (the same integer sum as the 2-D formula); FAST scores of the tile plus a 1-pixel ring go to
// LDS, and the strict 3x3 maximum writes nms = score where kept, else 0 (one byte array instead
// of score + flag: a kept score is >= 1).  Every value is an integer function of the same inputs
// as oracle/sfm_oracle_orb.c: bit-exact by construction.
constexpr int TW = 64, TH = 32;         // tile (output pixels)
constexpr int PW = TW + 8, PH = TH + 8;  // pyramid tile + 4-pixel halo (FAST 3 + NMS 1)

// FAST-9 scores of two pixels at once (packed i16 lanes: v_pk_min_i16 / v_pk_max_i16) from the 16
// circle differences: best over the 16 arcs of 9 of max(min d, min -d), with the arc minima by
// min of three 3-runs — exactly the spec's arc loop (integer min/max, |d| <= 255).
typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s2 smin(s2 a, s2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ s2 smax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ s2 fast_score2(const s2 (&d)[16]) {
    s2 nd[16], mn3[16], nm3[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) nd[i] = -d[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        mn3[i] = smin(smin(d[i], d[(i + 1) & 15]), d[(i + 2) & 15]);
        nm3[i] = smin(smin(nd[i], nd[(i + 1) & 15]), nd[(i + 2) & 15]);
    }
    s2 best = {0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const s2 b9 = smin(smin(mn3[i], mn3[(i + 3) & 15]), mn3[(i + 6) & 15]);
        const s2 k9 = smin(smin(nm3[i], nm3[(i + 3) & 15]), nm3[(i + 6) & 15]);
        best = smax(best, smax(b9, k9));
    }
    return best;
}

__global__ __launch_bounds__(256) void orb_tile_kernel(const uint8_t* __restrict__ imgs, int H,
                                                       int W, OrbLevels L,
                                                       const int32_t* __restrict__ maps, int thr,
                                                       uint8_t* __restrict__ pyr,
                                                       uint8_t* __restrict__ blur,
                                                       uint8_t* __restrict__ nms,
                                                       int32_t* __restrict__ segcnt) {
    __shared__ __attribute__((aligned(16))) uint8_t P[PH][PW];
    __shared__ __attribute__((aligned(16))) uint16_t Hb[TH + 6][TW];  // horizontal sums <= 65280
    __shared__ __attribute__((aligned(4))) uint8_t S[TH + 2][TW + 4];  // 68-B rows: dword reads
    __shared__ int MX[PW][3], MY[PH][3], GB[PW / 4];
    __shared__ uint32_t MXs[PW][2];  // v_perm selectors of each column's two taps (fast fill)
    // FAST candidate list (phase 3), then the blur / nms output rows (phase 4) in the same bytes
    __shared__ __attribute__((aligned(16))) uint16_t flist[(TH + 2) * (TW + 2)];
    static_assert(sizeof(flist) >= 2 * TH * TW, "blur / nms rows alias the candidate list");
    uint8_t (*Ob)[TW] = (uint8_t (*)[TW])flist;
    uint8_t (*On)[TW] = (uint8_t (*)[TW])((uint8_t*)flist + TH * TW);
    __shared__ int fcount;
    const int tid = threadIdx.x;
    const int t = blockIdx.x;
    int l = 0;
    while (l + 1 < L.nlev && t >= L.tileoff[l + 1]) ++l;
    const int tl = t - L.tileoff[l];
    const int w = L.W[l], h = L.H[l], pw = L.pitch[l];
    const int ty0 = tl / L.ntx[l], tx0 = tl - ty0 * L.ntx[l];
    const int y0 = ty0 * TH, x0 = tx0 * TW;
    const int64_t tot = L.off[L.nlev];
    const size_t ib = (size_t)blockIdx.y * tot + L.off[l];
    const uint8_t* img = imgs + (size_t)blockIdx.y * H * W;
    // the tile's uniform bases: per-lane offsets below are 32-bit
    const size_t tb = ib + (size_t)y0 * pw + x0;
    uint8_t* tpyr = pyr + tb;
    int32_t* tseg = segcnt + (size_t)blockIdx.y * L.segoff[L.nlev] + L.segoff[l] +
                    (int64_t)y0 * L.ntx[l] + tx0;
    // 1. pyramid tile with halo (clamped coordinates), four columns per thread: 720 groups of
    //    4 pixels (18 per row).  Level 0: one dword load per group away from the image border.
    //    Levels >= 1: the group's bilinear taps lie in a 16-byte window of each of its two source
    //    rows (window start GB: its first column's c0, dword-aligned, at most W - 16), so a group
    //    is two 16-byte loads; each pixel's two taps are cut from a window by two v_perm_b32 (the
    //    per-column selectors, lo/hi 8 bytes, set up once per tile) into u16 lanes and weighted
    //    by one v_dot2_u32_u16 - the same integer sum as the per-tap formula.  Tiles whose window
    //    does not hold every tap (large scale factors) or images with W % 4 != 0 take the per-byte
    //    path.
    constexpr int NG = PH * PW / 4, GPR = PW / 4;  // 720 groups, 18 per row
    const bool wal = (W & 3) == 0 && W >= 16;      // dword-aligned rows, a 16-byte window fits
    int slow = 0;
    if (l > 0) {
        int bad = 0;
        for (int k = tid; k < PW + PH; k += 256) {
            if (k < PW) {
                const int cx = min(max(x0 - 4 + k, 0), w - 1);
                const int32_t* m = maps + 3 * (L.mapx[l] + cx);
                const int c0 = m[0], c1 = m[1], wx = m[2];
                MX[k][0] = c0; MX[k][1] = c1; MX[k][2] = wx;
                const int cg = min(max(x0 - 4 + (k & ~3), 0), w - 1);
                const int base = min(maps[3 * (L.mapx[l] + cg)] & ~3, W - 16);
                const int k0 = c0 - base, k1 = c1 - base;
                bad |= (k0 < 0 || k1 > 15) ? 1 : 0;
                const unsigned lo0 = k0 < 8 ? k0 : 12, lo1 = k1 < 8 ? k1 : 12;  // 12: byte 0x00
                const unsigned hi0 = k0 >= 8 ? k0 - 8 : 12, hi1 = k1 >= 8 ? k1 - 8 : 12;
                MXs[k][0] = lo0 | 12u << 8 | lo1 << 16 | 12u << 24;
                MXs[k][1] = hi0 | 12u << 8 | hi1 << 16 | 12u << 24;
                if ((k & 3) == 0) GB[k >> 2] = base;
            } else {  // source rows as byte offsets (< 4095 * 4095 < 2^24)
                const int r = k - PW, cy = min(max(y0 - 4 + r, 0), h - 1);
                const int32_t* m = maps + 3 * (L.mapy[l] + cy);
                MY[r][0] = (int)__umul24((unsigned)m[0], (unsigned)W);
                MY[r][1] = (int)__umul24((unsigned)m[1], (unsigned)W);
                MY[r][2] = m[2];
            }
        }
        slow = __syncthreads_or(bad) || !wal;
    }
    if (l > 0 && !slow) {
        uint32_t A[3][4], B[3][4];
        int gr[3], gcl[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {  // every load issued before any is used
            const int g = min(tid + q * 256, NG - 1);
            gr[q] = g / GPR;
            gcl[q] = g - gr[q] * GPR;
            const uint32_t* pa = (const uint32_t*)(img + (unsigned)MY[gr[q]][0] + (unsigned)GB[gcl[q]]);
            const uint32_t* pb = (const uint32_t*)(img + (unsigned)MY[gr[q]][1] + (unsigned)GB[gcl[q]]);
#pragma unroll
            for (int i = 0; i < 4; ++i) { A[q][i] = pa[i]; B[q][i] = pb[i]; }
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (tid + q * 256 >= NG) continue;
            const unsigned wy = (unsigned)MY[gr[q]][2];
            uint32_t out = 0;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int col = gcl[q] * 4 + m;
                const uint32_t sl = MXs[col][0], sh = MXs[col][1], wx = (uint32_t)MX[col][2];
                const uint32_t ta = __builtin_amdgcn_perm(A[q][1], A[q][0], sl) |
                                    __builtin_amdgcn_perm(A[q][3], A[q][2], sh);
                const uint32_t tb2 = __builtin_amdgcn_perm(B[q][1], B[q][0], sl) |
                                     __builtin_amdgcn_perm(B[q][3], B[q][2], sh);
                const uint32_t wv = (wx << 16) | (2048u - wx);
                const unsigned t0 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, ta),
                                                           __builtin_bit_cast(ushort2_t, wv), 0u, false);
                const unsigned t1 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, tb2),
                                                           __builtin_bit_cast(ushort2_t, wv), 0u, false);
#ifdef ORB_ABL_FILL  // timing-only ablation
                const unsigned v = (t0 + t1) & 255u;
#else
                const unsigned v = (__umul24(t0, 2048u - wy) + __umul24(t1, wy) + (1u << 21)) >> 22;
#endif
                out |= v << (8 * m);
            }
            *(uint32_t*)&P[gr[q]][gcl[q] * 4] = out;
        }
    } else if (l == 0) {
        uint32_t v[3];
        int gr[3], gcl[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int g = min(tid + q * 256, NG - 1);
            gr[q] = g / GPR;
            gcl[q] = g - gr[q] * GPR;
            const int cy = min(max(y0 - 4 + gr[q], 0), h - 1), cx = x0 - 4 + gcl[q] * 4;
            const unsigned ro = __umul24((unsigned)cy, (unsigned)W);
            if (wal && cx >= 0 && cx + 3 < w) {
                v[q] = *(const uint32_t*)(img + ro + (unsigned)cx);
            } else {
                v[q] = 0;
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    v[q] |= (uint32_t)img[ro + (unsigned)min(max(cx + m, 0), w - 1)] << (8 * m);
            }
        }
#pragma unroll
        for (int q = 0; q < 3; ++q)
            if (tid + q * 256 < NG) *(uint32_t*)&P[gr[q]][gcl[q] * 4] = v[q];
    } else {  // per-byte bilinear (windows that do not fit, or W % 4 != 0)
        constexpr int PN = (PH * PW + 255) / 256;
        int v[PN], rr[PN], cc[PN];
        // (row, column) of k = tid + 256 q stepped without divisions: 256 = 3 PW + 40
        rr[0] = tid / PW;
        cc[0] = tid - rr[0] * PW;
#pragma unroll
        for (int q = 1; q < PN; ++q) {
            const int c = cc[q - 1] + (256 - (256 / PW) * PW);
            const bool wrap = c >= PW;
            cc[q] = wrap ? c - PW : c;
            rr[q] = rr[q - 1] + 256 / PW + (wrap ? 1 : 0);
        }
#pragma unroll
        for (int q = 0; q < PN; ++q) {
            const int k = tid + q * 256;
            v[q] = 0;
            if (k < PH * PW) {
                const int r = rr[q], c = cc[q];
                // 32-bit offsets off the image's uniform base; 24-bit products (exact)
                const unsigned o0 = (unsigned)MY[r][0], o1 = (unsigned)MY[r][1];
                const unsigned c0 = (unsigned)MX[c][0], c1 = (unsigned)MX[c][1];
                const unsigned wx = (unsigned)MX[c][2], wy = (unsigned)MY[r][2];
                const unsigned t0 = __umul24(img[o0 + c0], 2048u - wx) + __umul24(img[o0 + c1], wx);
                const unsigned t1 = __umul24(img[o1 + c0], 2048u - wx) + __umul24(img[o1 + c1], wx);
                v[q] = (int)((__umul24(t0, 2048u - wy) + __umul24(t1, wy) + (1u << 21)) >> 22);
            }
        }
#pragma unroll
        for (int q = 0; q < PN; ++q) {
            const int k = tid + q * 256;
            if (k < PH * PW) P[rr[q]][cc[q]] = (uint8_t)v[q];
        }
    }
    __syncthreads();
    // 2. pyramid out; horizontal blur of rows y0-3 .. y0+TH+2.  Every phase below issues the LDS
    //    reads of a batch of pixels before any arithmetic (compile-time trip counts, no data-
    //    dependent branches): the phases are LDS-latency chains otherwise.
    // (rows are pitch-padded to 64 B: a tile row is one aligned 64-B run; dword stores, columns
    //  past the level width land in the padding)
#pragma unroll
    for (int q = 0; q < TH * TW / 1024; ++q) {
        const int k = tid + q * 256, r = k >> 4, c4 = (k & 15) * 4;
        if (y0 + r < h)
            *(uint32_t*)(tpyr + __umul24((unsigned)r, (unsigned)pw) + (unsigned)c4) =
                *(const uint32_t*)&P[r + 4][c4 + 4];
    }
    {   // four outputs per thread from three aligned dwords of the pyramid row: the 7 taps as two
        // v_dot4_u32_u8 over byte windows cut by v_alignbyte (exact integer sums)
        constexpr int HG = (TH + 6) * TW / 4, HN = (HG + 255) / 256;  // 608 groups, 3 passes
        constexpr unsigned CA = 18u | 34u << 8 | 49u << 16 | 54u << 24;  // taps 0-3
        constexpr unsigned CB = 49u | 34u << 8 | 18u << 16;              // taps 4-6 (+ 0)
#pragma unroll
        for (int q = 0; q < HN; ++q) {
            const int g = tid + q * 256;
            if (g < HG) {
                const int r = g >> 4, c4 = (g & 15) * 4;  // output row r = pixel row y0-3+r
                const uint32_t* pr = (const uint32_t*)&P[r + 1][c4];  // P cols c4 .. c4+11
                const uint32_t d0 = pr[0], d1 = pr[1], d2 = pr[2];
#ifdef ORB_ABL_HBLUR  // timing-only ablation: one tap
                const uint4 o = make_uint4(d0 & 255, d1 & 255, d2 & 255, d0 >> 24);
#else
                uint4 o;
                o.x = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 1), CA,
                          __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 1), CB, 0, false), false);
                o.y = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 2), CA,
                          __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 2), CB, 0, false), false);
                o.z = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d1, d0, 3), CA,
                          __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d2, d1, 3), CB, 0, false), false);
                o.w = __builtin_amdgcn_udot4(d1, CA, __builtin_amdgcn_udot4(d2, CB, 0, false), false);
#endif
                *(uint2*)&Hb[r][c4] = make_uint2(o.x | o.y << 16, o.z | o.w << 16);
            }
        }
    }
    // 3. FAST scores of the tile + 1-pixel ring (0 outside the EDGE border).  Compass points 0, 4,
    //    8, 12: every 9-arc holds two of them, so a pixel with fewer than two brighter (or darker)
    //    than thr has best <= thr, score 0 exactly.  Passing pixels (a few % on textured images,
    //    but in most waves) are appended to an LDS list and scored densely, two per lane in the
    //    i16 halves of a register.
    {
        // four pixels per thread (17 groups per ring row; the last group's columns 66, 67 lie
        // outside the ring and never pass): 7 aligned dword reads cover the centres and the four
        // compass points, cut by v_alignbyte; the tests run on i16 pairs (v_pk_sub_i16)
        constexpr int GR = (TW + 4) / 4, FG = (TH + 2) * GR;  // 17, 578
        if (tid == 0) fcount = 0;
        __syncthreads();
        const s2 tp1 = {(short)(thr + 1), (short)(thr + 1)};
#pragma unroll
        for (int q = 0; q < (FG + 255) / 256; ++q) {
            const int g = tid + q * 256;
            if (g >= FG) continue;
            const int r = g / GR, c4 = (g - r * GR) * 4;
            const int py = r + 3;  // P row of the pixels; P cols c4+3 .. c4+6
            const uint32_t* rc = (const uint32_t*)&P[py][c4];
            const uint32_t* ru = (const uint32_t*)&P[py - 3][c4];
            const uint32_t* rd = (const uint32_t*)&P[py + 3][c4];
            const uint32_t d0 = rc[0], d1 = rc[1], d2 = rc[2];
            const uint32_t u0 = ru[0], u1 = ru[1], w0 = rd[0], w1 = rd[1];
            *(uint32_t*)&S[r][c4] = 0u;
#ifdef ORB_ABL_COMPASS  // timing-only ablation: no compass test
            if (thr >= 0) continue;
#endif
            const uint32_t cen = __builtin_amdgcn_alignbyte(d1, d0, 3);
            const uint32_t nbr[4] = {__builtin_amdgcn_alignbyte(w1, w0, 3),   // point 0: row + 3
                                     __builtin_amdgcn_alignbyte(d2, d1, 2),   // point 4: col + 3
                                     __builtin_amdgcn_alignbyte(u1, u0, 3),   // point 8: row - 3
                                     d0};                                     // point 12: col - 3
            unsigned bits = 0;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {  // pixels (2 hf, 2 hf + 1) in the i16 lanes
                const unsigned sel = hf ? 0x0c030c02u : 0x0c010c00u;
                const s2 cv = __builtin_bit_cast(s2, __builtin_amdgcn_perm(0u, cen, sel));
                const s2 cb = cv + tp1, cd = cv - tp1;
                s2 nb = {0, 0}, nd = {0, 0};  // number of compass points NOT brighter / darker
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const s2 nv = __builtin_bit_cast(s2, __builtin_amdgcn_perm(0u, nbr[e], sel));
                    nb += __builtin_bit_cast(s2, __builtin_bit_cast(ushort2_t, nv - cb) >> 15);
                    nd += __builtin_bit_cast(s2, __builtin_bit_cast(ushort2_t, cd - nv) >> 15);
                }
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const int c = c4 + 2 * hf + m;  // ring column of the pixel
                    const int gy = y0 - 1 + r, gx = x0 - 1 + c;
                    const bool inside = c < TW + 2 && gx >= EDGE && gx < w - EDGE &&
                                        gy >= EDGE && gy < h - EDGE;
                    if (inside && (nb[m] <= 2 || nd[m] <= 2)) bits |= 1u << (2 * hf + m);
                }
            }
#ifdef ORB_ABL_FAST  // timing-only ablation: no FAST candidates (compass still computed)
            if (thr >= 0) bits = 0;
#endif
            if (bits) {
                int o = atomicAdd(&fcount, __popc(bits));
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    if (bits & (1u << m)) flist[o++] = (uint16_t)(r * (TW + 2) + c4 + m);
            }
        }
        __syncthreads();
        const int nf = fcount;
        for (int i0 = 2 * tid; i0 < nf; i0 += 512) {
            s2 d[16];
            int kk[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int k = flist[min(i0 + q, nf - 1)];
                kk[q] = k;
                const int r = k / (TW + 2), c = k - r * (TW + 2);
                const int py = r + 3, px = c + 3;
                const int cv = P[py][px];
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    d[e][q] = (short)((int)P[py + c_fast_dy[e]][px + c_fast_dx[e]] - cv);
            }
            const s2 best = fast_score2(d);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (i0 + q >= nf) continue;
                const int k = kk[q], r = k / (TW + 2), c = k - r * (TW + 2);
                const int b = best[q];
                S[r][c] = (uint8_t)(b > thr ? b : 0);
            }
        }
    }
    __syncthreads();
    // 4. vertical blur and the strict 3x3 maximum, four columns per thread (16 threads per 64-pixel
    //    row segment, 16 rows per pass): 7 int4 reads of the horizontal sums and two aligned dwords
    //    of each of 3 score rows; the segment's survivors are counted for the candidate scatter
#pragma unroll
    for (int q = 0; q < TH / 16; ++q) {
        const int r = (tid >> 4) + 16 * q, c4 = (tid & 15) * 4;
        uint2 hp[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) hp[j] = *(const uint2*)&Hb[r + j][c4];
        uint32_t sw[3][2];  // S row r+i, S cols c4 .. c4+7 = tile cols c4-1 .. c4+6
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            sw[i][0] = *(const uint32_t*)&S[r + i][c4];
            sw[i][1] = *(const uint32_t*)&S[r + i][c4 + 4];
        }
        int sb[3][6];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) sb[i][j] = (int)((sw[i][j >> 2] >> (8 * (j & 3))) & 255u);
        uint32_t ob = 0, on = 0;
        int cnt = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            int hm[7];
#pragma unroll
            for (int j = 0; j < 7; ++j) hm[j] = (int)(((m < 2 ? hp[j].x : hp[j].y) >> (16 * (m & 1))) & 0xFFFFu);
#ifdef ORB_ABL_VBLUR  // timing-only ablation: one tap
            const unsigned acc = __umul24((unsigned)hm[3], 256u);
#else
            // hv <= 255 * 256: 24-bit products, the sum < 2^24 (exact)
            const unsigned acc =
                __umul24((unsigned)hm[0], 18u) + __umul24((unsigned)hm[1], 34u) +
                __umul24((unsigned)hm[2], 49u) + __umul24((unsigned)hm[3], 54u) +
                __umul24((unsigned)hm[4], 49u) + __umul24((unsigned)hm[5], 34u) +
                __umul24((unsigned)hm[6], 18u);
#endif
            ob |= ((acc + 32768u) >> 16) << (8 * m);
            const int s0 = sb[1][m + 1];
            const int nmax = max(max(max(sb[0][m], sb[0][m + 1]), max(sb[0][m + 2], sb[1][m])),
                                 max(max(sb[1][m + 2], sb[2][m]), max(sb[2][m + 1], sb[2][m + 2])));
            // strict maximum (a kept score is nonzero: only inside the EDGE border)
            const bool keep = y0 + r < h && x0 + c4 + m < w && s0 != 0 && s0 > nmax;
            on |= (keep ? (uint32_t)s0 : 0u) << (8 * m);
            cnt += keep ? 1 : 0;
        }
        *(uint32_t*)&Ob[r][c4] = ob;
        *(uint32_t*)&On[r][c4] = on;
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off, 16);
        if ((tid & 15) == 0 && y0 + r < h) tseg[__umul24((unsigned)r, (unsigned)L.ntx[l])] = cnt;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TH * TW / 1024; ++q) {
        const int k = tid + q * 256, r = k >> 4, c4 = (k & 15) * 4;
        if (y0 + r < h) {
            const unsigned o = __umul24((unsigned)r, (unsigned)pw) + (unsigned)c4;
            *(uint32_t*)(blur + tb + o) = *(const uint32_t*)&Ob[r][c4];
            *(uint32_t*)(nms + tb + o) = *(const uint32_t*)&On[r][c4];
        }
    }
}

// Wave per level row (4 per block): the row's survivors, packed (y << 20 | x << 8 | score), at
// the row's raster-order position (orb_scan_kernel) + the exclusive sum of its segment counts
// (the tile kernel's, one lane per segment); the segments' bytes are loaded eight at a time.
__global__ __launch_bounds__(256) void orb_cand_kernel(const uint8_t* __restrict__ nms,
                                                       OrbLevels L, const int32_t* __restrict__ segcnt,
                                                       const int32_t* __restrict__ rowpos,
                                                       int32_t* __restrict__ cand) {
    const int lane = threadIdx.x & 63;
    const int64_t rg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (rg >= L.rowoff[L.nlev]) return;  // wave-uniform
    int l = 0;
    while (l + 1 < L.nlev && rg >= L.rowoff[l + 1]) ++l;
    const int y = (int)(rg - L.rowoff[l]);
    const int w = L.W[l], h = L.H[l], ntx = L.ntx[l];
    if (y < EDGE || y >= h - EDGE) return;  // no survivors
    const size_t img = blockIdx.y;
    const int64_t nseg = L.segoff[L.nlev];
    const int sc = lane < ntx ? segcnt[img * nseg + L.segoff[l] + (int64_t)y * ntx + lane] : 0;
    int incl = sc;  // inclusive scan over the row's segments
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
    }
    const int base = rowpos[img * L.rowoff[L.nlev] + rg];
    const uint8_t* row = nms + img * L.off[L.nlev] + L.off[l] + (size_t)y * L.pitch[l];
    int32_t* out = cand + img * L.candoff[L.nlev] + L.candoff[l];
    for (int t0 = 0; t0 < ntx; t0 += 8) {
        int v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int x = (t0 + j) * TW + lane;
            v[j] = (t0 + j < ntx && x < w) ? row[x] : 0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned long long m = __ballot(v[j] != 0);
            if (m == 0ull) continue;  // wave-uniform
            const int sb = __shfl(incl - sc, t0 + j, 64);  // exclusive base of segment t0 + j
            if (v[j] != 0) {
                const int k = base + sb + __popcll(m & ((1ull << lane) - 1ull));
                const int x = (t0 + j) * TW + lane;
                out[k] = (int32_t)(((unsigned)y << 20) | ((unsigned)x << 8) | (unsigned)v[j]);
            }
        }
    }
}

// Block per (image, level): row totals (sum of the row's segment counts), exclusive scan over the
// rows (fixed order) -> row positions, and the level's candidate count (every survivor: the list
// has room for all of them, L.candoff).
__global__ __launch_bounds__(256) void orb_scan_kernel(OrbLevels L, const int32_t* __restrict__ segcnt,
                                                       int32_t* __restrict__ rowpos,
                                                       int32_t* __restrict__ ncand) {
    __shared__ int carry;
    __shared__ int wsum[4];
    const int l = blockIdx.x, tid = threadIdx.x;
    const size_t img = blockIdx.y;
    const int64_t nseg = L.segoff[L.nlev];
    const int ntx = L.ntx[l], h = L.H[l];
    const int32_t* sg = segcnt + img * nseg + L.segoff[l];
    int32_t* rp = rowpos + img * L.rowoff[L.nlev] + L.rowoff[l];
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int y0 = 0; y0 < h; y0 += 256) {
        const int y = y0 + tid;
        int v = 0;
        if (y >= EDGE && y < h - EDGE)
            for (int t = 0; t < ntx; ++t) v += sg[(int64_t)y * ntx + t];
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
    if (tid == 0) ncand[img * L.nlev + l] = carry;
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

// The same value through a reciprocal root computed once per keypoint: |n / sqrt(R2)| <= 18.4 for
// the pattern's points, so n * rinv + 1/2 is within 1e-13 of the exact value; when its fractional
// part is farther than 1e-9 from an integer the floor is already exact, otherwise (rare) the
// integer comparisons decide.
__device__ __forceinline__ int round_div_fast(long long n, long long R2, double rinv) {
    const double t = (double)n * rinv + 0.5;
    const double fl = floor(t), f = t - fl;
    if (f > 1e-9 && f < 1.0 - 1e-9) return (int)fl;
    return round_div(n, R2);
}

// Block per (image, level), SELT threads: the grid is only (levels x images) blocks, so each
// block is one CU's worth of waves — every phase is latency-bound per wave and runs 16-wide.
constexpr int SELT = 1024, SELW = SELT / 64;
__global__ __launch_bounds__(SELT) void orb_select_kernel(
    const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur, OrbLevels L,
    const int32_t* __restrict__ cand, const int32_t* __restrict__ ncand,
    const int32_t* __restrict__ pattern, int nfeat, float* __restrict__ slot_kp,
    uint8_t* __restrict__ slot_desc, int32_t* __restrict__ lvl_count) {
    __shared__ int hist[256];
    __shared__ int s_T, s_above, s_sel, s_ties;
    __shared__ int wcnt[SELW][2];
    __shared__ unsigned sel_c[SEL_MAX];
    __shared__ long long sel_r[SEL_MAX];
    __shared__ int sel_i[SEL_MAX];
    __shared__ int s_pat[1024];
    const int l = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const size_t img = blockIdx.y;
    const int nl = L.n[l];
    const int pw = L.pitch[l];
    if (tid == 0) lvl_count[img * L.nlev + l] = 0;
    if (nl <= 0) return;
    const int nc = ncand[img * L.nlev + l];
    const int32_t* cd = cand + img * L.candoff[L.nlev] + L.candoff[l];
    const int64_t tot = L.off[L.nlev];
    const uint8_t* lv = pyr + img * tot + L.off[l];
    const uint8_t* bl = blur + img * tot + L.off[l];
    for (int k = tid; k < 1024; k += SELT) s_pat[k] = pattern[k];
    // ---- the 2 n_l best FAST scores: histogram threshold, ties in raster order ----
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int k = tid; k < nc; k += SELT) atomicAdd(&hist[cd[k] & 255], 1);
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
    for (int k0 = 0; k0 < nc; k0 += SELT) {
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
            int te = 0, ts = 0;
            for (int q = 0; q < SELW; ++q) { te += wcnt[q][0]; ts += wcnt[q][1]; }
            s_ties += te;
            s_sel += ts;
        }
        __syncthreads();
    }
    const int n1 = min(s_sel, SEL_MAX);
    // ---- Harris response of the selected candidates: wave per candidate, lane per window pixel
    //      (the integer sums are order-free) ----
    int np2 = 1;
    while (np2 < n1) np2 <<= 1;
    for (int k = n1 + tid; k < np2; k += SELT) {
        sel_r[k] = LLONG_MIN;
        sel_i[k] = k;
    }
    for (int k = wv; k < n1; k += SELW) {
        const unsigned c = sel_c[k];
        const int y = (int)(c >> 20), x = (int)((c >> 8) & 4095u);
        int A = 0, B = 0, C = 0;  // |ix|, |iy| <= 1020: 49 squares < 2^31
        if (lane < 49) {
            const int v = lane / 7 - 3, u = lane % 7 - 3;
            const uint8_t* m = lv + (size_t)(y + v) * pw + (x + u);
            const int ix = (m[-pw + 1] + 2 * m[1] + m[pw + 1]) - (m[-pw - 1] + 2 * m[-1] + m[pw - 1]);
            const int iy = (m[pw - 1] + 2 * m[pw] + m[pw + 1]) - (m[-pw - 1] + 2 * m[-pw] + m[-pw + 1]);
            A = ix * ix; B = iy * iy; C = ix * iy;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            A += __shfl_xor(A, off, 64);
            B += __shfl_xor(B, off, 64);
            C += __shfl_xor(C, off, 64);
        }
        if (lane == 0) {
            const long long a = A, b = B, cc = C;
            sel_r[k] = 25 * (a * b - cc * cc) - (a + b) * (a + b);
            sel_i[k] = k;
        }
    }
    __syncthreads();
    // ---- bitonic sort: R descending, raster index ascending ----
    for (int size = 2; size <= np2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int k = tid; k < np2; k += SELT) {
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
    // ---- orientation and descriptor of the n_l best: wave per keypoint (lanes over the disk,
    //      then over the 256 tests: four ballots give the eight descriptor words) ----
    for (int k = wv; k < n2; k += SELW) {
        const unsigned c = sel_c[sel_i[k]];
        const int y = (int)(c >> 20), x = (int)((c >> 8) & 4095u);
        int a10 = 0, a01 = 0;  // |sum| <= 709 * 15 * 255 < 2^31
        for (int e = lane; e < (2 * RADIUS + 1) * (2 * RADIUS + 1); e += 64) {
            const int v = e / (2 * RADIUS + 1) - RADIUS, u = e % (2 * RADIUS + 1) - RADIUS;
            if (u * u + v * v > RADIUS * RADIUS) continue;
            const int I = lv[(size_t)(y + v) * pw + x + u];
            a10 += u * I;
            a01 += v * I;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            a10 += __shfl_xor(a10, off, 64);
            a01 += __shfl_xor(a01, off, 64);
        }
        const long long m10 = a10, m01 = a01;
        const long long R2 = m10 * m10 + m01 * m01;
        const size_t o = img * (size_t)nfeat + L.slot[l] + k;
        if (lane == 0) {
            double ang = atan2((double)m01, (double)m10) * (180.0 / 3.14159265358979323846);
            if (ang < 0.0) ang += 360.0;
            float* kp = slot_kp + 6 * o;
            kp[0] = (float)((double)x * L.sc[l]);
            kp[1] = (float)((double)y * L.sc[l]);
            kp[2] = (float)(31.0 * L.sc[l]);
            kp[3] = (float)ang;
            kp[4] = (float)((double)sel_r[k] / 25.0);
            kp[5] = (float)l;
        }
        const double rinv = R2 == 0 ? 0.0 : 1.0 / sqrt((double)R2);
        unsigned words[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 64 * j + lane;
            int q[4];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const long long px = s_pat[4 * t + 2 * e], py = s_pat[4 * t + 2 * e + 1];
                if (R2 == 0) {
                    q[2 * e] = (int)px;
                    q[2 * e + 1] = (int)py;
                } else {
                    q[2 * e] = round_div_fast(px * m10 - py * m01, R2, rinv);
                    q[2 * e + 1] = round_div_fast(px * m01 + py * m10, R2, rinv);
                }
            }
            const int i1 = bl[(size_t)(y + q[1]) * pw + x + q[0]];
            const int i2 = bl[(size_t)(y + q[3]) * pw + x + q[2]];
            const unsigned long long bits = __ballot(i1 < i2);
            words[2 * j] = (unsigned)bits;
            words[2 * j + 1] = (unsigned)(bits >> 32);
        }
        if (lane == 0) {
            uint4* d = (uint4*)(slot_desc + 32 * o);
            d[0] = make_uint4(words[0], words[1], words[2], words[3]);
            d[1] = make_uint4(words[4], words[5], words[6], words[7]);
        }
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

// OpenCV's learned pattern (generated header, tools/gen_orb_pattern.py).
void make_pattern(int32_t* pat) {
    for (int k = 0; k < 256 * 4; ++k) pat[k] = SFM_ORB_BIT_PATTERN_31[k];
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
    for (int l = 0; l < nlev; ++l) {
        SFM_REQUIRE(L.W[l] >= 1 && L.H[l] >= 1, "sfm_orb_batch: too many levels for the image size");
        // levels with no room inside the border or no budget detect nothing
        if (L.W[l] <= 2 * EDGE || L.H[l] <= 2 * EDGE) L.n[l] = 0;
        SFM_REQUIRE(2 * L.n[l] <= SEL_MAX, "sfm_orb_batch: n_features too large (per-level 2 n_l <= 1024)");
        L.slot[l] = slot;
        slot += L.n[l];
        L.pitch[l] = (L.W[l] + 63) & ~63;
        L.off[l + 1] = L.off[l] + (int64_t)L.pitch[l] * L.H[l];
        L.mapx[l] = nmap;
        nmap += L.W[l];
        L.mapy[l] = nmap;
        nmap += L.H[l];
    }
    int ntile = 0;
    int64_t nseg = 0, nrow = 0;
    for (int l = 0; l < nlev; ++l) {
        L.tileoff[l] = ntile;
        L.segoff[l] = nseg;
        L.rowoff[l] = nrow;
        nrow += L.H[l];
        L.ntx[l] = (L.W[l] + TW - 1) / TW;
        ntile += L.ntx[l] * ((L.H[l] + TH - 1) / TH);
        nseg += (int64_t)L.ntx[l] * L.H[l];
    }
    L.tileoff[nlev] = ntile;
    L.segoff[nlev] = nseg;
    L.rowoff[nlev] = nrow;
    L.candoff[0] = 0;
    for (int l = 0; l < nlev; ++l) {
        const int64_t cx = L.W[l] > 2 * EDGE ? (L.W[l] - 2 * EDGE + 1) / 2 : 0;
        const int64_t cy = L.H[l] > 2 * EDGE ? (L.H[l] - 2 * EDGE + 1) / 2 : 0;
        L.candoff[l + 1] = L.candoff[l] + cx * cy;
    }
    std::vector<int32_t> host(3 * (size_t)nmap + 1024);
    for (int l = 1; l < nlev; ++l) {
        axis_map(W, L.W[l], host.data() + 3 * (size_t)L.mapx[l]);
        axis_map(H, L.H[l], host.data() + 3 * (size_t)L.mapy[l]);
    }
    make_pattern(host.data() + 3 * (size_t)nmap);
    // workspace: tables | pyramid | blur | nms scores | segment counts | row positions | candidates |
    // candidate counts | level counts | slots (kp, desc)
    const size_t tot = (size_t)L.off[nlev];
    const size_t b_tab = sfm::align_up(sizeof(int32_t) * host.size(), 256);
    const size_t b_img = sfm::align_up(tot * n_img, 256);
    const size_t b_rows = sfm::align_up(sizeof(int32_t) * (size_t)nseg * n_img, 256);  // >= rows
    const size_t b_cand = sfm::align_up(sizeof(int32_t) * (size_t)L.candoff[nlev] * n_img, 256);
    const size_t b_cnt = sfm::align_up(sizeof(int32_t) * (size_t)nlev * n_img, 256);
    const size_t b_skp = sfm::align_up(sizeof(float) * 6 * (size_t)nfeat * n_img, 256);
    const size_t b_sd = sfm::align_up((size_t)32 * nfeat * n_img, 256);
    char* ws = (char*)sfm::workspace(ctx, b_tab + 3 * b_img + 2 * b_rows + b_cand + 2 * b_cnt +
                                              b_skp + b_sd);
    if (!ws) return SFM_ERR_NOMEM;
    int32_t* tab = (int32_t*)ws;
    uint8_t* pyr = (uint8_t*)(ws + b_tab);
    uint8_t* blur = pyr + b_img;
    uint8_t* nms = blur + b_img;
    int32_t* segcnt = (int32_t*)(nms + b_img);
    int32_t* rowpos = (int32_t*)((char*)segcnt + b_rows);
    int32_t* cand = (int32_t*)((char*)rowpos + b_rows);
    int32_t* ncand = (int32_t*)((char*)cand + b_cand);
    int32_t* lvl = (int32_t*)((char*)ncand + b_cnt);
    float* skp = (float*)((char*)lvl + b_cnt);
    uint8_t* sdesc = (uint8_t*)((char*)skp + b_skp);
    SFM_HIP_CHECK(hipMemcpyAsync(tab, host.data(), sizeof(int32_t) * host.size(),
                                 hipMemcpyHostToDevice, st));
    const int32_t* maps = tab;
    const int32_t* pattern = tab + 3 * (size_t)nmap;
    hipLaunchKernelGGL(orb_tile_kernel, dim3((unsigned)ntile, (unsigned)n_img), dim3(256), 0, st,
                       images, H, W, L, maps, prm->fast_threshold, pyr, blur, nms, segcnt);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_scan_kernel, dim3(nlev, n_img), dim3(256), 0, st, L, segcnt, rowpos,
                       ncand);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_cand_kernel, dim3((unsigned)((nrow + 3) / 4), (unsigned)n_img), dim3(256),
                       0, st, nms, L, segcnt, rowpos, cand);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_select_kernel, dim3(nlev, n_img), dim3(SELT), 0, st, pyr, blur, L,
                       cand, ncand, pattern, nfeat, skp, sdesc, lvl);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(orb_pack_kernel, dim3(n_img), dim3(256), 0, st, L, nfeat, skp, sdesc, lvl,
                       out_kp, out_desc, out_count);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
