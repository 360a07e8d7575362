// K1, ratio-test path: all-pairs 128-D L2 matching with the Lowe ratio test as a forward scan,
// a recovery step and a reverse scan over the ratio survivors (DESIGN.md §4.1 "forward/reverse").
//
// Same results as the fused kernel in match_mfma.hip and the oracle (oracle/sfm_oracle.c
// oracle_match: lowest-index nearest neighbour, second-smallest distance of the multiset, the
// exact ratio test den^2 d1 < num^2 d2 on squared distances, mutual cross check
// rnn[nn[q]] == q) — the rule restated from code/feature_matching.py:48-58 plus SURVEY.md §8a a3'.
// Used when a ratio test is on and the cross check is mutual or off; the OpenCV cross-check rule
// and ratio-free calls keep the fused kernel.
//
// Why a second path.  The fused kernel is VALU-issue-bound: every element of the
// 2048 x 2048 distance tile pays a key build, the row top-2 and the column side (key, max over
// query tiles, cross-lane transpose).  Here the hot loop keeps only the row top-2, on a value the
// MFMA produces directly:
//     e(q, j) = x'_q . y'_j - ceil(|y'_j|^2 / 2)        (accumulator initialised with -ceil(..))
// vr = 2 x'.y' - |y'|^2 = |x'|^2 - d^2 orders the trains of a query exactly; vr = 2e + p_j with
// p_j = |y'_j|^2 mod 2, so e orders them exactly up to ties in e.  Per query the scan keeps the top
// two e values (e1 >= e2, multiset) and the 32-train tile where e1 first appeared.  Then:
//   * d1 in [A - 2e1 - 1, A - 2e1], d2 in [A - 2e2 - 1, A - 2e2] (A = |x'_q|^2): a query that
//     cannot pass the ratio test even at the favourable ends is dropped (about half of them);
//   * recovery (block per pair): every other query recomputes the 32 dot products of its tile
//     exactly; if e1 > e2 the unique train with e == e1 is the nearest neighbour j1 and d1 is
//     exact; the ratio test is decided exactly unless d2's unit ambiguity straddles it; ties
//     (e1 == e2) and straddles take an exact full-row scan (rare);
//   * reverse scan (mutual only): the same MFMA scan with the survivors' j1 rows as queries and
//     the other image streamed: top-2 of e'(j1, q') = x'_q'.y'_j1 - ceil(|x'_q'|^2 / 2) over q';
//     q is j1's nearest query iff e'(j1, q) == E1 > E2 (E1 == E2 == e'(j1, q): exact column scan).
// MFMA work: 1 + (survivor fraction) of the fused kernel; VALU per element: 1.5 instructions of
// the top-2 network instead of about 4.5 + the transposes.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "match_common.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int D = 128;                       // i8 features per descriptor (x ^ 0x80)
#ifndef L2FR_WAVES
#define L2FR_WAVES 8
#endif
constexpr int WAVES = L2FR_WAVES;            // waves per scan workgroup (8, or 4)
constexpr int SCAN_THREADS = 64 * WAVES;
#ifndef L2FR_QT
#define L2FR_QT 4
#endif
constexpr int QT = L2FR_QT;                  // query tiles (32 queries) per wave: 4, or 2
constexpr int QB = WAVES * QT * 32;          // queries per workgroup (1024 resp. 512)
constexpr int SCAN_MIN_WAVES = 8 / QT;       // waves per SIMD the scan kernel is built for (2 or 4)
#ifndef L2FR_CHUNK
#define L2FR_CHUNK 256
#endif
constexpr int CHUNK = L2FR_CHUNK;            // train rows per LDS stage of the scan (256 or 512)
constexpr int GROUP = 256;                   // train rows per recovery group (8 tiles)
constexpr int NT = CHUNK / 32;               // tiles per stage
constexpr int NK = D / 32;                   // MFMA k-steps per tile (32x32x32 form)
constexpr int SLOTS = D / 16;                // 16-B slots per row
constexpr int PIECES = CHUNK * D / 1024 / WAVES;
constexpr int RPP = 1024 / D;                // rows per 1 KB DMA piece
constexpr int KALIGN = CHUNK > GROUP ? CHUNK : GROUP;
constexpr int KMAX = 4096;
constexpr int PAD_INIT = -(1 << 30);         // accumulator init of a padded train row
constexpr int E_VALID = -(1 << 23);          // e of a real element is > -2^22

enum : unsigned char { ST_DROP = 0, ST_CAND = 1, ST_SLOW = 2, ST_PASS = 3 };

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }  // conflict-free b128 reads

// Top-2 insertion of two values: ts = max(ts, med3(tb, x, y)), tb = max3(tb, x, y).  The median
// is written as max(min(tb,x), min(max(tb,x),y)), which the compiler emits as one v_med3_i32 and
// pads against the MFMA that produced x and y (hipcc does not pad hazards into an asm statement,
// so no asm may read an accumulator first).  The compiler turns max(ts, med) pairs into v_max3.
// The new tb: one asm v_max3_i32 that takes the median as an extra operand, so it issues after
// the compiler's padded read (L2FR_NO_ASM_MAX3: plain max(), which compiles to two v_max_i32).
__device__ __forceinline__ void top2_insert(int& tb, int& ts, int x, int y) {
    const int med = max(min(tb, x), min(max(tb, x), y));
#ifndef L2FR_NO_ASM_MAX3
    int top;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(top) : "v"(tb), "v"(x), "v"(y), "v"(med));
#else
    const int top = max(max(x, y), tb);
#endif
    ts = max(ts, med);
    tb = top;
}

// Exact i8 dot product of two 128-byte feature rows (v_dot4_i32_i8).
__device__ __forceinline__ int dot128(const uint4* x, const uint4* y) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint4 u = x[k], v = y[k];
        s = __builtin_amdgcn_sdot4((int)u.x, (int)v.x, s, false);
        s = __builtin_amdgcn_sdot4((int)u.y, (int)v.y, s, false);
        s = __builtin_amdgcn_sdot4((int)u.z, (int)v.z, s, false);
        s = __builtin_amdgcn_sdot4((int)u.w, (int)v.w, s, false);
    }
    return s;
}

// Per descriptor: the i8 row x ^ 0x80, A = |x'|^2 and the scan's accumulator init -ceil(A/2)
// (PAD_INIT for the padding rows up to k_pad).
__device__ __forceinline__ void prep_one(int img, int j, const uint8_t* __restrict__ desc,
                                         const int32_t* __restrict__ n_kp, int k_max, int k_pad,
                                         int32_t* __restrict__ norm, int32_t* __restrict__ cinit,
                                         uint8_t* __restrict__ zero_row,
                                         uint4* __restrict__ desc_i8) {
    if (img == 0 && j < D) zero_row[j] = 0;
    if (j >= k_pad) return;
    int nv = 0;
    if (j < k_max) {
        const uint4* p = (const uint4*)(desc + ((size_t)img * k_max + j) * D);
        uint4* o8 = desc_i8 + ((size_t)img * k_max + j) * SLOTS;
#pragma unroll
        for (int q = 0; q < SLOTS; ++q) {
            const uint4 v = p[q];
            const uint4 x = make_uint4(v.x ^ 0x80808080u, v.y ^ 0x80808080u, v.z ^ 0x80808080u,
                                       v.w ^ 0x80808080u);
            o8[q] = x;
            // |x'|^2 of the signed bytes x' = x - 128, four at a time (exact integer sums)
            nv = __builtin_amdgcn_sdot4((int)x.x, (int)x.x, nv, false);
            nv = __builtin_amdgcn_sdot4((int)x.y, (int)x.y, nv, false);
            nv = __builtin_amdgcn_sdot4((int)x.z, (int)x.z, nv, false);
            nv = __builtin_amdgcn_sdot4((int)x.w, (int)x.w, nv, false);
        }
    }
    const size_t o = (size_t)img * k_pad + j;
    norm[o] = nv;
    cinit[o] = (j < n_kp[img]) ? -((nv + 1) >> 1) : PAD_INIT;
}

// Pair orders by streamed image, counting sort in LDS: block 0 orders by pairs[p][1] (forward
// scan) into order_f, block 1 by pairs[p][0] (reverse scan) into order_r.
// Block 0 also cuts order_f into recovery ranges: runs of at most REC_R consecutive entries with
// the same train image, rng[r] = (first entry, length), *n_rng of them, and their pairs (rinfo).
constexpr int REC_R = 4;  // pairs (sharing their train image) per recovery block

// The forward scan's UNITS (order block unit_blk of l2fr_setup_kernel): the pairs grouped by query image
// pairs[p][0], UNIT of them per unit (the query fragments are loaded once for all, and each next
// pair's first train chunk is staged under the previous pair's last one); an image's leftover
// pairs make one shorter unit.  uinfo[UNIT u] = (p, a, b, n_kp[a] | n_kp[b] << 16), uinfo[UNIT u + j]
// = (p_j, b_j, n_kp[b_j], 0) for j > 0, p_j = -1 past the unit's pairs; the full units first (by
// query image), then the shorter ones, so the scan's last dispatched blocks are the short ones.
// *n_units = their count.  Which pairs share a unit follows the atomic slot order: it moves no
// result (each pair's records are its own).
#ifndef L2FR_UNIT
#define L2FR_UNIT 2
#endif
constexpr int UNIT = L2FR_UNIT;
__device__ void build_units(const int32_t* __restrict__ pairs, int n_pairs, int n_img,
                            const int32_t* __restrict__ n_kp, int4* __restrict__ uinfo,
                            int32_t* __restrict__ n_units, int* lds) {
    int* cur = lds;                  // [n_img] counts, then slot cursors
    int* fu = lds + n_img;           // [n_img + 1] full units before image i
    int* ru = lds + 2 * n_img + 1;   // [n_img + 1] short units before image i
    __shared__ int ftot;
    const int tid = threadIdx.x;
    for (int i = tid; i < n_img; i += 1024) cur[i] = 0;
    __syncthreads();
    // a pair without queries or trains emits nothing (as its one-pair block exits at once): it
    // joins no unit, so every unit record has rows on both sides
    auto live = [&](int a, int b) { return n_kp[a] > 0 && n_kp[b] > 0; };
    for (int p = tid; p < n_pairs; p += 1024)
        if (live(pairs[2 * p], pairs[2 * p + 1])) atomicAdd(&cur[pairs[2 * p]], 1);
    __syncthreads();
    if (tid == 0) {
        int f = 0, r = 0;
        for (int i = 0; i < n_img; ++i) {
            const int c = cur[i];
            fu[i] = f;
            ru[i] = r;
            f += c / UNIT;
            r += (c % UNIT) != 0;
            cur[i] = 0;
        }
        fu[n_img] = f;
        ru[n_img] = r;
        ftot = f;
        *n_units = f + r;
    }
    __syncthreads();
    // the short units' records start as padding (p = -1); their real pairs overwrite them below
    for (int t = tid; t < ru[n_img] * UNIT; t += 1024) uinfo[(size_t)ftot * UNIT + t] = make_int4(-1, 0, 0, 0);
    __syncthreads();
    for (int p = tid; p < n_pairs; p += 1024) {
        const int a = pairs[2 * p], b = pairs[2 * p + 1];
        if (!live(a, b)) continue;
        const int k = atomicAdd(&cur[a], 1);
        const int nf = UNIT * (fu[a + 1] - fu[a]);
        const int u = k < nf ? fu[a] + k / UNIT : ftot + ru[a];
        const int jj = k < nf ? k % UNIT : k - nf;
        uinfo[(size_t)u * UNIT + jj] = jj ? make_int4(p, b, n_kp[b], 0)
                                          : make_int4(p, a, b, n_kp[a] | (n_kp[b] << 16));
    }
}

__device__ void order_block(int ob, const int32_t* __restrict__ pairs, int n_pairs, int n_img,
                            int32_t* __restrict__ order_f, int32_t* __restrict__ order_r,
                            int2* __restrict__ rng, int32_t* __restrict__ n_rng,
                            const int32_t* __restrict__ n_kp, int4* __restrict__ rinfo,
                            int4* __restrict__ sinfo_f, int unit_blk, int4* __restrict__ uinfo,
                            int32_t* __restrict__ n_units, int* hist) {
    if (ob == unit_blk) {
        build_units(pairs, n_pairs, n_img, n_kp, uinfo, n_units, hist);
        return;
    }
    const int tid = threadIdx.x, col = ob == 0 ? 1 : 0;
    int32_t* order = ob == 0 ? order_f : order_r;
    for (int i = tid; i < n_img; i += 1024) hist[i] = 0;
    __syncthreads();
    for (int p = tid; p < n_pairs; p += 1024) atomicAdd(&hist[pairs[2 * p + col]], 1);
    __syncthreads();
    int* roff = hist + n_img;  // block 0: first recovery range of each train image
    if (tid == 0) {
        int off = 0, nr = 0;
        for (int i = 0; i < n_img; ++i) {
            const int c = hist[i];
            roff[i] = nr;
            nr += (c + REC_R - 1) / REC_R;
            hist[i] = off;
            off += c;
        }
        if (ob == 0) *n_rng = nr;
    }
    __syncthreads();
    if (ob == 0)
        for (int i = tid; i < n_img; i += 1024) {
            const int c = (i + 1 < n_img ? hist[i + 1] : n_pairs) - hist[i];
            for (int k = 0; k < c; k += REC_R)
                rng[roff[i] + k / REC_R] = make_int2(hist[i] + k, min(REC_R, c - k));
        }
    __syncthreads();
    __syncthreads();
    for (int p = tid; p < n_pairs; p += 1024) {
        const int a = pairs[2 * p], b = pairs[2 * p + 1];
        const int slot = atomicAdd(&hist[col ? b : a], 1);
        order[slot] = p;
        // block 0: the forward scan's per-slot pair record, so its blocks start after ONE
        // dependent load instead of the pair_order -> pairs -> n_kp chain
        if (ob == 0) sinfo_f[slot] = make_int4(p, a, b, n_kp[a] | (n_kp[b] << 16));
    }
    if (ob != 0) return;
    // the recovery ranges' pairs: rinfo[r][e] = (p, a, b, n_kp[a] | n_kp[b] << 16), p = -1 past
    // the range's length (order_f and rng come from this block: visible after the barrier)
    __threadfence_block();
    __syncthreads();
    const int nr = *n_rng;
    for (int r = tid; r < nr; r += 1024) {
        const int2 g = rng[r];
#pragma unroll
        for (int e = 0; e < REC_R; ++e) {
            int4 v = make_int4(-1, 0, 0, 0);
            if (e < g.y) {
                const int p = order[g.x + e], a = pairs[2 * p], b = pairs[2 * p + 1];
                v = make_int4(p, a, b, n_kp[a] | (n_kp[b] << 16));
            }
            rinfo[(size_t)r * REC_R + e] = v;
        }
    }
}

// The ratio path's set-up in ONE launch of 1024-thread blocks: blocks [0, n_prep) convert the
// descriptors (prep_one: the i8 rows, |x'|^2, the scan's accumulator init; bpi blocks per image),
// the n_order blocks after them sort the pairs (order_block), concurrently with the conversion —
// the two are independent, and the order blocks' latency-bound serial prefix no longer waits its
// own launch (round 6: prep 10.4 + order 9.0 us as two launches at cfg2).
__global__ __launch_bounds__(1024) void l2fr_setup_kernel(
    int n_prep, int bpi, const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp,
    int k_max, int k_pad, int32_t* __restrict__ norm, int32_t* __restrict__ cinit,
    uint8_t* __restrict__ zero_row, uint4* __restrict__ desc_i8, const int32_t* __restrict__ pairs,
    int n_pairs, int n_img, int32_t* __restrict__ order_f, int32_t* __restrict__ order_r,
    int2* __restrict__ rng, int32_t* __restrict__ n_rng, int4* __restrict__ rinfo,
    int4* __restrict__ sinfo_f, int unit_blk, int4* __restrict__ uinfo,
    int32_t* __restrict__ n_units) {
    extern __shared__ int hist[];
    const int b = (int)blockIdx.x;
    if (b < n_prep) {
        const int img = b / bpi;
        prep_one(img, (b - img * bpi) * 1024 + (int)threadIdx.x, desc, n_kp, k_max, k_pad, norm,
                 cinit, zero_row, desc_i8);
        return;
    }
    order_block(b - n_prep, pairs, n_pairs, n_img, order_f, order_r, rng, n_rng, n_kp, rinfo,
                sinfo_f, unit_blk, uinfo, n_units, hist);
}

// Ratio bounds of one forward record: DROP (cannot pass even at the favourable ends of the d1, d2
// intervals), SLOW (e1 == e2: the nearest neighbour is not unique in e) or CAND.
__device__ __forceinline__ unsigned char classify(int4 r, long long A, int rnum, int rden,
                                                  long long max_dist) {
    const long long d1lo = max(A - 2LL * r.x - 1, 0LL);
    const long long d2hi = r.y > E_VALID ? A - 2LL * r.y : sfm::DIST_INF;
    if (!sfm::ratio_ok(d1lo, d2hi, rnum, rden, true) || (max_dist >= 0 && !(d1lo < max_dist)))
        return ST_DROP;
    return (r.y == r.x) ? ST_SLOW : ST_CAND;
}

// What the forward scan needs to classify its records (unused by the reverse scan).
struct FwdCls {
    const int32_t* norm;     // [n_img][k_pad] |x'|^2
    int rnum, rden;          // ratio num/den
    long long max_dist;
    int4* qst;               // [P][k_pad] DROP / SLOW statuses
    uint8_t* cls;            // [P][k_pad] e1 tile of a candidate (< 128), 0xFF otherwise
};

#ifdef L2FR_CLOCK
// Diagnostic build only (-DL2FR_CLOCK): per forward-scan block, wave 0 stamps (realtime entry,
// realtime after the prologue barrier, memtime there, realtime at the end of each chunk (16),
// memtime and realtime at the loop end, realtime at exit, HW_ID, XCC_ID).
constexpr int L2FR_CLOCK_SLOTS = 1 << 16;
constexpr int L2FR_CLOCK_W = 24;
__device__ unsigned long long g_l2fr_clock[L2FR_CLOCK_W * L2FR_CLOCK_SLOTS];
#define L2FR_STAMP(i, v) \
    if (!REV && tid == 0 && blockIdx.x < L2FR_CLOCK_SLOTS) g_l2fr_clock[L2FR_CLOCK_W * (size_t)blockIdx.x + (i)] = (v)
#else
#define L2FR_STAMP(i, v)
#endif

// The MFMA scan.  Forward (REV = false): queries = image pairs[p][0] rows 0..n-1, streamed trains =
// image pairs[p][1].  Reverse (REV = true): queries = the survivor list's j1 rows of image
// pairs[p][1] (entries 0..qcount[p]-1), streamed = image pairs[p][0].  Output per query entry:
// (e1, e2, tile of e1, 0) at out[p][entry].
//
// Geometry as the fused kernel (match_mfma.hip): 512-thread workgroup = 8 waves x 4 query tiles,
// query fragments in VGPRs for the whole kernel, trains through LDS in 256-row chunks,
// double-buffered LDS-DMA with an XOR-swizzled row image, XCD-aware block order.  Per 32-train
// tile and query tile: 4 MFMAs whose accumulator starts at the trains' -ceil(|y'|^2/2), then the
// top-2 network ts = max(ts, med3(tb, x, y)), tb = max3(tb, x, y) — 1.5 VALU per element, no key
// build, no column side.
template <bool REV>
__global__ __launch_bounds__(SCAN_THREADS, SCAN_MIN_WAVES) void l2fr_scan_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ cinit, const uint8_t* __restrict__ zero_row,
    const int32_t* __restrict__ pairs, int n_qblk, const int32_t* __restrict__ pair_order,
    const int4* __restrict__ sinfo, int n_blk, const int4* __restrict__ qlist,
    const int32_t* __restrict__ qcount, int4* __restrict__ out, FwdCls fc,
    const int32_t* __restrict__ n_units) {
    __shared__ __attribute__((aligned(16))) unsigned char lds0[CHUNK * D + CHUNK * 4];
    __shared__ __attribute__((aligned(16))) unsigned char lds1[CHUNK * D + CHUNK * 4];

    int p, qi, ti, nq, nb, qb;
    int p2 = -1, ti2 = 0, nb2 = 0;   // unit mode: the unit's next pair (same query image)
    int pos = 0, kk = 0;             // unit mode: the unit, the record of the next pair
    if (!REV && n_units) {
        // Unit mode (build_units): a block takes one unit of up to two pairs; units go round-robin
        // over the 8 XCDs (pos = 8 j + blockIdx % 8), all units' query block 0 first, then block
        // 1, the single-pair units last in each pass.  The grid is sized for one pair per unit:
        // the blocks past the units exit at once.
        const int nu = *n_units;
        const int u8 = (nu + 7) >> 3;
        const int l = (int)(blockIdx.x >> 3);
        qb = u8 > 0 ? l / u8 : n_qblk;
        pos = (l - qb * u8) * 8 + (int)(blockIdx.x & 7);
        if (qb >= n_qblk || pos >= nu) return;  // block-uniform, before any barrier
        const int4 u = sinfo[(size_t)UNIT * pos];
        asm volatile("" : : "s"(u.x), "s"(u.y), "s"(u.z), "s"(u.w));
        p = u.x;
        qi = u.y;
        ti = u.z;
        nq = u.w & 0xFFFF;
        nb = u.w >> 16;   // > 0: build_units places only pairs with rows on both sides
    } else {
        // XCD-aware block order: workgroups go round-robin over the 8 XCDs (blockIdx % 8); XCD x
        // owns the x-th contiguous run of ppx pairs of pair_order (pairs sharing the streamed image
        // are adjacent, so its L2 serves them) and runs all their query block 0s first, then block
        // 1s (in the reverse scan most block 1s are empty and exit at once, after the real work).
        const int ppx = (int)(gridDim.x >> 3) / n_qblk;
        const int l = (int)(blockIdx.x >> 3);
        const int pos = (int)(blockIdx.x & 7) * ppx + l % ppx;
        qb = l / ppx;
        if (pos >= n_blk) return;  // block-uniform, before any barrier
        if (REV) {
            p = pair_order[pos];
            qi = pairs[2 * p + 1];
            ti = pairs[2 * p];
            nq = qcount[p];
            nb = n_kp[ti];
        } else {  // one record (order kernel): pair, query image, train image, both counts
            const int4 u = sinfo[pos];
            // all four fields before the early exit: one s_load_dwordx4, not two dependent loads
            asm volatile("" : : "s"(u.x), "s"(u.y), "s"(u.z), "s"(u.w));
            p = u.x;
            qi = u.y;
            ti = u.z;
            nq = u.w & 0xFFFF;
            nb = u.w >> 16;
        }
    }
    if (qb * QB >= nq || nb <= 0) return;  // block-uniform
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    L2FR_STAMP(0, __builtin_amdgcn_s_memrealtime());

    const uint8_t* db = desc + (size_t)ti * k_max * D;
    const int32_t* cib = cinit + (size_t)ti * k_pad;
    int n_chunk = (nb + CHUNK - 1) / CHUNK;
    const uint8_t* db2 = desc;
    const int32_t* cib2 = cinit;
    // unit mode: the unit's pair after record kk (p2 = -1: none)
    auto find_next = [&]() {
        p2 = -1;
        if (REV || !n_units || ++kk >= UNIT) return;
        const int4 v = sinfo[(size_t)UNIT * pos + kk];
        p2 = v.x;
        ti2 = v.y;
        nb2 = v.z;
        db2 = desc + (size_t)ti2 * k_max * D;
        cib2 = cinit + (size_t)ti2 * k_pad;
    };
    find_next();

    // chunk ch of train image (sdb, scib, snb rows) into the LDS stage dst
    auto stage = [&](const uint8_t* sdb, const int32_t* scib, int snb, int ch, unsigned char* dst) {
#pragma unroll
        for (int i = 0; i < PIECES; ++i) {
            const int piece = wave * PIECES + i;
            const int row = piece * RPP + lane / SLOTS;
            const int slot = (lane % SLOTS) ^ swz(row);
            const int j = ch * CHUNK + row;
            const uint8_t* src = (j < snb) ? sdb + (size_t)j * D + slot * 16 : zero_row + slot * 16;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + piece * 1024), 16, 0, 0);
        }
        if (tid < CHUNK / 4) {  // the chunk's accumulator init: whole waves 0 (.. 1)
            const int32_t* src = scib + ch * CHUNK + tid * 4;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + CHUNK * D + wave * 1024),
                                             16, 0, 0);
        }
    };
    // the next stage after chunk ch: this pair's next chunk, or the unit's second pair's first
    auto stage_next = [&](int ch, unsigned char* dst) {
        if (ch + 1 < n_chunk) stage(db, cib, nb, ch + 1, dst);
        else if (p2 >= 0) stage(db2, cib2, nb2, 0, dst);
    };

    const int qbase = qb * QB + wave * QT * 32;
    const bool active = qbase < nq;  // wave-uniform
    const uint8_t* da = desc + (size_t)qi * k_max * D;

    // One query's record (e1, e2, tile of e1) -> out, and the forward scan's ratio classification.
    auto emit = [&](int e, int e1, int e2, int t) {
        const int4 rec = make_int4(e1, e2, t, 0);
        out[(size_t)p * k_pad + e] = rec;
        if (!REV) {  // ratio bounds: drop / slow now, candidates go to the recovery
            const unsigned char st =
                classify(rec, fc.norm[(size_t)qi * k_pad + e], fc.rnum, fc.rden, fc.max_dist);
            fc.cls[(size_t)p * k_pad + e] = st == ST_CAND ? (uint8_t)t : (uint8_t)0xFF;
            if (st != ST_CAND) fc.qst[(size_t)p * k_pad + e] = make_int4(st, 0, 0, 0);
        }
    };

#if L2FR_MFMA16
    // v_mfma_i32_16x16x64_i8 form: the wave's 4*32 queries as 8 subtiles of 16 (B fragments: lane
    // l holds query row l%16, bytes 32*(l/16) + 16*s of k-step s), a 32-train tile as 2 subtiles of
    // 16 (A fragments, same byte map).  Accumulator register r of lane l is train row
    // 16*u + 4*(l/16) + r of the tile, query l%16 of the subtile; lanes l, l^16, l^32, l^48 share a
    // query.  Same matrix cycles per tile (32 MFMAs of 16 instead of 16 of 32).
    constexpr int QS = 2 * QT;
    const int g4 = lane >> 4, r16 = lane & 15;
    v4i bq[QS][2];
    int tb[QS], ts[QS], t1[QS];
#pragma unroll
    for (int c = 0; c < QS; ++c) {
        const int e = qbase + c * 16 + r16;
        int row = -1;
        if (e < nq) row = REV ? qlist[(size_t)p * k_pad + e].y : e;
        const v4i* src = (const v4i*)((row >= 0) ? da + (size_t)row * D + 32 * g4 : zero_row + 32 * g4);
        bq[c][0] = src[0];
        bq[c][1] = src[1];
        tb[c] = INT_MIN; ts[c] = INT_MIN; t1[c] = 0;
    }
    v4i acc[QS][2];
    auto process = [&](int ch, const unsigned char* cur, unsigned char* nxt) __attribute__((always_inline)) {
        stage_next(ch, nxt);
        const int nt = min(NT, (nb - ch * CHUNK + 31) >> 5);
        if (active) {
            const int* Ci = (const int*)(cur + CHUNK * D);
            auto load_tile = [&](int tt, v4i (&af)[2][2], v4i (&init)[2]) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int row = tt * 32 + 16 * u + r16;
                    const int sw = swz(row);
#pragma unroll
                    for (int s = 0; s < 2; ++s)
#ifdef L2FR_ABL_NOLDS
                        af[u][s] = bq[(tt + u + s) & (QS - 1)][s];
#else
                        af[u][s] = *(const v4i*)(cur + row * D + (((2 * g4 + s) ^ sw) << 4));
#endif
#ifdef L2FR_ABL_NOLDS
                    init[u] = v4i{tt, u, tt, u};
#else
                    init[u] = *(const v4i*)(Ci + tt * 32 + 16 * u + 4 * g4);
#endif
                }
            };
            v4i af[2][2], init[2];
            load_tile(0, af, init);
            for (int tt = 0; tt < nt; ++tt) {
                const int gt = ch * NT + tt;
#ifndef L2FR_NO_MPRIO  // the MFMA block at raised priority (its issue wins over the partner's VALU)
                __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int c = 0; c < QS; ++c)
                            acc[c][u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                                af[u][s], bq[c][s], s == 0 ? init[u] : acc[c][u], 0, 0, 0);
#ifndef L2FR_NO_MPRIO
                __builtin_amdgcn_s_setprio(0);
#endif
                if (tt + 1 < nt) load_tile(tt + 1, af, init);
#pragma unroll
                for (int c = 0; c < QS; ++c) {
                    const int o = tb[c];
#ifdef L2FR_ABL_NOEPI
                    tb[c] = max(tb[c], acc[c][0][0] ^ acc[c][1][3]);
#else
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        top2_insert(tb[c], ts[c], acc[c][u][0], acc[c][u][1]);
                        top2_insert(tb[c], ts[c], acc[c][u][2], acc[c][u][3]);
                    }
#endif
                    t1[c] = (tb[c] != o) ? gt : t1[c];
                }
            }
        }
    };
#else
    v4i bq[QT][NK];
    int tb[QT], ts[QT], t1[QT];
#pragma unroll
    for (int c = 0; c < QT; ++c) {
        const int e = qbase + c * 32 + r32;
        int row = -1;
        if (e < nq) row = REV ? qlist[(size_t)p * k_pad + e].y : e;
        const v4i* src = (const v4i*)((row >= 0) ? da + (size_t)row * D + (D / 2) * h
                                                 : zero_row + (D / 2) * h);
#pragma unroll
        for (int s = 0; s < NK; ++s) bq[c][s] = src[s];
        tb[c] = INT_MIN; ts[c] = INT_MIN; t1[c] = 0;
    }

    v16i acc[QT];
    auto epi_all = [&](int gt) {  // top-2 of all query tiles of the tile in acc
#pragma unroll
        for (int u = 0; u < QT; ++u) {
            const int o = tb[u];
#ifdef L2FR_ABL_NOEPI  // ablation: no top-2 network (MFMA + staging cost)
            tb[u] = max(tb[u], acc[u][0] ^ acc[u][15]);
#else
#pragma unroll
            for (int r = 0; r < 16; r += 2) top2_insert(tb[u], ts[u], acc[u][r], acc[u][r + 1]);
#endif
            t1[u] = (tb[u] != o) ? gt : t1[u];
        }
    };

    auto process = [&](int ch, const unsigned char* cur, unsigned char* nxt) __attribute__((always_inline)) {
        stage_next(ch, nxt);
        const int nt = min(NT, (nb - ch * CHUNK + 31) >> 5);
        if (active) {
            const int* Ci = (const int*)(cur + CHUNK * D);
            // A fragments (train rows) and the accumulator init of tile tt; accumulator register r
            // of this lane is train row 8*(r/4) + 4*h + r%4
            auto load_tile = [&](int tt, v4i (&af)[NK], v16i& init) {
                const int row = tt * 32 + r32;
                const int sw = swz(row);
#pragma unroll
                for (int s = 0; s < NK; ++s)
#ifdef L2FR_ABL_NOLDS
                    af[s] = bq[(tt + s) & (QT - 1)][s];
#else
                    af[s] = *(const v4i*)(cur + row * D + ((((SLOTS / 2) * h + s) ^ sw) << 4));
#endif
#pragma unroll
                for (int g = 0; g < 4; ++g) {
#ifdef L2FR_ABL_NOLDS
                    const v4i cv = v4i{tt, g, tt, g};
#else
                    const v4i cv = *(const v4i*)(Ci + tt * 32 + 8 * g + 4 * h);
#endif
                    init[4 * g + 0] = cv.x; init[4 * g + 1] = cv.y;
                    init[4 * g + 2] = cv.z; init[4 * g + 3] = cv.w;
                }
            };
            v4i af[NK];
            v16i init;
            load_tile(0, af, init);
            for (int tt = 0; tt < nt; ++tt) {
                const int gt = ch * NT + tt;
#ifndef L2FR_NO_MPRIO
                __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
                for (int s = 0; s < NK; ++s)
#pragma unroll
                    for (int c = 0; c < QT; ++c)
                        acc[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[c][s],
                                                                        s == 0 ? init : acc[c], 0, 0, 0);
#ifndef L2FR_NO_MPRIO
                __builtin_amdgcn_s_setprio(0);
#endif
                if (tt + 1 < nt) load_tile(tt + 1, af, init);
                epi_all(gt);
            }
        }
    };
#endif

    // the pair's records: top-2 of the lane halves / quarters, then emit
    auto epilogue = [&]() {
#if L2FR_MFMA16
#pragma unroll
        for (int c = 0; c < QS; ++c) {
            // lanes l, l^16, l^32, l^48 hold four row groups of every tile of the same query
            int e1 = tb[c], e2 = ts[c], t = t1[c];
#pragma unroll
            for (int m = 16; m <= 32; m <<= 1) {
                const int P1 = __shfl_xor(e1, m), P2 = __shfl_xor(e2, m), PT = __shfl_xor(t, m);
                e2 = max(min(e1, P1), max(e2, P2));
                t = e1 > P1 ? t : (P1 > e1 ? PT : min(t, PT));
                e1 = max(e1, P1);
            }
            const int e = qbase + c * 16 + r16;
            if (g4 == 0 && e < nq) emit(e, e1, e2, t);
            tb[c] = INT_MIN; ts[c] = INT_MIN; t1[c] = 0;
        }
#else
#pragma unroll
        for (int c = 0; c < QT; ++c) {
            // lanes l and l^32 hold the two 16-row halves of every tile of the same query
            const int P1 = __shfl_xor(tb[c], 32), P2 = __shfl_xor(ts[c], 32),
                      PT = __shfl_xor(t1[c], 32);
            const int e1 = max(tb[c], P1);
            const int e2 = max(min(tb[c], P1), max(ts[c], P2));
            const int t = tb[c] > P1 ? t1[c] : (P1 > tb[c] ? PT : min(t1[c], PT));
            const int e = qbase + c * 32 + r32;
            if (h == 0 && e < nq) emit(e, e1, e2, t);
            tb[c] = INT_MIN; ts[c] = INT_MIN; t1[c] = 0;   // a unit's second pair starts afresh
        }
#endif
    };

    if (n_chunk > 0) stage(db, cib, nb, 0, lds0);
    __syncthreads();
    L2FR_STAMP(1, __builtin_amdgcn_s_memrealtime());
    L2FR_STAMP(2, __builtin_amdgcn_s_memtime());
    // the chunks of the unit's pairs in turn through the two LDS stages (g: the stage parity over
    // the whole unit); a pair's records leave after its last chunk, the next pair's first chunk
    // already staged
    // one pair's chunks two at a time, from stage s0 (the other one s1): static LDS addresses
    auto run_pair = [&](unsigned char* s0, unsigned char* s1) __attribute__((always_inline)) {
        for (int ch = 0; ch < n_chunk; ch += 2) {
            process(ch, s0, s1);
            __syncthreads();
            if (ch < 16) L2FR_STAMP(3 + ch, __builtin_amdgcn_s_memrealtime());
            if (ch + 1 < n_chunk) process(ch + 1, s1, s0);
            __syncthreads();
            if (ch + 1 < 16) L2FR_STAMP(4 + ch, __builtin_amdgcn_s_memrealtime());
        }
    };
    int g = 0;   // the stage that holds the pair's first chunk
    for (;;) {
        if (g & 1)
            run_pair(lds1, lds0);
        else
            run_pair(lds0, lds1);
        g += n_chunk;
        L2FR_STAMP(19, __builtin_amdgcn_s_memtime());
        L2FR_STAMP(20, __builtin_amdgcn_s_memrealtime());
        if (active) epilogue();
        if (p2 < 0) break;
        p = p2;
        ti = ti2;
        nb = nb2;
        db = db2;
        cib = cib2;
        n_chunk = (nb + CHUNK - 1) / CHUNK;
        find_next();
    }
#ifdef L2FR_CLOCK
    L2FR_STAMP(21, __builtin_amdgcn_s_memrealtime());
    L2FR_STAMP(22, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4));   // HW_ID
    L2FR_STAMP(23, (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20));  // XCC_ID
#endif
}

// Exact (d1, j1, d2) of one query over all trains (multiset second, lowest-index j1), block-wide.
// Returns through LDS slot `res` (valid for every thread after the call).
struct Top2 { long long b1; int j1; long long b2; };

__device__ __forceinline__ Top2 top2_merge(Top2 x, Top2 y) {
    const bool xf = (x.b1 < y.b1) || (x.b1 == y.b1 && x.j1 < y.j1);
    Top2 r;
    r.b1 = xf ? x.b1 : y.b1;
    r.j1 = xf ? x.j1 : y.j1;
    r.b2 = min(min(x.b2, y.b2), xf ? y.b1 : x.b1);
    return r;
}

__device__ Top2 exact_row_scan(const uint4* qrow, const uint8_t* db, const int32_t* normb, int nb,
                               int qnorm, Top2* red) {
    const int tid = threadIdx.x;
    uint4 x[SLOTS];
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) x[s] = qrow[s];
    Top2 m{sfm::DIST_INF, INT_MAX, sfm::DIST_INF};
    for (int j = tid; j < nb; j += 256) {
        const int dot = dot128(x, (const uint4*)(db + (size_t)j * D));
        const long long d = (long long)qnorm + normb[j] - 2LL * dot;
        m = top2_merge(m, Top2{d, j, sfm::DIST_INF});
    }
    red[tid] = m;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) red[tid] = top2_merge(red[tid], red[tid + s]);
        __syncthreads();
    }
    const Top2 r = red[0];
    __syncthreads();
    return r;
}

// Ordered compaction of int4 records (block of 256), returns the new base.
__device__ __forceinline__ int compact_rec(bool keep, int4 rec, int base, int* wsum, int4* dst) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long bal = __ballot(keep);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; ++w) {
        const int s = wsum[w];
        off += (w < wave) ? s : 0;
        tot += s;
    }
    if (keep) dst[base + off + pre] = rec;
    __syncthreads();
    return base + tot;
}

// Recovery (block of 256 per (pair, group of 8 train tiles)).  The group's 256 train rows (with
// their accumulator init and |y'|^2) are staged in LDS, slot-swizzled for conflict-free
// row-per-lane reads; the candidates of the group (cls == group, written by the forward scan) are
// processed in batches of 64 whose query rows and records are staged too, so the only global
// traffic is a few bulk loads per block.  Per candidate, 32 lanes (one train each) recompute the
// tile's dot products exactly, the unique train with e == e1 is the nearest neighbour j1, and the
// ratio test is decided exactly where d2's unit ambiguity allows: qst[p][q] = (status, j1, d1).
__global__ __launch_bounds__(256) void l2fr_recover_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ cinit,
    const int32_t* __restrict__ pairs, const int4* __restrict__ fwd,
    const uint8_t* __restrict__ cls, int rnum, int rden, long long max_dist,
    int4* __restrict__ qst) {
    __shared__ uint4 tiles[GROUP * SLOTS];   // 256 train rows, slot s of row r at s ^ (r & 7)
    __shared__ int tci[GROUP], tnb[GROUP];   // their accumulator init and |y'|^2
    __shared__ uint4 qrows[64 * SLOTS];      // a batch of 64 candidate query rows
    __shared__ int4 crec[64];
    __shared__ int cq[64], cA[64];
    __shared__ short clist[KMAX];
    __shared__ int ccount;
    const int p = blockIdx.x, grp = blockIdx.y, tid = threadIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int ntiles = (nb + 31) >> 5, tg = grp * 8;
    if (na <= 0 || nb <= 0 || tg >= ntiles) return;  // block-uniform
    const int4* fw = fwd + (size_t)p * k_pad;
    int4* qs = qst + (size_t)p * k_pad;
    const uint4* qa = (const uint4*)(desc + (size_t)a * k_max * D);
    const uint4* db = (const uint4*)(desc + (size_t)b * k_max * D);

    // bulk loads first (one round trip): train rows, their tables, the candidate classes
    uint4 rv[SLOTS];
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) {
        const int i = tid + 256 * k, j = tg * 32 + i / SLOTS;
        rv[k] = (j < nb) ? db[(size_t)j * SLOTS + i % SLOTS] : make_uint4(0, 0, 0, 0);
    }
    const int tj = tg * 32 + tid;  // < k_pad: groups cover 256 rows, k_pad is a multiple of 256
    const int ci = cinit[(size_t)b * k_pad + tj], nn = norm[(size_t)b * k_pad + tj];
    uint4 cv = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    if (tid * 16 < na) cv = ((const uint4*)(cls + (size_t)p * k_pad))[tid];
    if (tid == 0) ccount = 0;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) {
        const int i = tid + 256 * k, r = i / SLOTS, sl = i % SLOTS;
        tiles[r * SLOTS + (sl ^ (r & 7))] = rv[k];
    }
    tci[tid] = ci;
    tnb[tid] = nn;
    __syncthreads();
    const unsigned cw[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int q = tid * 16 + k;
        if (q < na && ((cw[k >> 2] >> (8 * (k & 3))) & 0xFF) >> 3 == (unsigned)grp)
            clist[atomicAdd(&ccount, 1)] = (short)q;
    }
    __syncthreads();
    const int nc = ccount;
    const int g = tid >> 5, t = tid & 31;
    for (int c0 = 0; c0 < nc; c0 += 64) {
        const int nbat = min(64, nc - c0);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int i = tid + 256 * k, c = i / SLOTS;
            if (c < nbat) qrows[i] = qa[(size_t)clist[c0 + c] * SLOTS + i % SLOTS];
        }
        if (tid < nbat) {
            const int q = clist[c0 + tid];
            cq[tid] = q;
            crec[tid] = fw[q];
            cA[tid] = norm[(size_t)a * k_pad + q];
        }
        __syncthreads();
        for (int c = g; c < nbat; c += 8) {
            const int q = cq[c];
            const int4 r = crec[c];
            const int row = (r.z - tg) * 32 + t, j = r.z * 32 + t;
            const uint4* x = &qrows[c * SLOTS];
            const uint4* y = &tiles[row * SLOTS];
            int dot = 0;
#pragma unroll
            for (int k = 0; k < SLOTS; ++k) {
                const uint4 u = x[k], v = y[k ^ (row & 7)];
                dot = __builtin_amdgcn_sdot4((int)u.x, (int)v.x, dot, false);
                dot = __builtin_amdgcn_sdot4((int)u.y, (int)v.y, dot, false);
                dot = __builtin_amdgcn_sdot4((int)u.z, (int)v.z, dot, false);
                dot = __builtin_amdgcn_sdot4((int)u.w, (int)v.w, dot, false);
            }
            const bool hit = (j < nb) && (dot + tci[row] == r.x);
            const unsigned long long bal = __ballot(hit);
            const unsigned m = (unsigned)(bal >> (32 * (g & 1)));
            if (t == 0 && m == 0) qs[q] = make_int4(ST_SLOW, 0, 0, 0);  // defensive
            if (m != 0 && t == __builtin_ctz(m)) {
                const long long A = cA[c];
                const long long d1 = A - (2LL * dot - tnb[row]);
                const long long d2lo = r.y > E_VALID ? A - 2LL * r.y - 1 : sfm::DIST_INF;
                const long long d2hi = r.y > E_VALID ? A - 2LL * r.y : sfm::DIST_INF;
                int st;
                if (max_dist >= 0 && !(d1 < max_dist)) st = ST_DROP;
                else if (sfm::ratio_ok(d1, d2lo, rnum, rden, true)) st = ST_PASS;
                else if (!sfm::ratio_ok(d1, d2hi, rnum, rden, true)) st = ST_DROP;
                else st = ST_SLOW;
                qs[q] = make_int4(st, j, (int)d1, 0);
            }
        }
        __syncthreads();
    }
}

// Recovery, MFMA form: one block of 256 (4 waves) per (range of up to REC_R pairs that share
// their train image b, group of 8 train tiles of b).  A gather: ~1.2 M candidates at cfg2, each
// needing its query row and one 32-train tile, so the kernel is built for few dependent round
// trips (3), one load of b's train rows per REC_R pairs, no LDS atomics and no LDS staging of
// query rows:
//   1. the range's pairs (rinfo); then one round of independent loads: the pairs' candidate
//      classes (cls, written by the forward scan: the e1 tile of a candidate), wave w's train
//      tiles 2w, 2w+1 of the group as A fragments, the group's accumulator inits
//      -ceil(|y'|^2/2) and norm parities (LDS);
//   2. the group's candidates of all the pairs, sorted by tile (a block prefix sum of packed
//      per-thread tile counts): wave w's are those of its two tiles;
//   3. per wave, one round of loads for up to 4 sub-batches of 32 of its candidates: query rows
//      straight into B fragments, forward records and |x'|^2; per sub-batch e = x'.y' -
//      ceil(|y'|^2/2) for the 2 tiles x 32 candidates (8 MFMAs: ~1 % of the scan's matrix work).
// A candidate's nearest neighbour j1 is the unique train of its e1 tile with e == e1 (e1 > e2 for
// every candidate); the lane finds the row by compares, d1 = |x'|^2 - 2 e1 - (|y'_j1|^2 mod 2)
// exactly, and the ratio test is decided exactly where d2's unit ambiguity allows:
// qst[p][q] = (status, j1, d1).
#ifndef L2FR_REC_SB
#define L2FR_REC_SB 2
#endif
constexpr int REC_SB = L2FR_REC_SB;  // sub-batches of 32 candidates per wave and load round
__global__ __launch_bounds__(256, REC_SB > 2 ? 2 : 3) void l2fr_recover_mfma_kernel(
    const uint8_t* __restrict__ desc, int k_max, int k_pad, const int32_t* __restrict__ norm,
    const int32_t* __restrict__ cinit, const int4* __restrict__ rinfo,
    const int32_t* __restrict__ n_rng, const int4* __restrict__ fwd,
    const uint8_t* __restrict__ cls, int rnum, int rden, long long max_dist,
    int4* __restrict__ qst) {
    __shared__ unsigned short clist[REC_R * KMAX];  // (pair in range) << 12 | query, by tile
    __shared__ __attribute__((aligned(16))) int gini[GROUP];
    __shared__ unsigned char gpar[GROUP];
    __shared__ unsigned long long wlo[4], whi[4];
    __shared__ int toff[9];
    const int ri = blockIdx.x, grp = blockIdx.y, tid = threadIdx.x;
    if (ri >= *n_rng) return;  // block-uniform
    const int wave = tid >> 6, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    int4 pi[REC_R];
#pragma unroll
    for (int e = 0; e < REC_R; ++e) pi[e] = rinfo[(size_t)ri * REC_R + e];
    const int b = pi[0].z, nb = pi[0].w >> 16;
    const int ntiles = (nb + 31) >> 5, tg = grp * 8;
    if (nb <= 0 || tg >= ntiles) return;  // block-uniform
    const uint8_t* db = desc + (size_t)b * k_max * D;

    // 1. independent loads
    uint4 cv[REC_R];
#pragma unroll
    for (int e = 0; e < REC_R; ++e) {
        cv[e] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (pi[e].x >= 0 && tid * 16 < (pi[e].w & 0xFFFF))
            cv[e] = ((const uint4*)(cls + (size_t)pi[e].x * k_pad))[tid];
    }
    v4i af[2][NK];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int row = (tg + 2 * wave + u) * 32 + r32;
#pragma unroll
        for (int s = 0; s < NK; ++s)
            af[u][s] = row < nb ? *(const v4i*)(db + (size_t)row * D + 64 * h + 16 * s) : v4i{0, 0, 0, 0};
    }
    {
        const size_t o = (size_t)b * k_pad + tg * 32 + tid;  // < k_pad: k_pad is a multiple of 256
        gini[tid] = cinit[o];
        gpar[tid] = (unsigned char)(norm[o] & 1);
    }
    // 2. the group's candidates by tile, in (pair, query) order within a tile: a SWAR byte match
    //    gives each thread its candidate mask (cls >> 3 == group), per-thread tile counts packed
    //    as 16-bit fields (tiles 0-3 in lo, 4-7 in hi), one block prefix sum
    unsigned msk[REC_R];
    unsigned long long lo = 0, hi = 0;
    const unsigned g8 = 0x01010101u * ((unsigned)grp << 3);
#pragma unroll
    for (int e = 0; e < REC_R; ++e) {
        const int na = pi[e].x >= 0 ? (pi[e].w & 0xFFFF) : 0;
        const unsigned cw[4] = {cv[e].x, cv[e].y, cv[e].z, cv[e].w};
        unsigned m = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned t = (cw[k] ^ g8) & 0xF8F8F8F8u;                      // 0 byte: match
            const unsigned nz = ((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t;           // bit 7: byte != 0
            const unsigned z = ~nz & 0x80808080u;
            m |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
        }
        const int lim = na - tid * 16;   // queries past na are not candidates
        m &= lim >= 16 ? 0xFFFFu : (lim <= 0 ? 0u : (1u << lim) - 1u);
        msk[e] = m;
        for (unsigned mm = m; mm; mm &= mm - 1) {
            const int k = __builtin_ctz(mm);
            const unsigned c = (cw[k >> 2] >> (8 * (k & 3))) & 7u;
            const unsigned long long one = 1ull << (16 * (c & 3));
            if (c & 4) hi += one; else lo += one;
        }
    }
    unsigned long long plo = lo, phi = hi;  // inclusive wave prefix
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long vl = __shfl_up(plo, d), vh = __shfl_up(phi, d);
        if (lane >= d) { plo += vl; phi += vh; }
    }
    if (lane == 63) { wlo[wave] = plo; whi[wave] = phi; }
    __syncthreads();
    unsigned long long blo = 0, bhi = 0, tlo = 0, thi = 0;  // before this wave; block totals
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        blo += w < wave ? wlo[w] : 0ull;
        bhi += w < wave ? whi[w] : 0ull;
        tlo += wlo[w];
        thi += whi[w];
    }
    // this thread's first slot per tile, packed as 16-bit fields like the counts
    unsigned long long slo = 0, shi = 0;
    {
        int o = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const unsigned long long tot = t < 4 ? tlo : thi, bef = t < 4 ? blo : bhi,
                                     mine = t < 4 ? plo - lo : phi - hi;
            const int sh = 16 * (t & 3);
            const unsigned long long v =
                (unsigned long long)(o + (int)((bef >> sh) & 0xFFFF) + (int)((mine >> sh) & 0xFFFF)) << sh;
            if (t < 4) slo |= v; else shi |= v;
            if (tid == 0) toff[t] = o;
            o += (int)((tot >> sh) & 0xFFFF);
        }
        if (tid == 0) toff[8] = o;
    }
#pragma unroll
    for (int e = 0; e < REC_R; ++e) {
        const unsigned cw[4] = {cv[e].x, cv[e].y, cv[e].z, cv[e].w};
        for (unsigned mm = msk[e]; mm; mm &= mm - 1) {
            const int k = __builtin_ctz(mm);
            const unsigned c = (cw[k >> 2] >> (8 * (k & 3))) & 7u;
            const int sh = 16 * (c & 3);
            const unsigned long long cur = (c & 4) ? shi : slo, inc = 1ull << sh;
            clist[(int)((cur >> sh) & 0xFFFF)] = (unsigned short)((e << 12) | (tid * 16 + k));
            if (c & 4) shi += inc; else slo += inc;
        }
    }
    __syncthreads();
    // 3. this wave's candidates: those of tiles 2w, 2w+1
    const int w0 = toff[2 * wave], w1 = toff[2 * wave + 2];
    const int t0 = tg + 2 * wave;
    for (int c0 = w0; c0 < w1; c0 += 32 * REC_SB) {
        v4i bf[REC_SB][NK];
        int4 rc[REC_SB];
        int qq[REC_SB], pp[REC_SB], AA[REC_SB];
#pragma unroll
        for (int k = 0; k < REC_SB; ++k) {
            const int c = c0 + 32 * k + r32;
            qq[k] = -1;
            if (c < w1) {
                const int en = clist[c], e = en >> 12, q = en & 0xFFF;
                int p = pi[0].x, a = pi[0].y;
#pragma unroll
                for (int f = 1; f < REC_R; ++f) {
                    p = e == f ? pi[f].x : p;
                    a = e == f ? pi[f].y : a;
                }
                const uint8_t* xr = desc + ((size_t)a * k_max + q) * D + 64 * h;
#pragma unroll
                for (int s = 0; s < NK; ++s) bf[k][s] = *(const v4i*)(xr + 16 * s);
                rc[k] = fwd[(size_t)p * k_pad + q];
                AA[k] = norm[(size_t)a * k_pad + q];
                qq[k] = q;
                pp[k] = p;
            } else {
#pragma unroll
                for (int s = 0; s < NK; ++s) bf[k][s] = v4i{0, 0, 0, 0};
                rc[k] = make_int4(0, 0, -1, 0);
            }
        }
#pragma unroll
        for (int k = 0; k < REC_SB; ++k) {
            if (c0 + 32 * k >= w1) break;  // wave-uniform
            const int4 r = rc[k];
            const int mine = r.z - t0;  // 0 / 1: the candidate's tile (always one of the wave's)
            int hit = -1;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                v16i acc;
                const int* gi = gini + (2 * wave + u) * 32 + 4 * h;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const v4i c4 = *(const v4i*)(gi + 8 * g);
                    acc[4 * g + 0] = c4.x; acc[4 * g + 1] = c4.y;
                    acc[4 * g + 2] = c4.z; acc[4 * g + 3] = c4.w;
                }
#pragma unroll
                for (int s = 0; s < NK; ++s)
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[u][s], bf[k][s], acc, 0, 0, 0);
#pragma unroll
                for (int rr = 0; rr < 16; ++rr)
                    hit = (mine == u && acc[rr] == r.x) ? 8 * (rr >> 2) + 4 * h + (rr & 3) : hit;
            }
            hit = max(hit, __shfl_xor(hit, 32));
            if (h == 0 && qq[k] >= 0) {
                int4* qs = qst + (size_t)pp[k] * k_pad;
                if (hit < 0) {
                    qs[qq[k]] = make_int4(ST_SLOW, 0, 0, 0);  // defensive
                } else {
                    const int jg = (2 * wave + mine) * 32 + hit;  // row in the group
                    const long long A = AA[k];
                    const long long d1 = A - 2LL * r.x - gpar[jg];
                    const long long d2lo = r.y > E_VALID ? A - 2LL * r.y - 1 : sfm::DIST_INF;
                    const long long d2hi = r.y > E_VALID ? A - 2LL * r.y : sfm::DIST_INF;
                    int st;
                    if (max_dist >= 0 && !(d1 < max_dist)) st = ST_DROP;
                    else if (sfm::ratio_ok(d1, d2lo, rnum, rden, true)) st = ST_PASS;
                    else if (!sfm::ratio_ok(d1, d2hi, rnum, rden, true)) st = ST_DROP;
                    else st = ST_SLOW;
                    qs[qq[k]] = make_int4(st, tg * 32 + jg, (int)d1, 0);
                }
            }
        }
    }
}

// Exact full-row scans for the SLOW queries (ties in e, straddled ratio decisions: rare), then the
// ordered compaction of the survivors (q, j1, d1, 0) into surv[p][0..scount[p]-1] (block of 256
// per pair).
__global__ __launch_bounds__(256) void l2fr_compact_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ pairs,
    const int4* __restrict__ qst, int rnum, int rden, long long max_dist,
    int4* __restrict__ surv, int32_t* __restrict__ scount, int32_t* __restrict__ out_count,
    int32_t* __restrict__ out_match, int32_t* __restrict__ out_dist) {
    __shared__ Top2 red[256];
    __shared__ int slow[256];
    __shared__ int nslow, wsum[8];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    // out_count != nullptr (the ratio rule without cross check): the survivors ARE the output —
    // the final kernel's copy of them in the same order, written here instead of surv
    const bool direct = out_count != nullptr;
    int32_t* om = direct ? out_match + (size_t)p * k_max * 2 : nullptr;
    int32_t* od = direct ? out_dist + (size_t)p * k_max : nullptr;
    if (na <= 0 || nb <= 0) {
        if (tid == 0) {
            if (direct) out_count[p] = 0;
            else scount[p] = 0;
        }
        return;
    }
    const int4* qs = qst + (size_t)p * k_pad;
    const int32_t* na_norm = norm + (size_t)a * k_pad;
    const int32_t* nb_norm = norm + (size_t)b * k_pad;
    const uint4* qa = (const uint4*)(desc + (size_t)a * k_max * D);
    const uint8_t* db = desc + (size_t)b * k_max * D;
    int4* sv = surv + (size_t)p * k_pad;
    int base = 0;
    for (int q0 = 0; q0 < na; q0 += 256) {
        const int q = q0 + tid;
        int4 r = (q < na) ? qs[q] : make_int4(ST_DROP, 0, 0, 0);
        if (tid == 0) nslow = 0;
        __syncthreads();
        if (r.x == ST_SLOW) slow[atomicAdd(&nslow, 1)] = tid;
        __syncthreads();
        const int ns = nslow;
        for (int i = 0; i < ns; ++i) {
            const int who = slow[i], qq = q0 + who;
            const Top2 e = exact_row_scan(qa + (size_t)qq * SLOTS, db, nb_norm, nb, na_norm[qq], red);
            if (tid == who) {
                bool keep = sfm::ratio_ok(e.b1, e.b2, rnum, rden, true);
                keep = keep && (max_dist < 0 || e.b1 < max_dist);
                r = make_int4(keep ? ST_PASS : ST_DROP, e.j1, (int)e.b1, 0);
            }
        }
        const bool keep = r.x == ST_PASS;
        if (direct)
            base = sfm::compact256(keep, q, r.y, r.z, base, wsum, om, od);
        else
            base = compact_rec(keep, make_int4(q, r.y, r.z, 0), base, wsum, sv);
    }
    if (tid == 0) {
        if (direct) out_count[p] = base;
        else scount[p] = base;
    }
}

// Mutual decision from the reverse scan + ordered output (block of 256 per pair).
__global__ __launch_bounds__(256) void l2fr_final_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ cinit,
    const int32_t* __restrict__ pairs, const int4* __restrict__ surv,
    const int32_t* __restrict__ scount, const int4* __restrict__ rev, int mutual,
    int32_t* __restrict__ out_count, int32_t* __restrict__ out_match,
    int32_t* __restrict__ out_dist) {
    __shared__ int wsum[8];
    __shared__ int amb[256];
    __shared__ int namb;
    __shared__ unsigned char keepx[256];
    __shared__ long long redd[256];
    __shared__ int redq[256];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int S = (na > 0 && nb > 0) ? scount[p] : 0;
    const int4* sv = surv + (size_t)p * k_pad;
    const int4* rv = rev + (size_t)p * k_pad;
    const int32_t* na_norm = norm + (size_t)a * k_pad;
    const int32_t* nb_norm = norm + (size_t)b * k_pad;
    const int32_t* ca = cinit + (size_t)a * k_pad;
    const uint8_t* da = desc + (size_t)a * k_max * D;
    const uint4* dbv = (const uint4*)(desc + (size_t)b * k_max * D);
    int32_t* om = out_match + (size_t)p * k_max * 2;
    int32_t* od = out_dist + (size_t)p * k_max;
    int base = 0;
    for (int k0 = 0; k0 < S; k0 += 256) {
        const int k = k0 + tid;
        int4 s = make_int4(0, 0, 0, 0);
        bool keep = false;
        if (tid == 0) namb = 0;
        __syncthreads();
        if (k < S) {
            s = sv[k];
            keep = true;
            if (mutual) {
                const int4 r = rv[k];
                const int dot = (int)(((long long)na_norm[s.x] + nb_norm[s.y] - s.z) >> 1);
                const int ep = dot + ca[s.x];
                keep = (ep == r.x) && (r.y < r.x);
                if (ep == r.x && r.y == r.x) amb[atomicAdd(&namb, 1)] = tid;
            }
        }
        keepx[tid] = keep;
        __syncthreads();
        const int nam = namb;
        for (int i = 0; i < nam; ++i) {  // exact column scan: is q the lowest-index nearest query?
            const int who = amb[i];
            const int4 e = sv[k0 + who];
            uint4 y[SLOTS];
#pragma unroll
            for (int u = 0; u < SLOTS; ++u) y[u] = dbv[(size_t)e.y * SLOTS + u];
            long long bd = sfm::DIST_INF;
            int bq = INT_MAX;
            for (int q = tid; q < na; q += 256) {
                const int dot = dot128((const uint4*)(da + (size_t)q * D), y);
                const long long d = (long long)na_norm[q] + nb_norm[e.y] - 2LL * dot;
                if (d < bd) { bd = d; bq = q; }
            }
            redd[tid] = bd; redq[tid] = bq;
            __syncthreads();
            for (int st = 128; st > 0; st >>= 1) {
                if (tid < st) {
                    const long long od2 = redd[tid + st];
                    const int oq = redq[tid + st];
                    if (od2 < redd[tid] || (od2 == redd[tid] && oq < redq[tid])) {
                        redd[tid] = od2; redq[tid] = oq;
                    }
                }
                __syncthreads();
            }
            if (tid == 0) keepx[who] = (redq[0] == e.x);
            __syncthreads();
        }
        keep = keepx[tid] != 0 && k < S;
        base = sfm::compact256(keep, s.x, s.y, s.z, base, wsum, om, od);
    }
    if (tid == 0) out_count[p] = base;
}

// Debug dump of an intermediate record table into the match outputs (SFM_L2FR_DEBUG=1/2/3).
__global__ void l2fr_dump_kernel(const int32_t* __restrict__ n_kp, const int32_t* __restrict__ pairs,
                                 int k_max, int k_pad, const int4* __restrict__ rec,
                                 const int32_t* __restrict__ cnt, int32_t* __restrict__ out_count,
                                 int32_t* __restrict__ out_match, int32_t* __restrict__ out_dist) {
    const int p = blockIdx.x;
    const int n = cnt ? cnt[p] : n_kp[pairs[2 * p]];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int4 r = rec[(size_t)p * k_pad + i];
        out_match[((size_t)p * k_max + i) * 2] = r.x;
        out_match[((size_t)p * k_max + i) * 2 + 1] = r.y;
        out_dist[(size_t)p * k_max + i] = r.z;
    }
    if (threadIdx.x == 0) out_count[p] = n;
}

}  // namespace

// Forward/reverse L2 matcher (ratio test on, cross check mutual or off).
int sfm_match_l2fr_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                          int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                          const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                          int32_t* out_dist) {
    hipStream_t st = ctx->stream;
    if (k_max == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_pairs, st));
        return SFM_OK;
    }
    const int k_pad = (int)sfm::align_up((size_t)k_max, KALIGN);
    SFM_REQUIRE(k_pad <= KMAX, "sfm_match_batch: L2 matcher needs k_max <= 4096");
    const int n_qblk = (k_max + QB - 1) / QB;
    const size_t tab = (size_t)n_img * k_pad * sizeof(int32_t);
    const size_t recb = (size_t)n_pairs * k_pad * sizeof(int4);
    const size_t cntb = sfm::align_up(sizeof(int32_t) * (size_t)n_pairs, 256);
    const size_t descb = sfm::align_up((size_t)n_img * k_max * D, 256);
    const size_t ordb = sfm::align_up(sizeof(int32_t) * (size_t)n_pairs, 256);
    const size_t clsb = sfm::align_up((size_t)n_pairs * k_pad, 256);
    const int n_rng_max = n_pairs / REC_R + n_img + 1;  // recovery ranges (runs per train image)
    const size_t rngb = sfm::align_up(sizeof(int2) * (size_t)n_rng_max, 256);
    const size_t rinfob = sizeof(int4) * (size_t)n_rng_max * REC_R;
    const size_t sinfob = sfm::align_up(sizeof(int4) * (size_t)n_pairs, 256);
    const size_t uinfob = sfm::align_up(UNIT * sizeof(int4) * (size_t)n_pairs, 256);
    char* ws = (char*)sfm::workspace(ctx, 256 + 2 * tab + 3 * recb + cntb + descb + 2 * ordb + clsb +
                                              256 + rngb + rinfob + 256 + sinfob + uinfob + 256);
    if (!ws) return SFM_ERR_NOMEM;
    char* w = ws;
    uint8_t* zero_row = (uint8_t*)w; w += 256;
    int32_t* norm = (int32_t*)w; w += tab;
    int32_t* cinit = (int32_t*)w; w += tab;
    int4* fwd = (int4*)w; w += recb;
    int4* surv = (int4*)w; w += recb;
    int4* rev = (int4*)w; w += recb;
    int32_t* scount = (int32_t*)w; w += cntb;
    uint8_t* desc_i8 = (uint8_t*)w; w += descb;
    int32_t* ord_f = (int32_t*)w; w += ordb;
    int32_t* ord_r = (int32_t*)w; w += ordb;
    uint8_t* cls = (uint8_t*)w; w += clsb;
    int32_t* n_rng = (int32_t*)w; w += 256;
    int2* rng = (int2*)w; w += rngb;
    int4* rinfo = (int4*)w; w += rinfob;
    int4* sinfo_f = (int4*)sfm::align_up((size_t)w, 256);
    int4* uinfo = (int4*)((char*)sinfo_f + sinfob);
    int32_t* n_units = (int32_t*)((char*)uinfo + uinfob);
    // the forward scan by units of two pairs sharing their query image (build_units;
    // SFM_L2FR_UNITS=0: one pair per block, XCD-contiguous runs by train image)
    static const bool units_env = [] {
        const char* e = getenv("SFM_L2FR_UNITS");
        return !(e && e[0] == '0');
    }();
    // build_units keeps 3 n_img + 2 ints in LDS (64 KB per block): beyond ~5 400 images the
    // one-pair blocks
    const bool units = units_env && (3 * (size_t)n_img + 2) * sizeof(int) <= 65536;
    const int ppx = (n_pairs + 7) / 8;  // pairs per XCD run (scan kernel block order)
    const int n_blk = n_pairs;
    const int grid = 8 * ppx * n_qblk;
    const bool mutual = prm->cross_check == SFM_XC_MUTUAL;

    const int32_t* sord_f = ord_f;
    const int32_t* sord_r = ord_r;
    const int unit_blk = units ? (mutual ? 2 : 1) : -1;
    const int bpi = (k_pad + 1023) / 1024, n_prep = bpi * n_img;
    hipLaunchKernelGGL(l2fr_setup_kernel, dim3(n_prep + (mutual ? 2 : 1) + (units ? 1 : 0)),
                       dim3(1024), ((units ? 3 : 2) * (size_t)n_img + 2) * sizeof(int), st, n_prep,
                       bpi, desc, n_kp, k_max, k_pad, norm, cinit, zero_row, (uint4*)desc_i8, pairs,
                       n_pairs, n_img, ord_f, ord_r, rng, n_rng, rinfo, sinfo_f, unit_blk, uinfo,
                       n_units);
    SFM_HIP_CHECK(hipGetLastError());
    // qst (per-query status of the recovery) shares the reverse scan's output buffer: it is
    // consumed by the compaction before the reverse scan writes there.
    int4* qst = rev;
    const FwdCls fc{norm, prm->ratio_num, prm->ratio_den, (long long)prm->max_dist, qst, cls};
    hipLaunchKernelGGL(l2fr_scan_kernel<false>, dim3(grid), dim3(SCAN_THREADS), 0, st, desc_i8, n_kp, k_max,
                       k_pad, cinit, zero_row, pairs, n_qblk, sord_f,
                       (const int4*)(units ? uinfo : sinfo_f), n_blk, (const int4*)nullptr,
                       (const int32_t*)nullptr, fwd, fc, (const int32_t*)(units ? n_units : nullptr));
    SFM_HIP_CHECK(hipGetLastError());
    const char* dbg = getenv("SFM_L2FR_DEBUG");
    const int dmode = dbg ? atoi(dbg) : 0;
    if (dmode == 1) {
        hipLaunchKernelGGL(l2fr_dump_kernel, dim3(n_pairs), dim3(256), 0, st, n_kp, pairs, k_max,
                           k_pad, (const int4*)fwd, (const int32_t*)nullptr, out_count, out_match,
                           out_dist);
        return SFM_OK;
    }
#ifdef L2FR_RECOVER_VALU
    hipLaunchKernelGGL(l2fr_recover_kernel, dim3(n_pairs, k_pad / GROUP), dim3(256), 0, st, desc_i8,
                       n_kp, k_max, k_pad, norm, cinit, pairs, fwd, (const uint8_t*)cls,
                       prm->ratio_num, prm->ratio_den, (long long)prm->max_dist, qst);
#else
    hipLaunchKernelGGL(l2fr_recover_mfma_kernel, dim3(n_rng_max, k_pad / GROUP), dim3(256), 0, st,
                       desc_i8, k_max, k_pad, norm, cinit, (const int4*)rinfo, (const int32_t*)n_rng,
                       (const int4*)fwd, (const uint8_t*)cls, prm->ratio_num, prm->ratio_den,
                       (long long)prm->max_dist, qst);
#endif
    SFM_HIP_CHECK(hipGetLastError());
    // the ratio rule alone: the compaction writes the output itself (no final kernel)
    const bool direct = !mutual && dmode == 0;
    hipLaunchKernelGGL(l2fr_compact_kernel, dim3(n_pairs), dim3(256), 0, st, desc_i8, n_kp, k_max,
                       k_pad, norm, pairs, (const int4*)qst, prm->ratio_num, prm->ratio_den,
                       (long long)prm->max_dist, surv, scount, direct ? out_count : nullptr,
                       out_match, out_dist);
    SFM_HIP_CHECK(hipGetLastError());
    if (direct) return SFM_OK;
    if (dmode == 2) {
        hipLaunchKernelGGL(l2fr_dump_kernel, dim3(n_pairs), dim3(256), 0, st, n_kp, pairs, k_max,
                           k_pad, (const int4*)surv, (const int32_t*)scount, out_count, out_match,
                           out_dist);
        return SFM_OK;
    }
    if (mutual) {
        hipLaunchKernelGGL(l2fr_scan_kernel<true>, dim3(grid), dim3(SCAN_THREADS), 0, st, desc_i8, n_kp,
                           k_max, k_pad, cinit, zero_row, pairs, n_qblk, sord_r,
                           (const int4*)nullptr, n_blk,
                           (const int4*)surv, (const int32_t*)scount, rev, fc,
                           (const int32_t*)nullptr);
        SFM_HIP_CHECK(hipGetLastError());
    }
    if (dmode == 3) {
        hipLaunchKernelGGL(l2fr_dump_kernel, dim3(n_pairs), dim3(256), 0, st, n_kp, pairs, k_max,
                           k_pad, (const int4*)rev, (const int32_t*)scount, out_count, out_match,
                           out_dist);
        return SFM_OK;
    }
    hipLaunchKernelGGL(l2fr_final_kernel, dim3(n_pairs), dim3(256), 0, st, desc_i8, n_kp, k_max,
                       k_pad, norm, cinit, pairs, surv, scount, rev, mutual ? 1 : 0, out_count,
                       out_match, out_dist);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

#ifdef L2FR_CLOCK
// Diagnostic build only: the stamps of the last forward scan (L2FR_CLOCK_W per block).
extern "C" int sfm_debug_l2fr_stamps(unsigned long long* host, int32_t n_blocks) {
    const size_t n = L2FR_CLOCK_W * (size_t)std::min(n_blocks, L2FR_CLOCK_SLOTS);
    SFM_HIP_CHECK(hipDeviceSynchronize());
    SFM_HIP_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_l2fr_clock), n * sizeof(unsigned long long)));
    return SFM_OK;
}
#endif
