// All-pairs descriptor matching on MFMA (K1, SURVEY.md §8a a1/a3').
//
// Replaces the arithmetic behind cv2.BFMatcher(...).match (code/feature_matching.py:48-50),
// fused with the Lowe ratio test and the cross check, for both descriptor kinds:
//   L2 (128-byte SIFT-like): features x' = x ^ 0x80 (D = 128), d^2 = |x'|^2 + |y'|^2 - 2 x'.y';
//   Hamming (256-bit ORB, the reference's own NORM_HAMMING matcher): the bits as 0/1 bytes
//   (D = 256), d = popc(x) + popc(y) - 2 x.y — the same contraction and the same epilogue.
// (The L2 description below; the Hamming instantiation only changes D and the query tiles/wave.)
//
// Exact integer formulation.  With x' = x - 128 (u8 -> i8, a free XOR 0x80):
//     d^2(i,j) = |x'_i|^2 + |y'_j|^2 - 2 x'_i.y'_j
// The dot products run on v_mfma_i32_32x32x32_i8 (exact int32).  For a fixed query i the best
// train maximises  vr = 2 dot - |y'_j|^2  (= |x'_i|^2 - d^2);  for a fixed train j the best
// query maximises  -d^2.
//
// One key per element serves both directions:
//     Kr = 256 dot + crow_j = 128 vr + (127 - j mod 128)          one v_lshl_add
//     Kc = Kr + ccol_i      = -128 d^2 + (127 - j mod 128) + (127 - q_in_wave)   one v_add
// For a fixed query, Kc - Kr is a constant, so the row top-2 runs on Kr; for a fixed train the
// j term of Kc is a constant, so max Kc over queries is the (smallest d^2, lowest query) winner.
// |128 d^2| < 2^30 for any u8 descriptors, so neither key overflows.
//
// Geometry.  A 512-thread workgroup owns 1024 queries of one pair (8 waves x 4 query tiles of 32;
// the query descriptors are the MFMA B operand, held in 64 VGPRs per wave for the whole kernel)
// and streams every train of the other image through LDS in chunks of 256 rows (8 tiles), double
// buffered with global_load_lds (LDS-DMA) and an XOR-swizzled row image (conflict-free
// ds_read_b128; the swizzle is applied on the DMA source address).  MFMA output tile
// D[32 trains][32 queries]: the query is the lane, the 16 accumulator registers of a lane are 16
// of the 32 train rows (the other 16 live in lane ^ 32).
//  * row direction (per query: best, argbest, second over trains) is lane-local: a max3/med3
//    network on Kr keeps the top-2 of each group of 128 trains; (best, argbest, second) is merged
//    once per group.
//  * column direction (per train: best query): Kc, v_max3 over the wave's 4 query tiles, then a
//    transpose-reduce across the 32 lanes
//    of each half (permlane16_swap + DPP: 40 instructions for 16 registers) that leaves one train
//    row per lane pair, and one 64-bit LDS atomic max per lane merges the 8 waves.  Each workgroup
//    writes its column slab once; the finalize kernel merges the slabs of a pair.
// The prep kernel writes the descriptors once as i8 (x ^ 0x80); padded trains/queries read a
// constant all-zero i8 row (dot = 0), so their keys are the table constants alone and never win.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "match_common.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int WAVES = 8;              // waves per workgroup
constexpr int STAGE_BYTES = 32768;    // train bytes per LDS stage (CHUNK = STAGE_BYTES / D rows)
constexpr int KALIGN = 256;           // tables are padded to a multiple of 256 (row-key index field)
constexpr int KMAX_L2 = 4096;         // largest k_max of the fused key kernel (static LDS column state)
constexpr int KMAX_MU = 8192;         // largest k_max of the column-winner kernel (dynamic LDS:
                                      // k_pad u64 = 64 KB at 8192, beside the 33 KB of stages)

// Feature geometry per metric: D i8 features per row; QT query tiles (32 each) per wave.
//   L2:      D = 128 (x ^ 0x80 = x - 128),              QT = 4 -> 1024 queries per workgroup
//   Hamming: D = 256 (the 256 bits as 0/1 bytes),       QT = 2 ->  512 queries per workgroup
// Both use d = n_i + n_j - 2 dot (n = |x'|^2 resp. popcount): one kernel, exact int32.
template <int D> struct Geo {
    static constexpr int QT = D == 128 ? 4 : 2;
    static constexpr int QB = WAVES * QT * 32;
    static constexpr int CHUNK = STAGE_BYTES / D;   // 256 resp. 128 trains per stage
    static constexpr int NK = D / 32;               // MFMA k-steps per tile
    static constexpr int SLOTS = D / 16;            // 16-B slots per row
};
template <int D> __device__ __forceinline__ int swz(int row) {
    return D == 128 ? ((row >> 1) & 7) : (row & 15);  // conflict-free ds_read_b128
}
// Padding constants (valid keys: Kr, Kc >= -128 * 128 * 255^2 > -2^30; |crow|, |ccol| < 2^28):
// a padded train (dot = 0) has Kr = ROW_PAD, a padded query Kc < -2^30.  Only the (padded train,
// padded query) sum wraps; padded train rows are never read.
constexpr int ROW_PAD = -(3 << 29);       // crow of padded trains
constexpr int COL_PAD = -(3 << 29);       // ccol of padded queries
constexpr int VALID_MIN = -(1 << 23);     // decoded vr / -d^2 of real elements are > this
// Mutual kernel (value-only row side): e = x'.y' - ceil(n_y/2) of a real element is > -2^22.
constexpr int MU_PAD_ROW = -(1 << 23);    // accumulator init of padded trains: e below every real e
constexpr int MU_E_VALID = -(1 << 22);
constexpr int MU_COL_PAD = -(3 << 29);    // column constant of padded queries (zero rows: e <= 0)

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ int mad24(int a, int b, int c) { return __mul24(a, b) + c; }
// 3-input max / median as single instructions.  Plain max/min expressions let the compiler share
// max(tb, x) between the median and the max and emit two v_max_i32 instead of one v_max3_i32.
__device__ __forceinline__ int vmax3(int a, int b, int c) {
    int r;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ int vmed3(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// v_max3_i32 issued after `d0` and `d1` are computed (extra asm operands): lets an asm max3 read
// MFMA results once a compiler-emitted instruction has taken the padded first read.
__device__ __forceinline__ int vmax3_after(int a, int b, int c, int d0, int d1) {
    int r;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c), "v"(d0), "v"(d1));
    return r;
}

// No-return 64-bit LDS atomic max.  Inline asm: the compiler's LDS-DMA alias tracking treats a
// builtin atomic to the column-state object as possibly aliasing the in-flight staging DMA and
// inserts vmcnt(0); this one is ordered only by the lgkmcnt(0) of the barrier that precedes
// every read of the column state.
__device__ __forceinline__ void lds_max_u64(unsigned long long* p, unsigned long long v) {
    const unsigned addr = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned long long*)p;
    asm volatile("ds_max_u64 %0, %1" : : "v"(addr), "v"(v) : "memory");
}

template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}
// lane ^ 4 inside a 16-lane row with two bank-masked DPP moves (banks = 4-lane groups):
// banks 0,2 read lane+4 (row_shl:4), banks 1,3 read lane-4 (row_shr:4).  No LDS round trip.
__device__ __forceinline__ int dpp_xor4(int x) {
    int y = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xF, 0x5, false);
    return __builtin_amdgcn_update_dpp(y, x, 0x114, 0xF, 0xA, false);
}

// Max-reduce each of 16 registers over the 32 lanes of its wave half; on return lane l holds the
// result for register r(l) = 8*b1 + 4*b2 + 2*b3 + b4 (b_k = bit k of l); lanes l and l^1 agree.
__device__ __forceinline__ int transpose_max16(const int (&c)[16], int lane) {
    int m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // lane bit 4: rows (16 lanes) swapped pairwise
        auto s = __builtin_amdgcn_permlane16_swap(c[2 * k], c[2 * k + 1], false, false);
        m[k] = max((int)s[0], (int)s[1]);
    }
    const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
    int n[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // lane bit 3: xor 8 inside a 16-lane row = row_ror:8
        const int t0 = max(m[2 * k], dpp<0x128>(m[2 * k]));
        const int t1 = max(m[2 * k + 1], dpp<0x128>(m[2 * k + 1]));
        n[k] = b3 ? t1 : t0;
    }
    int o[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // lane bit 2: xor 4
        const int send = b2 ? n[2 * k] : n[2 * k + 1];
        const int keep = b2 ? n[2 * k + 1] : n[2 * k];
        o[k] = max(keep, dpp_xor4(send));
    }
    // lane bit 1: quad_perm [2,3,0,1]; lane bit 0: quad_perm [1,0,3,2]
    const int p0 = max(o[0], dpp<0x4E>(o[0]));
    const int p1 = max(o[1], dpp<0x4E>(o[1]));
    const int q = b1 ? p1 : p0;
    return max(q, dpp<0xB1>(q));
}

// Per descriptor: the i8 feature row (L2: x ^ 0x80; Hamming: bits -> 0/1 bytes), its norm
// (|x'|^2 resp. popcount) and the row-key constant, padded to k_pad (multiple of 256).
// BITV: the byte value of a set bit (Hamming): 1 for the fused / column-winner kernels, 16 for the
// key-in-the-accumulator Hamming kernel (16 x 16 = 256: the MFMA then yields 256 dot).
template <int METRIC, bool CINIT = false, int BITV = 1>
__global__ void mfma_prep_kernel(const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp,
                                 int k_max, int k_pad, int32_t* __restrict__ norm,
                                 int32_t* __restrict__ crow, uint8_t* __restrict__ zero_row,
                                 uint4* __restrict__ desc_i8) {
    constexpr int DIN = METRIC == SFM_METRIC_L2 ? 128 : 32;   // input bytes per descriptor
    constexpr int D = METRIC == SFM_METRIC_L2 ? 128 : 256;    // feature bytes per row
    const int img = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (img == 0 && j < D) zero_row[j] = 0;  // i8 zero row for padded trains / queries
    if (j >= k_pad) return;
    int nv = 0;
    if (j < k_max) {
        const uint4* p = (const uint4*)(desc + ((size_t)img * k_max + j) * DIN);
        uint4* o8 = desc_i8 + ((size_t)img * k_max + j) * (D / 16);
        if (METRIC == SFM_METRIC_L2) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint4 v = p[q];
                const uint4 x = make_uint4(v.x ^ 0x80808080u, v.y ^ 0x80808080u,
                                           v.z ^ 0x80808080u, v.w ^ 0x80808080u);
                o8[q] = x;
                // |x'|^2 of the signed bytes x' = x - 128, four at a time (exact integer sums)
                nv = __builtin_amdgcn_sdot4((int)x.x, (int)x.x, nv, false);
                nv = __builtin_amdgcn_sdot4((int)x.y, (int)x.y, nv, false);
                nv = __builtin_amdgcn_sdot4((int)x.z, (int)x.z, nv, false);
                nv = __builtin_amdgcn_sdot4((int)x.w, (int)x.w, nv, false);
            }
        } else {
            // bit b of byte k (OpenCV's bit order is irrelevant: the distance counts all bits)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint4 v = p[q];
                const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    nv += __popc(w[e]);
                    unsigned o[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t) {  // 4 bits of word e -> one u32 of 0/1 bytes
                        const unsigned nib = (w[e] >> (4 * t)) & 0xFu;
                        o[t] = ((nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21)) *
                               (unsigned)BITV;
                    }
                    o8[8 * q + 2 * e] = make_uint4(o[0], o[1], o[2], o[3]);
                    o8[8 * q + 2 * e + 1] = make_uint4(o[4], o[5], o[6], o[7]);
                }
            }
        }
    }
    const size_t o = (size_t)img * k_pad + j;
    norm[o] = nv;
    // row key Kr = 128 vr + (127 - j mod 128) = 256 dot + crow;  vr = 2 dot - n_j
    if (CINIT)  // mutual kernel: accumulator init -ceil(n/2) (its padding: MU_PAD_ROW)
        crow[o] = (j < n_kp[img]) ? -((nv + 1) >> 1) : MU_PAD_ROW;
    else
        crow[o] = (j < n_kp[img]) ? (-128 * nv + 127 - (j & 127)) : ROW_PAD;
}

// Pair order by train image (counting sort in LDS; one block): consecutive entries share image b.
__global__ __launch_bounds__(1024) void pair_order_kernel(const int32_t* __restrict__ pairs,
                                                          int n_pairs, int n_img,
                                                          int32_t* __restrict__ order,
                                                          int32_t* __restrict__ unused) {
    extern __shared__ int hist[];
    const int tid = threadIdx.x;
    for (int i = tid; i < n_img; i += 1024) hist[i] = 0;
    __syncthreads();
    for (int p = tid; p < n_pairs; p += 1024) atomicAdd(&hist[pairs[2 * p + 1]], 1);
    __syncthreads();
    if (tid == 0) {
        int off = 0;
        for (int i = 0; i < n_img; ++i) { const int c = hist[i]; hist[i] = off; off += c; }
    }
    __syncthreads();
    for (int p = tid; p < n_pairs; p += 1024) order[atomicAdd(&hist[pairs[2 * p + 1]], 1)] = p;
}

// TOP2 = false: the row side keeps only (best, argbest) — the second-best value is what the ratio
// test needs, and the ordered-pair path (sfm_match_batch_both, no ratio) drops its med3 + max.
template <int D, bool TOP2 = true>
__global__ __launch_bounds__(512, 2) void mfma_match_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ crow_tab,
    const uint8_t* __restrict__ zero_row, const int32_t* __restrict__ pairs, int n_qblk,
    const int32_t* __restrict__ pair_order, int n_blk, int4* __restrict__ rowres,
    unsigned long long* __restrict__ colpart) {
    // LDS: two DMA staging objects ([CHUNK][128 B] train rows + [CHUNK] crow each) and the column
    // state, all distinct __shared__ objects: with the chunk loop unrolled by two every access
    // names its buffer statically, so the compiler's LDS-DMA alias tracking does not make reads
    // of one buffer wait (vmcnt) for the DMA into the other.
    constexpr int QT = Geo<D>::QT, QB = Geo<D>::QB, CHUNK = Geo<D>::CHUNK, NK = Geo<D>::NK;
    constexpr int SLOTS = Geo<D>::SLOTS, NT = CHUNK / 32;
    constexpr int PIECES = CHUNK * D / 1024 / WAVES;  // 1 KB LDS-DMA pieces per wave per chunk
    constexpr int RPP = 1024 / D;                     // rows per 1 KB piece
    __shared__ __attribute__((aligned(16))) unsigned char lds0[CHUNK * D + CHUNK * 4];
    __shared__ __attribute__((aligned(16))) unsigned char lds1[CHUNK * D + CHUNK * 4];
    __shared__ unsigned long long lds_col[KMAX_L2];

    // XCD-aware block mapping: workgroups are dispatched round-robin over the 8 XCDs (L % 8), so
    // XCD x takes the x-th contiguous run of the blocks ordered by train image (pair_order): the
    // blocks an XCD runs together stream the same train descriptors through its own L2.  The
    // grid is padded to 8 * per_xcd blocks (every XCD slot exists); slots past n_blk exit.
    const int per_xcd = (int)(gridDim.x >> 3);
    const int sblk = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
    if (sblk >= n_blk) return;  // block-uniform, before any barrier
    const int p = pair_order[sblk / n_qblk], qb = sblk % n_qblk;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    for (int j = tid; j < k_pad; j += 512) lds_col[j] = 0ull;

    const uint8_t* db = desc + (size_t)b * k_max * D;
    const int32_t* crb = crow_tab + (size_t)b * k_pad;
    const int n_chunk = (nb + CHUNK - 1) / CHUNK;

    // stage chunk ch into buffer dst: PIECES x 1 KB LDS-DMA pieces per wave (+ the crow piece);
    // lane L of a piece lands in slot L % SLOTS of row L / SLOTS and fetches the swizzled slot
    auto stage = [&](int ch, unsigned char* dst) {
#pragma unroll
        for (int i = 0; i < PIECES; ++i) {
            const int piece = wave * PIECES + i;
            const int row = piece * RPP + lane / SLOTS;
            const int slot = (lane % SLOTS) ^ swz<D>(row);
            const int j = ch * CHUNK + row;
            const uint8_t* src = (j < nb) ? db + (size_t)j * D + slot * 16 : zero_row + slot * 16;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + piece * 1024), 16, 0, 0);
        }
        if (wave == 0 && lane < CHUNK / 4) {
            const int32_t* src = crb + ch * CHUNK + lane * 4;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + CHUNK * D), 16, 0, 0);
        }
    };

    const int qbase = qb * QB + wave * QT * 32;
    const bool active = qbase < na;  // wave-uniform
    v4i bq[QT][NK];
    int ccol[QT], B1[QT], J1[QT], B2[QT], tb[QT], ts[QT];
    const uint8_t* da = desc + (size_t)a * k_max * D;
#pragma unroll
    for (int c = 0; c < QT; ++c) {
        const int q = qbase + c * 32 + r32;
        const v4i* src = (const v4i*)((q < na) ? da + (size_t)q * D + (D / 2) * h : zero_row + (D / 2) * h);
#pragma unroll
        for (int s = 0; s < NK; ++s) bq[c][s] = src[s];
        // Kc = Kr + ccol = -128 d^2 + (127 - j mod 128) + (127 - q_in_wave)
        ccol[c] = (q < na) ? (-128 * norm[(size_t)a * k_pad + q] + 127 - (c * 32 + r32)) : COL_PAD;
        B1[c] = INT_MIN; J1[c] = -1; B2[c] = INT_MIN;
        tb[c] = INT_MIN; ts[c] = INT_MIN;
    }
    // process chunk ch from buffer cur while chunk ch+1 streams into buffer nxt
    auto process = [&](int ch, const unsigned char* cur, unsigned char* nxt) {
        if (ch + 1 < n_chunk) stage(ch + 1, nxt);
            const int nt = min(NT, (nb - ch * CHUNK + 31) >> 5);
            if (active) {
                const unsigned char* A = cur;
                const int* Cr = (const int*)(cur + CHUNK * D);
                // one 32-train tile: MFMAs for the 4 query tiles + both epilogues; returns the
                // transposed column key of this lane's train row
                auto tile = [&](int tt) -> int {
                    const int row = tt * 32 + r32;
                    const int sw = swz<D>(row);
                    v4i af[NK];
#pragma unroll
                    for (int s = 0; s < NK; ++s)
                        af[s] = *(const v4i*)(A + row * D + ((((SLOTS / 2) * h + s) ^ sw) << 4));
                    int crow[16];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const v4i cv = *(const v4i*)(Cr + tt * 32 + 8 * g + 4 * h);
                        crow[4 * g + 0] = cv.x; crow[4 * g + 1] = cv.y;
                        crow[4 * g + 2] = cv.z; crow[4 * g + 3] = cv.w;
                    }
                    int colacc[16];
#pragma unroll
                    for (int c = 0; c < QT; c += 2) {
                        v16i acc0 = {0}, acc1 = {0};
#pragma unroll
                        for (int s = 0; s < NK; ++s) {
                            acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[c][s], acc0, 0, 0, 0);
                            acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[c + 1][s], acc1, 0, 0, 0);
                        }
#pragma unroll
                        for (int r = 0; r < 16; r += 2) {
                            // row direction on Kr: running top-2 of the 128-train group
                            const int x0 = mad24(acc0[r], 256, crow[r]);
                            const int y0 = mad24(acc0[r + 1], 256, crow[r + 1]);
                            if (TOP2) ts[c] = max(ts[c], vmed3(tb[c], x0, y0));
                            tb[c] = vmax3(tb[c], x0, y0);
                            const int x1 = mad24(acc1[r], 256, crow[r]);
                            const int y1 = mad24(acc1[r + 1], 256, crow[r + 1]);
                            if (TOP2) ts[c + 1] = max(ts[c + 1], vmed3(tb[c + 1], x1, y1));
                            tb[c + 1] = vmax3(tb[c + 1], x1, y1);
                            // column direction on Kc = Kr + ccol (full-rate add)
                            const int a0 = x0 + ccol[c], a1 = x1 + ccol[c + 1];
                            const int b0 = y0 + ccol[c], b1 = y1 + ccol[c + 1];
                            colacc[r] = (c == 0) ? max(a0, a1) : vmax3(colacc[r], a0, a1);
                            colacc[r + 1] = (c == 0) ? max(b0, b1) : vmax3(colacc[r + 1], b0, b1);
                        }
                    }
                    return transpose_max16(colacc, lane);
                };
                const int rr = ((lane >> 1) & 1) * 8 + ((lane >> 2) & 1) * 4 + ((lane >> 3) & 1) * 2 +
                               ((lane >> 4) & 1);
                const int rowoff = (rr & 3) + 8 * (rr >> 2) + 4 * h;
                // lane pair's train row j: e = Kc - (127 - j mod 128) = -128 d^2 + (127 - q_in_wave)
                auto col_merge = [&](int tt, int key) {
                    const int j = ch * CHUNK + tt * 32 + rowoff;
                    const int e = key - (127 - (j & 127));
                    const int nd = e >> 7;  // -d^2 (padding: out of range)
                    if (!(lane & 1) && nd > VALID_MIN && nd <= 0) {
                        const unsigned vb = (unsigned)nd ^ 0x80000000u;
                        const unsigned gq = (unsigned)(qbase + 127 - (e & 127));
                        lds_max_u64(&lds_col[j],
                                    ((unsigned long long)vb << 32) | (unsigned long long)(0xFFFFFFFFu - gq));
                    }
                };
                // merge the 128-train group's top-2 into the running (best, argbest, second)
                auto row_merge = [&](int gbase) {
#pragma unroll
                    for (int c = 0; c < QT; ++c) {
                        const int v1 = tb[c] >> 7, v2 = ts[c] >> 7;
                        const int j1 = gbase + 127 - (tb[c] & 127);
                        const bool up = v1 > B1[c];
                        B2[c] = up ? max(B1[c], v2) : max(B2[c], v1);
                        J1[c] = up ? j1 : J1[c];
                        B1[c] = max(B1[c], v1);
                        tb[c] = INT_MIN; ts[c] = INT_MIN;
                    }
                };
                // lds_col is its own __shared__ object, disjoint from the LDS-DMA staging buffers, so
                // these atomics need not wait for the in-flight DMA of the next chunk.
                for (int tt = 0; tt < nt; ++tt) {
                    col_merge(tt, tile(tt));
                    if ((tt & 3) == 3 || tt == nt - 1) row_merge(ch * CHUNK + (tt & ~3) * 32);
                }
            }
    };
    if (n_chunk > 0) stage(0, lds0);
    __syncthreads();
    for (int ch = 0; ch < n_chunk; ch += 2) {
        process(ch, lds0, lds1);
        __syncthreads();  // chunk ch+1 landed (vmcnt drained); everyone is done with lds0
        if (ch + 1 < n_chunk) process(ch + 1, lds1, lds0);
        __syncthreads();
    }

    if (active) {
#pragma unroll
        for (int c = 0; c < QT; ++c) {
            const int P1 = __shfl_xor(B1[c], 32), PJ = __shfl_xor(J1[c], 32),
                      P2 = __shfl_xor(B2[c], 32);
            const bool take = (P1 > B1[c]) || (P1 == B1[c] && PJ >= 0 && PJ < J1[c]);
            const int nb2 = max(min(B1[c], P1), max(B2[c], P2));
            if (take) { B1[c] = P1; J1[c] = PJ; }
            B2[c] = nb2;
            const int q = qbase + c * 32 + r32;
            if (h == 0 && q < na) rowres[(size_t)p * k_pad + q] = make_int4(B1[c], J1[c], B2[c], 0);
        }
    }
    unsigned long long* dst = colpart + ((size_t)p * n_qblk + qb) * k_pad;
    for (int j = tid; j < k_pad; j += 512) dst[j] = lds_col[j];
}

// Finalize: cross check + ratio + max distance, ordered compaction (one 256-thread block / pair).
__global__ __launch_bounds__(256) void l2_finalize_kernel(
    const int32_t* __restrict__ n_kp, int k_max, int k_pad, const int32_t* __restrict__ norm,
    const int32_t* __restrict__ pairs, int n_qblk, const int4* __restrict__ rowres,
    const unsigned long long* __restrict__ colpart, int xc, int rnum, int rden,
    long long max_dist, int squared, int32_t* __restrict__ out_count,
    int32_t* __restrict__ out_match, int32_t* __restrict__ out_dist) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_best[];
    __shared__ int wsum[8];
    const int p = blockIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int tid = threadIdx.x;
    const unsigned long long* cp = colpart + (size_t)p * n_qblk * k_pad;
    int32_t* om = out_match + (size_t)p * k_max * 2;
    int32_t* od = out_dist + (size_t)p * k_max;
    int base = 0;
    if (na <= 0 || nb <= 0) {
        if (tid == 0) out_count[p] = 0;
        return;
    }
    if (xc == SFM_XC_OPENCV) {
        for (int i = tid; i < na; i += 256) lds_best[i] = ~0ull;
        __syncthreads();
        for (int j = tid; j < nb; j += 256) {
            unsigned long long best = 0;
            for (int q = 0; q < n_qblk; ++q) best = max(best, cp[(size_t)q * k_pad + j]);
            if (best == 0) continue;
            const int v = (int)((unsigned)(best >> 32) ^ 0x80000000u);  // -d^2
            const int gq = (int)(0xFFFFFFFFu - (unsigned)best);
            if (gq < 0 || gq >= na) continue;  // defensive: a column winner is always a query
            const long long d = -(long long)v;
            atomicMin(&lds_best[gq], ((unsigned long long)d << 32) | (unsigned)j);
        }
        __syncthreads();
        for (int i0 = 0; i0 < na; i0 += 256) {
            const int i = i0 + tid;
            bool keep = false;
            int j = 0, d = 0;
            if (i < na) {
                const unsigned long long e = lds_best[i];
                if (e != ~0ull) {
                    d = (int)(e >> 32);
                    j = (int)(unsigned)e;
                    keep = (max_dist < 0) || ((long long)d < max_dist);
                }
            }
            base = sfm::compact256(keep, i, j, d, base, wsum, om, od);
        }
    } else {
        for (int i0 = 0; i0 < na; i0 += 256) {
            const int i = i0 + tid;
            bool keep = false;
            int j = 0;
            long long d1 = 0;
            if (i < na) {
                const int4 rr = rowres[(size_t)p * k_pad + i];
                j = rr.y;
                if (j >= 0 && j < nb && rr.x > VALID_MIN) {
                    const long long nx = norm[(size_t)a * k_pad + i];
                    d1 = nx - rr.x;
                    const long long d2 = (rr.z > VALID_MIN) ? nx - rr.z : sfm::DIST_INF;
                    keep = true;
                    if (xc == SFM_XC_MUTUAL) {
                        unsigned long long best = 0;
                        for (int q = 0; q < n_qblk; ++q) best = max(best, cp[(size_t)q * k_pad + j]);
                        keep = (int)(0xFFFFFFFFu - (unsigned)best) == i;
                    }
                    keep = keep && sfm::ratio_ok(d1, d2, rnum, rden, squared != 0);
                    keep = keep && (max_dist < 0 || d1 < max_dist);
                }
            }
            base = sfm::compact256(keep, i, j, (int)d1, base, wsum, om, od);
        }
    }
    if (tid == 0) out_count[p] = base;
}


// ---- Mutual cross check on a value-only row side (L2; DESIGN.md §4.1 "mutual kernel") ----------
//
// The row side needs no train index under the mutual rule: the column side already names, for
// every train j, its nearest query (exact, lowest index).  So the row side keeps only the top-2
// VALUES of e = x'.y' - ceil(|y'|^2/2) — produced by the MFMA itself (accumulator initialised from
// the trains' -ceil(|y'|^2/2) table), no key build — and the column key is built from e:
//     Kc = 256 e + (-128 |x'_q|^2 + 127 - q_in_wave) = 128 (2e - |x'_q|^2) + (127 - q_in_wave)
// (one v_lshl_add_u32; 2e - |x'_q|^2 = -d^2 - p_j with p_j = |y'_j|^2 mod 2, constant per train).
// Finalize: every train's column winner q proposes (d, j); a query keeps its smallest proposal
// D*.  If e1 > e2, the only train with d <= |x'|^2 - 2 e1 is the query's unique nearest neighbour
// j1 (d = |x'|^2 - 2e - p_j, so any other train is >= 1 farther), hence q is mutual iff D* <=
// |x'|^2 - 2 e1, and then d1 = D* exactly; d2 lies in [|x'|^2 - 2e2 - 1, |x'|^2 - 2e2], which
// decides the ratio test unless it straddles it.  e1 == e2 and straddles take an exact row scan.
__device__ __forceinline__ void mu_top2(int& tb, int& ts, int x, int y) {
    // compiler-emitted v_med3_i32 (the compiler pads the MFMA -> VALU hazard), then the asm
    // v_max3_i32 ordered after it by the median operand (hipcc pads nothing into an asm statement)
    const int med = max(min(tb, x), min(max(tb, x), y));
    int top;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(top) : "v"(tb), "v"(x), "v"(y), "v"(med));
    ts = max(ts, med);
    tb = top;
}

// ROWS = false: column side only (the OpenCV cross-check rule needs nothing else).
// Workgroup shape of the column-winner kernel: MU_WAVES waves x QT query tiles, MU_CHUNK_BYTES of
// train rows per LDS stage, built for MU_MINW waves per SIMD.  Default 4 waves x 16 KB stages x 2
// waves/SIMD: interleaved A/B on cfg3 (profiles/r01_k1_shapes.txt), mutual + ratio 1.00 ms against
// 1.04 (8 waves, 32 KB), 1.05 (8 waves, 16 KB), 1.22 (4 waves, 32 KB) and 1.06 (3 waves/SIMD,
// spills); the column-only kernel is shape-neutral (0.84 ms).
#ifndef MU_WAVES
#define MU_WAVES 4
#endif
#ifndef MU_CHUNK_BYTES
#define MU_CHUNK_BYTES 16384
#endif
#ifndef MU_MINW
#define MU_MINW 2
#endif
template <int D> constexpr int mu_qb() { return MU_WAVES * Geo<D>::QT * 32; }
#ifdef MU_CLOCK
constexpr int MU_CLOCK_SLOTS = 1 << 16;
constexpr int MU_CLOCK_W = 8;  // per block: loop memtime/realtime start+end, entry/exit realtime, HW_ID, XCC_ID
__device__ unsigned long long g_mu_clock[MU_CLOCK_W * MU_CLOCK_SLOTS];
#endif

template <int D, bool ROWS>
__global__ __launch_bounds__(64 * MU_WAVES, MU_MINW) void mfma_mutual_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ cinit,
    const uint8_t* __restrict__ zero_row, const int32_t* __restrict__ pairs, int n_qblk,
    const int32_t* __restrict__ pair_order, int n_blk, int4* __restrict__ rowres,
    unsigned long long* __restrict__ colpart, int col_atomic) {
    constexpr int QT = Geo<D>::QT, QB = mu_qb<D>(), CHUNK = MU_CHUNK_BYTES / D, NK = Geo<D>::NK;
    constexpr int SLOTS = Geo<D>::SLOTS, NT = CHUNK / 32, NTHR = 64 * MU_WAVES;
    constexpr int PIECES = CHUNK * D / 1024 / MU_WAVES, RPP = 1024 / D;
    static_assert(PIECES >= 1 && CHUNK % 32 == 0 && CHUNK / 4 <= 64, "stage geometry");
    __shared__ __attribute__((aligned(16))) unsigned char lds0[CHUNK * D + CHUNK * 4];
    __shared__ __attribute__((aligned(16))) unsigned char lds1[CHUNK * D + CHUNK * 4];
    extern __shared__ unsigned long long lds_col[];  // [k_pad], dynamic

#ifdef MU_CLOCK
    const unsigned long long tin = __builtin_amdgcn_s_memrealtime();
#endif
    const int per_xcd = (int)(gridDim.x >> 3);
    const int sblk = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
    if (sblk >= n_blk) return;  // block-uniform, before any barrier
    const int qb = sblk % n_qblk;
    const int p = pair_order[sblk / n_qblk];
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    for (int j = tid; j < k_pad; j += NTHR) lds_col[j] = 0ull;

    const uint8_t* db = desc + (size_t)b * k_max * D;
    const int32_t* cib = cinit + (size_t)b * k_pad;
    const int n_chunk = (nb + CHUNK - 1) / CHUNK;
    auto stage = [&](int ch, unsigned char* dst) {
#pragma unroll
        for (int i = 0; i < PIECES; ++i) {
            const int piece = wave * PIECES + i;
            const int row = piece * RPP + lane / SLOTS;
            const int slot = (lane % SLOTS) ^ swz<D>(row);
            const int j = ch * CHUNK + row;
            const uint8_t* src = (j < nb) ? db + (size_t)j * D + slot * 16 : zero_row + slot * 16;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + piece * 1024), 16, 0, 0);
        }
        if (wave == 0 && lane < CHUNK / 4) {
            const int32_t* src = cib + ch * CHUNK + lane * 4;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + CHUNK * D), 16, 0, 0);
        }
    };

    const int qbase = qb * QB + wave * QT * 32;
    const bool active = qbase < na;  // wave-uniform
    v4i bq[QT][NK];
    int ccol[QT], tb[QT], ts[QT];
    const uint8_t* da = desc + (size_t)a * k_max * D;
#pragma unroll
    for (int c = 0; c < QT; ++c) {
        const int q = qbase + c * 32 + r32;
        const v4i* src = (const v4i*)((q < na) ? da + (size_t)q * D + (D / 2) * h : zero_row + (D / 2) * h);
#pragma unroll
        for (int s = 0; s < NK; ++s) bq[c][s] = src[s];
        ccol[c] = (q < na) ? (-128 * norm[(size_t)a * k_pad + q] + 127 - (c * 32 + r32)) : MU_COL_PAD;
        tb[c] = INT_MIN; ts[c] = INT_MIN;
    }
    const int rr = ((lane >> 1) & 1) * 8 + ((lane >> 2) & 1) * 4 + ((lane >> 3) & 1) * 2 +
                   ((lane >> 4) & 1);
    const int rowoff = (rr & 3) + 8 * (rr >> 2) + 4 * h;

    auto process = [&](int ch, const unsigned char* cur, unsigned char* nxt) {
        if (ch + 1 < n_chunk) stage(ch + 1, nxt);
        const int nt = min(NT, (nb - ch * CHUNK + 31) >> 5);
        if (active) {
            const unsigned char* A = cur;
            const int* Ci = (const int*)(cur + CHUNK * D);
            // A fragments + accumulator init of tile tt (accumulator register r of this lane is
            // train row 8*(r/4) + 4*h + r%4)
            auto load_tile = [&](int tt, v4i (&af)[NK], v16i& init) {
                const int row = tt * 32 + r32;
                const int sw = swz<D>(row);
#pragma unroll
                for (int s = 0; s < NK; ++s)
                    af[s] = *(const v4i*)(A + row * D + ((((SLOTS / 2) * h + s) ^ sw) << 4));
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const v4i cv = *(const v4i*)(Ci + tt * 32 + 8 * g + 4 * h);
                    init[4 * g + 0] = cv.x; init[4 * g + 1] = cv.y;
                    init[4 * g + 2] = cv.z; init[4 * g + 3] = cv.w;
                }
            };
            v4i af[NK];
            v16i init;
            for (int tt = 0; tt < nt; ++tt) {
                load_tile(tt, af, init);
                int colacc[16];
#pragma unroll
                for (int c = 0; c < QT; c += 2) {
                    v16i acc0 = init, acc1 = init;
#ifdef MU_MPRIO  // A/B: the MFMA group at raised priority (as the ratio path's scan)
                    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
                    for (int s = 0; s < NK; ++s) {
                        acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[c][s], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[c + 1][s], acc1, 0, 0, 0);
                    }
#ifdef MU_MPRIO
                    __builtin_amdgcn_s_setprio(0);
#endif
#pragma unroll
                    for (int r = 0; r < 16; r += 2) {
                        if constexpr (ROWS) {
                            mu_top2(tb[c], ts[c], acc0[r], acc0[r + 1]);
                            mu_top2(tb[c + 1], ts[c + 1], acc1[r], acc1[r + 1]);
                        }
                        // column keys: 256 e + ccol (wraps only for padded-train rows, never merged)
#ifdef MU_DIAG_NOKEY  // timing-only bound (wrong results): the column key build costs nothing
                        const int a0 = acc0[r], a1 = acc1[r], b0 = acc0[r + 1], b1 = acc1[r + 1];
#else
                        const int a0 = (int)(((unsigned)acc0[r] << 8) + (unsigned)ccol[c]);
                        const int a1 = (int)(((unsigned)acc1[r] << 8) + (unsigned)ccol[c + 1]);
                        const int b0 = (int)(((unsigned)acc0[r + 1] << 8) + (unsigned)ccol[c]);
                        const int b1 = (int)(((unsigned)acc1[r + 1] << 8) + (unsigned)ccol[c + 1]);
#endif
                        colacc[r] = (c == 0) ? max(a0, a1) : vmax3(colacc[r], a0, a1);
                        colacc[r + 1] = (c == 0) ? max(b0, b1) : vmax3(colacc[r + 1], b0, b1);
                    }
                }
                const int key = transpose_max16(colacc, lane);
                const int j = ch * CHUNK + tt * 32 + rowoff;
                if (!(lane & 1) && j < nb) {
                    const int nd = key >> 7;  // 2e - |x'_q|^2 = -d^2 - p_j
                    const unsigned gq = (unsigned)(qbase + 127 - (key & 127));
                    lds_max_u64(&lds_col[j], ((unsigned long long)((unsigned)nd ^ 0x80000000u) << 32) |
                                                 (unsigned long long)(0xFFFFFFFFu - gq));
                }
            }
        }
    };
#ifdef MU_CLOCK  // diagnostic build only: in-kernel clock (MI355X_MICROARCH.md "DVFS give-back" 6)
    const unsigned long long t0c = __builtin_amdgcn_s_memtime(), t0r = __builtin_amdgcn_s_memrealtime();
#endif
    if (n_chunk > 0) stage(0, lds0);
    __syncthreads();
    for (int ch = 0; ch < n_chunk; ch += 2) {
        process(ch, lds0, lds1);
        __syncthreads();
        if (ch + 1 < n_chunk) process(ch + 1, lds1, lds0);
        __syncthreads();
    }
#ifdef MU_CLOCK
    {   // stamps to a buffer of their own, read only by sfm_debug_clock_stamps (never an output)
        const unsigned long long t1c = __builtin_amdgcn_s_memtime(), t1r = __builtin_amdgcn_s_memrealtime();
        if (tid == 0 && blockIdx.x < MU_CLOCK_SLOTS) {
            unsigned long long* d = g_mu_clock + MU_CLOCK_W * (size_t)blockIdx.x;
            d[0] = t0c; d[1] = t0r; d[2] = t1c; d[3] = t1r; d[4] = tin;
            d[6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
            d[7] = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
        }
    }
#endif
    if (ROWS && active) {
#pragma unroll
        for (int c = 0; c < QT; ++c) {
            const int P1 = __shfl_xor(tb[c], 32), P2 = __shfl_xor(ts[c], 32);
            const int e1 = max(tb[c], P1);
            const int e2 = max(min(tb[c], P1), max(ts[c], P2));
            const int q = qbase + c * 32 + r32;
            // 8-B row records (e1, e2): half the row bytes of round 1's 16-B layout
            if (h == 0 && q < na) ((int2*)rowres)[(size_t)p * k_pad + q] = make_int2(e1, e2);
        }
    }
#ifdef MU_DIAG_NOMERGE  // timing-only bound (wrong results): no column-table merge at block end
    if (false) {
#else
    if (col_atomic) {
#endif
        // merged across the pair's query blocks in place (zeroed before the launch; the grid
        // keeps every pair's blocks on one XCD, so the merge happens in that XCD's L2)
        unsigned long long* dst = colpart + (size_t)p * k_pad;
        for (int j = tid; j < k_pad; j += NTHR) {
            const unsigned long long v = lds_col[j];
            if (v != 0ull) atomicMax(dst + j, v);
        }
    } else {
        unsigned long long* dst = colpart + ((size_t)p * n_qblk + qb) * k_pad;
        for (int j = tid; j < k_pad; j += NTHR) dst[j] = lds_col[j];
    }
#ifdef MU_CLOCK
    __syncthreads();
    if (tid == 0 && blockIdx.x < MU_CLOCK_SLOTS)
        g_mu_clock[MU_CLOCK_W * (size_t)blockIdx.x + 5] = __builtin_amdgcn_s_memrealtime();
#endif
}

// ---- Hamming with the key built by the MFMA itself (sfm_match_batch_both's Hamming path) ----------
//
// The reference's own matcher is Hamming (ORB, code/feature_matching.py:48).  With the bits as
// 0/16 bytes the i8 MFMA yields 256 dot exactly, the accumulator init is the train constant
// crow_j = -128 n_j + (127 - j mod 128) (from LDS, as the mutual kernel's init), and ONE extra
// 32-deep MFMA k-step adds the query constant -128 n_q + (127 - q mod 64): its A fragment is a
// constant (eight 64s and a 1 in the lane-half-0 bytes), its B fragment per query holds eight
// digits d_t in [-128, 0] with sum -2 n_q and the byte 127 - q mod 64.  So every element's
// accumulator is already
//     K = -128 d + (127 - j mod 128) + (127 - q mod 64),        d = n_j + n_q - 2 dot,
// the key of BOTH directions: for a fixed query (lane) the q term is a constant (row top-1 by
// max3, the nearest train and its lowest index decode from K - (127 - q mod 64)); for a fixed
// train the j term is (column max over the query tiles + the wave transpose, as the fused kernel).
// No VALU op builds a key: per element 0.5 (row max3) + 0.5 (column max) + the transpose, against
// the fused key kernel's mad24 + max3 + add + max3 + transpose.  Padded queries get eight -128
// digits (K <= -65536 + 254, below every real key >= -32768); padded trains the prep's ROW_PAD.
// Outputs the fused kernel's formats: rowres (n_q - d1, J1) per query, column winners merged by
// 64-bit atomicMax into one row per pair (colpart zeroed before the launch); both_finalize_kernel
// then writes (a, b) and (b, a).
template <bool ROWS>
__global__ __launch_bounds__(64 * MU_WAVES, MU_MINW) void ham_key_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ crow_tab,
    const uint8_t* __restrict__ zero_row, const int32_t* __restrict__ pairs, int n_qblk,
    const int32_t* __restrict__ pair_order, int n_blk, int4* __restrict__ rowres,
    unsigned long long* __restrict__ colpart) {
    constexpr int D = 256, QT = Geo<D>::QT, QB = mu_qb<D>(), CHUNK = MU_CHUNK_BYTES / D;
    constexpr int NK = Geo<D>::NK, SLOTS = Geo<D>::SLOTS, NT = CHUNK / 32, NTHR = 64 * MU_WAVES;
    constexpr int PIECES = CHUNK * D / 1024 / MU_WAVES, RPP = 1024 / D;
    static_assert(QT == 2 && QT * 32 <= 128, "query index field: 127 - q mod 64");
    __shared__ __attribute__((aligned(16))) unsigned char lds0[CHUNK * D + CHUNK * 4];
    __shared__ __attribute__((aligned(16))) unsigned char lds1[CHUNK * D + CHUNK * 4];
    extern __shared__ unsigned long long lds_col[];  // [k_pad], dynamic

    const int per_xcd = (int)(gridDim.x >> 3);
    const int sblk = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
    if (sblk >= n_blk) return;  // block-uniform, before any barrier
    const int p = pair_order[sblk / n_qblk], qb = sblk % n_qblk;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    for (int j = tid; j < k_pad; j += NTHR) lds_col[j] = 0ull;

    const uint8_t* db = desc + (size_t)b * k_max * D;
    const int32_t* crb = crow_tab + (size_t)b * k_pad;
    const int n_chunk = (nb + CHUNK - 1) / CHUNK;
    auto stage = [&](int ch, unsigned char* dst) {
#pragma unroll
        for (int i = 0; i < PIECES; ++i) {
            const int piece = wave * PIECES + i;
            const int row = piece * RPP + lane / SLOTS;
            const int slot = (lane % SLOTS) ^ swz<D>(row);
            const int j = ch * CHUNK + row;
            const uint8_t* src = (j < nb) ? db + (size_t)j * D + slot * 16 : zero_row + slot * 16;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + piece * 1024), 16, 0, 0);
        }
        if (wave == 0 && lane < CHUNK / 4) {
            const int32_t* src = crb + ch * CHUNK + lane * 4;
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(dst + CHUNK * D), 16, 0, 0);
        }
    };

    const int qbase = qb * QB + wave * QT * 32;
    const bool active = qbase < na;  // wave-uniform
    v4i bq[QT][NK], bx[QT];
    int nq[QT], tb[QT], B1[QT], J1[QT];
    const uint8_t* da = desc + (size_t)a * k_max * D;
    // the extra k-step: A = 64 in bytes 0..7 and 1 in byte 8 of the lane-half-0 fragment
    const v4i ax = h ? v4i{0, 0, 0, 0} : v4i{0x40404040, 0x40404040, 1, 0};
#pragma unroll
    for (int c = 0; c < QT; ++c) {
        const int q = qbase + c * 32 + r32;
        const v4i* src = (const v4i*)((q < na) ? da + (size_t)q * D + (D / 2) * h : zero_row + (D / 2) * h);
#pragma unroll
        for (int s = 0; s < NK; ++s) bq[c][s] = src[s];
        nq[c] = (q < na) ? norm[(size_t)a * k_pad + q] : 0;
        // digits of -2 n_q (each in [-128, 0]) in bytes 0..7, 127 - q mod 64 in byte 8
        const int m = (q < na) ? 2 * nq[c] : 1024;
        unsigned w0 = 0, w1 = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int dgt = -min(max(m - 128 * t, 0), 128);
            const unsigned byte = (unsigned)(dgt & 0xFF);
            if (t < 4) w0 |= byte << (8 * t); else w1 |= byte << (8 * (t - 4));
        }
        bx[c] = h ? v4i{0, 0, 0, 0} : v4i{(int)w0, (int)w1, 127 - (c * 32 + r32), 0};
        tb[c] = INT_MIN; B1[c] = INT_MIN; J1[c] = -1;
    }
    const int rr = ((lane >> 1) & 1) * 8 + ((lane >> 2) & 1) * 4 + ((lane >> 3) & 1) * 2 +
                   ((lane >> 4) & 1);
    const int rowoff = (rr & 3) + 8 * (rr >> 2) + 4 * h;
    // merge the 128-train group's running row maximum into (best, argbest)
    auto row_merge = [&](int gbase) {
#pragma unroll
        for (int c = 0; c < QT; ++c) {
            const int v = tb[c] - (127 - (c * 32 + r32));  // -128 d + (127 - j mod 128)
            const int v1 = v >> 7;
            const int j1 = gbase + 127 - (v & 127);
            const bool up = v1 > B1[c];
            J1[c] = up ? j1 : J1[c];
            B1[c] = up ? v1 : B1[c];
            tb[c] = INT_MIN;
        }
    };

    auto process = [&](int ch, const unsigned char* cur, unsigned char* nxt) {
        if (ch + 1 < n_chunk) stage(ch + 1, nxt);
        const int nt = min(NT, (nb - ch * CHUNK + 31) >> 5);
        if (active) {
            const unsigned char* A = cur;
            const int* Ci = (const int*)(cur + CHUNK * D);
            for (int tt = 0; tt < nt; ++tt) {
                const int row = tt * 32 + r32;
                const int sw = swz<D>(row);
                v4i af[NK];
#pragma unroll
                for (int s = 0; s < NK; ++s)
                    af[s] = *(const v4i*)(A + row * D + ((((SLOTS / 2) * h + s) ^ sw) << 4));
                v16i init;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const v4i cv = *(const v4i*)(Ci + tt * 32 + 8 * g + 4 * h);
                    init[4 * g + 0] = cv.x; init[4 * g + 1] = cv.y;
                    init[4 * g + 2] = cv.z; init[4 * g + 3] = cv.w;
                }
                v16i acc0 = init, acc1 = init;
#pragma unroll
                for (int s = 0; s < NK; ++s) {
                    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[0][s], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[1][s], acc1, 0, 0, 0);
                }
                acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ax, bx[0], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ax, bx[1], acc1, 0, 0, 0);
                int colacc[16];
#pragma unroll
                for (int r = 0; r < 16; r += 2) {
                    // the column max first: compiler-emitted, so the MFMA -> VALU read hazard
                    // is padded (hipcc pads nothing into an asm statement); the row max3 is asm
                    // ordered after it through the extra operands (one v_max3 per 2 elements)
                    colacc[r] = max(acc0[r], acc1[r]);
                    colacc[r + 1] = max(acc0[r + 1], acc1[r + 1]);
                    if constexpr (ROWS) {
                        tb[0] = vmax3_after(tb[0], acc0[r], acc0[r + 1], colacc[r], colacc[r + 1]);
                        tb[1] = vmax3_after(tb[1], acc1[r], acc1[r + 1], colacc[r], colacc[r + 1]);
                    }
                }
                const int key = transpose_max16(colacc, lane);
                const int j = ch * CHUNK + tt * 32 + rowoff;
                const int e = key - (127 - (j & 127));   // -128 d + (127 - q_in_wave)
                const int nd = e >> 7;                    // -d; padded queries: < -256
                if (!(lane & 1) && j < nb && nd >= -256) {
                    const unsigned gq = (unsigned)(qbase + 127 - (e & 127));
                    lds_max_u64(&lds_col[j], ((unsigned long long)((unsigned)nd ^ 0x80000000u) << 32) |
                                                 (unsigned long long)(0xFFFFFFFFu - gq));
                }
                if (ROWS) {
                    const int g = ch * NT + tt;          // global tile: groups of 4 = 128 trains
                    if ((g & 3) == 3 || ch * CHUNK + tt * 32 + 32 >= nb) row_merge((g & ~3) * 32);
                }
            }
        }
    };
    if (n_chunk > 0) stage(0, lds0);
    __syncthreads();
    for (int ch = 0; ch < n_chunk; ch += 2) {
        process(ch, lds0, lds1);
        __syncthreads();
        if (ch + 1 < n_chunk) process(ch + 1, lds1, lds0);
        __syncthreads();
    }
    if (ROWS && active) {
#pragma unroll
        for (int c = 0; c < QT; ++c) {
            const int P1 = __shfl_xor(B1[c], 32), PJ = __shfl_xor(J1[c], 32);
            const bool take = (P1 > B1[c]) || (P1 == B1[c] && PJ >= 0 && PJ < J1[c]);
            if (take) { B1[c] = P1; J1[c] = PJ; }
            const int q = qbase + c * 32 + r32;
            // the fused kernel's row record: x = n_q - d1 (= vr), y = J1
            if (h == 0 && q < na)
                rowres[(size_t)p * k_pad + q] =
                    make_int4(B1[c] == INT_MIN ? INT_MIN : nq[c] + B1[c], J1[c], INT_MIN, 0);
        }
    }
    unsigned long long* dst = colpart + (size_t)p * k_pad;
    for (int j = tid; j < k_pad; j += NTHR) {
        const unsigned long long v = lds_col[j];
        if (v != 0ull) atomicMax(dst + j, v);
    }
}

// Exact dot product of two D-byte i8 rows (v_dot4_i32_i8).
template <int D>
__device__ __forceinline__ int mu_dot(const uint4* x, const uint4* y) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < D / 16; ++k) {
        const uint4 u = x[k], v = y[k];
        s = __builtin_amdgcn_sdot4((int)u.x, (int)v.x, s, false);
        s = __builtin_amdgcn_sdot4((int)u.y, (int)v.y, s, false);
        s = __builtin_amdgcn_sdot4((int)u.z, (int)v.z, s, false);
        s = __builtin_amdgcn_sdot4((int)u.w, (int)v.w, s, false);
    }
    return s;
}

// Finalize of the mutual kernel (block of MU_FT threads per pair; dynamic LDS: k_pad u64).
// A wide block: every pass over the trains / queries is one global round trip, so fewer passes
// (2 at k = 2048) is what makes this latency-bound kernel fast.
#ifndef MU_FT_THREADS
#define MU_FT_THREADS 512  // 256: +0.5 % K1 at cfg4 (k1_variants_ab.txt)
#endif
constexpr int MU_FT = MU_FT_THREADS;
template <int D>
__global__ __launch_bounds__(MU_FT) void mutual_finalize_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ pairs, int n_qblk,
    const int4* __restrict__ rowres, const unsigned long long* __restrict__ colpart, int rnum,
    int rden, long long max_dist, int32_t* __restrict__ out_count, int32_t* __restrict__ out_match,
    int32_t* __restrict__ out_dist) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_best[];
    __shared__ int wsum[MU_FT / 64], slow[MU_FT], nslow;
    __shared__ long long rb1[MU_FT], rb2[MU_FT];
    __shared__ int rj1[MU_FT];
    __shared__ unsigned char keepx[MU_FT];
    __shared__ int jx[MU_FT], dx[MU_FT];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    if (na <= 0 || nb <= 0) {
        if (tid == 0) out_count[p] = 0;
        return;
    }
    const unsigned long long* cp = colpart + (size_t)p * n_qblk * k_pad;
    const int32_t* na_norm = norm + (size_t)a * k_pad;
    const int32_t* nb_norm = norm + (size_t)b * k_pad;
    constexpr bool SQ = D == 128;  // L2 reports d^2 (ratio on squares), Hamming d
    constexpr int RS = D / 16;     // uint4 per feature row
    const uint4* qa = (const uint4*)(desc + (size_t)a * k_max * D);
    const uint4* dbv = (const uint4*)(desc + (size_t)b * k_max * D);
    int32_t* om = out_match + (size_t)p * k_max * 2;
    int32_t* od = out_dist + (size_t)p * k_max;
    auto col_winner = [&](int j) {  // train j's nearest query (lowest index), or -1
        unsigned long long best = 0;
        for (int q = 0; q < n_qblk; ++q) best = max(best, cp[(size_t)q * k_pad + j]);
        return best == 0 ? -1 : (int)(0xFFFFFFFFu - (unsigned)best);
    };
    for (int i = tid; i < na; i += MU_FT) lds_best[i] = ~0ull;
    __syncthreads();
    for (int j = tid; j < nb; j += MU_FT) {
        unsigned long long best = 0;
        for (int q = 0; q < n_qblk; ++q) best = max(best, cp[(size_t)q * k_pad + j]);
        if (best == 0) continue;
        const int nd = (int)((unsigned)(best >> 32) ^ 0x80000000u);
        const int gq = (int)(0xFFFFFFFFu - (unsigned)best);
        if (gq < 0 || gq >= na) continue;  // defensive: a column winner is always a query
        const long long d = -(long long)nd - (nb_norm[j] & 1);
        atomicMin(&lds_best[gq], ((unsigned long long)d << 32) | (unsigned)j);
    }
    __syncthreads();
    int base = 0;
    for (int i0 = 0; i0 < na; i0 += MU_FT) {
        const int i = i0 + tid;
        bool keep = false, sl = false;
        int jj = 0;
        long long d1 = 0;
        if (tid == 0) nslow = 0;
        if (i < na) {
            const int2 r = ((const int2*)rowres)[(size_t)p * k_pad + i];
            const long long A = na_norm[i];
            const unsigned long long e = lds_best[i];
            const long long Dp = e != ~0ull ? (long long)(e >> 32) : sfm::DIST_INF;  // best proposal
            const long long d1lo = max(A - 2LL * r.x - 1, 0LL);
            const long long d2lo = r.y > MU_E_VALID ? A - 2LL * r.y - 1 : sfm::DIST_INF;
            const long long d2hi = r.y > MU_E_VALID ? A - 2LL * r.y : sfm::DIST_INF;
            // not mutual: no train whose nearest query is i lies within the nearest distance
            // (if i were mutual with its nearest neighbour j1, j1 would propose d1 <= A - 2e1);
            // then the bounds: the ratio test / max_dist cannot pass even at the favourable ends
            if (Dp <= A - 2LL * r.x && sfm::ratio_ok(d1lo, d2hi, rnum, rden, SQ) &&
                (max_dist < 0 || d1lo < max_dist)) {
                if (r.x == r.y) {
                    sl = true;  // nearest neighbour not unique in e: exact row scan
                } else {        // unique nearest neighbour = the proposing train, d1 = D exactly
                    d1 = Dp;
                    jj = (int)(unsigned)e;
                    if (sfm::ratio_ok(d1, d2lo, rnum, rden, SQ)) keep = true;
                    else if (sfm::ratio_ok(d1, d2hi, rnum, rden, SQ)) sl = true;
                    keep = keep && (max_dist < 0 || d1 < max_dist);
                }
            }
        }
        keepx[tid] = keep;
        jx[tid] = jj;
        dx[tid] = (int)d1;
        __syncthreads();
        if (sl) slow[atomicAdd(&nslow, 1)] = tid;
        __syncthreads();
        const int ns = nslow;
        for (int s = 0; s < ns; ++s) {  // exact row scan of query i0 + slow[s] (rare)
            const int who = slow[s], q = i0 + who;
            uint4 x[RS];
#pragma unroll
            for (int u = 0; u < RS; ++u) x[u] = qa[(size_t)q * RS + u];
            long long b1 = sfm::DIST_INF, b2 = sfm::DIST_INF;
            int j1 = INT_MAX;
            for (int j = tid; j < nb; j += MU_FT) {
                const long long d = (long long)na_norm[q] + nb_norm[j] - 2LL * mu_dot<D>(x, dbv + (size_t)j * RS);
                if (d < b1) { b2 = b1; b1 = d; j1 = j; } else if (d < b2) { b2 = d; }
            }
            rb1[tid] = b1; rb2[tid] = b2; rj1[tid] = j1;
            __syncthreads();
            for (int st = MU_FT / 2; st > 0; st >>= 1) {
                if (tid < st) {
                    const long long ob1 = rb1[tid + st], ob2 = rb2[tid + st];
                    const int oj = rj1[tid + st];
                    const bool other = ob1 < rb1[tid] || (ob1 == rb1[tid] && oj < rj1[tid]);
                    const long long m2 = min(min(rb2[tid], ob2), other ? rb1[tid] : ob1);
                    if (other) { rb1[tid] = ob1; rj1[tid] = oj; }
                    rb2[tid] = m2;
                }
                __syncthreads();
            }
            if (tid == 0) {
                const int n1 = rj1[0];
                bool k = n1 >= 0 && n1 < nb && col_winner(n1) == q;
                k = k && sfm::ratio_ok(rb1[0], rb2[0], rnum, rden, SQ);
                k = k && (max_dist < 0 || rb1[0] < max_dist);
                keepx[who] = k;
                jx[who] = n1;
                dx[who] = (int)rb1[0];
            }
            __syncthreads();
        }
        const bool kk = i < na && keepx[tid];
        base = sfm::compact_n<MU_FT>(kk, i, jx[tid], dx[tid], base, wsum, om, od);
    }
    if (tid == 0) out_count[p] = base;
}

// Finalize of the column-only kernel, the OpenCV cross-check rule (oracle_match cross_check 2, the
// reference's BFMatcher(crossCheck=True), code/feature_matching.py:48): every train j proposes
// (d, j) to its nearest query; each query keeps the smallest proposal (lowest j on ties).
__global__ __launch_bounds__(256) void opencv_finalize_kernel(
    const int32_t* __restrict__ n_kp, int k_max, int k_pad, const int32_t* __restrict__ norm,
    const int32_t* __restrict__ pairs, int n_qblk, const unsigned long long* __restrict__ colpart,
    long long max_dist, int32_t* __restrict__ out_count, int32_t* __restrict__ out_match,
    int32_t* __restrict__ out_dist) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_best[];
    __shared__ int wsum[4];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    if (na <= 0 || nb <= 0) {
        if (tid == 0) out_count[p] = 0;
        return;
    }
    const unsigned long long* cp = colpart + (size_t)p * n_qblk * k_pad;
    const int32_t* nb_norm = norm + (size_t)b * k_pad;
    for (int i = tid; i < na; i += 256) lds_best[i] = ~0ull;
    __syncthreads();
    for (int j = tid; j < nb; j += 256) {
        unsigned long long best = 0;
        for (int q = 0; q < n_qblk; ++q) best = max(best, cp[(size_t)q * k_pad + j]);
        if (best == 0) continue;
        const int nd = (int)((unsigned)(best >> 32) ^ 0x80000000u);  // -d - p_j
        const int gq = (int)(0xFFFFFFFFu - (unsigned)best);
        if (gq < 0 || gq >= na) continue;
        const long long d = -(long long)nd - (nb_norm[j] & 1);
        atomicMin(&lds_best[gq], ((unsigned long long)d << 32) | (unsigned)j);
    }
    __syncthreads();
    int base = 0;
    int32_t* om = out_match + (size_t)p * k_max * 2;
    int32_t* od = out_dist + (size_t)p * k_max;
    for (int i0 = 0; i0 < na; i0 += 256) {
        const int i = i0 + tid;
        bool keep = false;
        int j = 0, d = 0;
        if (i < na) {
            const unsigned long long e = lds_best[i];
            if (e != ~0ull) {
                d = (int)(e >> 32);
                j = (int)(unsigned)e;
                keep = max_dist < 0 || (long long)d < max_dist;
            }
        }
        base = sfm::compact256(keep, i, j, d, base, wsum, om, od);
    }
    if (tid == 0) out_count[p] = base;
}

// Both directions of an unordered pair (a, b) from ONE fused-key tile (sfm_match_batch_both; the
// reference enumerates ordered pairs i != j, code/pipeline.py:38-41).  The tile holds, per query i
// of a, its nearest train J1[i] of b (exact, lowest index) with d1 = n_i - B1, and per train j of b
// its nearest query of a (exact, lowest index) in colpart.  Forward (a, b) = the usual finalize;
// reverse (b, a) swaps the roles: the queries are b's rows (the tile's columns), the trains a's.
//   OpenCV rule:  forward — every train j proposes (d, j) to its nearest query, each query keeps
//                 the smallest proposal (lowest j on ties);  reverse — every row i proposes
//                 (d1[i], i) to J1[i] (the train-side NN of the reverse problem), each column j
//                 keeps the smallest (lowest i on ties): oracle_match cross_check 2 on (b, a).
//   mutual:       forward keeps i iff colwin(J1[i]) = i;  reverse keeps j iff J1[colwin(j)] = j.
//   none:         forward (J1[i], d1[i]);  reverse (colwin(j), its d).
// No ratio test (it needs the reverse problem's second-best; the caller matches both orders).
// Outputs: pair p's forward result in slot p, its reverse (n_dirs = 2) in slot n_pairs + p.
// n_dirs = 1 is the single-order Hamming path (ham_key_kernel, sfm_match_batch).
__global__ __launch_bounds__(256) void both_finalize_kernel(
    const int32_t* __restrict__ n_kp, int k_max, int k_pad, const int32_t* __restrict__ norm,
    const int32_t* __restrict__ pairs, int n_pairs, int n_qblk, const int4* __restrict__ rowres,
    const unsigned long long* __restrict__ colpart, int xc, long long max_dist,
    int32_t* __restrict__ out_count, int32_t* __restrict__ out_match,
    int32_t* __restrict__ out_dist, int n_dirs) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_best[];
    __shared__ int wsum[4];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    if (na <= 0 || nb <= 0) {
        if (tid == 0) {
            out_count[p] = 0;
            if (n_dirs == 2) out_count[n_pairs + p] = 0;
        }
        return;
    }
    const unsigned long long* cp = colpart + (size_t)p * n_qblk * k_pad;
    const int4* rr = rowres + (size_t)p * k_pad;
    const int32_t* na_norm = norm + (size_t)a * k_pad;
    // train j's nearest query (lowest index) and its distance; false if none
    auto col_winner = [&](int j, int& q, int& d) {
        unsigned long long best = 0;
        for (int k = 0; k < n_qblk; ++k) best = max(best, cp[(size_t)k * k_pad + j]);
        if (best == 0) return false;
        d = -(int)((unsigned)(best >> 32) ^ 0x80000000u);
        q = (int)(0xFFFFFFFFu - (unsigned)best);
        return q >= 0 && q < na;
    };
    // query i's nearest train (lowest index) and its distance; false if none
    auto row_winner = [&](int i, int& j, int& d) {
        const int4 r = rr[i];
        j = r.y;
        d = na_norm[i] - r.x;
        return j >= 0 && j < nb && r.x > VALID_MIN;
    };
    auto dist_ok = [&](int d) { return max_dist < 0 || (long long)d < max_dist; };
    for (int dir = 0; dir < n_dirs; ++dir) {
        const int nq = dir == 0 ? na : nb;   // queries of this direction
        const int nt = dir == 0 ? nb : na;   // its trains
        const size_t slot = (size_t)(dir == 0 ? p : n_pairs + p);
        int32_t* om = out_match + slot * k_max * 2;
        int32_t* od = out_dist + slot * k_max;
        if (xc == SFM_XC_OPENCV) {
            for (int i = tid; i < nq; i += 256) lds_best[i] = ~0ull;
            __syncthreads();
            for (int t = tid; t < nt; t += 256) {  // train t proposes to its nearest query
                int q, d;
                const bool ok = dir == 0 ? col_winner(t, q, d) : row_winner(t, q, d);
                if (ok) atomicMin(&lds_best[q], ((unsigned long long)(unsigned)d << 32) | (unsigned)t);
            }
            __syncthreads();
        }
        int base = 0;
        for (int i0 = 0; i0 < nq; i0 += 256) {
            const int i = i0 + tid;
            bool keep = false;
            int j = 0, d = 0;
            if (i < nq) {
                if (xc == SFM_XC_OPENCV) {
                    const unsigned long long e = lds_best[i];
                    if (e != ~0ull) {
                        d = (int)(e >> 32);
                        j = (int)(unsigned)e;
                        keep = true;
                    }
                } else {
                    keep = dir == 0 ? row_winner(i, j, d) : col_winner(i, j, d);
                    if (keep && xc == SFM_XC_MUTUAL) {
                        int back, dd;
                        keep = (dir == 0 ? col_winner(j, back, dd) : row_winner(j, back, dd)) &&
                               back == i;
                    }
                }
                keep = keep && dist_ok(d);
            }
            base = sfm::compact256(keep, i, j, d, base, wsum, om, od);
        }
        if (tid == 0) out_count[slot] = base;
        __syncthreads();  // lds_best is reused by the reverse direction
    }
}

}  // namespace

// MFMA matcher for both metrics (L2: D = 128; Hamming: D = 256 bit-expanded).
static int mfma_match_launch(sfm_ctx* ctx, int metric, const uint8_t* desc, const int32_t* n_kp,
                             int32_t n_img, int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                             const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                             int32_t* out_dist) {
    hipStream_t st = ctx->stream;
    if (k_max == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_pairs, st));
        return SFM_OK;
    }
    const bool l2 = metric == SFM_METRIC_L2;
    const int D = l2 ? 128 : 256;
    const int QB = l2 ? Geo<128>::QB : Geo<256>::QB;
    const int k_pad = (int)sfm::align_up((size_t)k_max, KALIGN);
    if (k_pad > KMAX_L2) {
        sfm::set_error("sfm_match_batch: MFMA matcher needs k_max <= 4096");
        return SFM_ERR_INVALID;
    }
    const int n_qblk = (k_max + QB - 1) / QB;
    const size_t tab = (size_t)n_img * k_pad * sizeof(int32_t);
    const size_t rowb = (size_t)n_pairs * k_pad * sizeof(int4);
    const size_t colb = (size_t)n_pairs * n_qblk * k_pad * sizeof(unsigned long long);
    const size_t descb = sfm::align_up((size_t)n_img * k_max * D, 256);
    const size_t ordb = sfm::align_up(sizeof(int32_t) * ((size_t)n_pairs + n_img), 256);
    char* ws = (char*)sfm::workspace(ctx, 256 + 2 * tab + rowb + colb + descb + ordb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    uint8_t* zero_row = (uint8_t*)ws;
    int32_t* norm = (int32_t*)(ws + 256);
    int32_t* crow = (int32_t*)(ws + 256 + tab);
    int4* rowres = (int4*)(ws + 256 + 2 * tab);
    unsigned long long* colpart = (unsigned long long*)(ws + 256 + 2 * tab + rowb);
    uint8_t* desc_i8 = (uint8_t*)(ws + 256 + 2 * tab + rowb + colb);
    int32_t* pair_order = (int32_t*)(ws + 256 + 2 * tab + rowb + colb + descb);
    const int n_blk = n_pairs * n_qblk;
    const int grid = 8 * ((n_blk + 7) / 8);  // every XCD gets the same number of block slots
    hipLaunchKernelGGL(pair_order_kernel, dim3(1), dim3(1024), sizeof(int) * (size_t)n_img, st, pairs, n_pairs, n_img,
                       pair_order, pair_order + n_pairs);
    SFM_HIP_CHECK(hipGetLastError());
    if (l2) {
        hipLaunchKernelGGL(mfma_prep_kernel<SFM_METRIC_L2>, dim3(k_pad / 256, n_img), dim3(256), 0,
                           st, desc, n_kp, k_max, k_pad, norm, crow, zero_row, (uint4*)desc_i8);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(mfma_match_kernel<128>, dim3(grid), dim3(512), 0, st,
                           desc_i8, n_kp, k_max, k_pad, norm, crow, zero_row, pairs, n_qblk,
                           pair_order, n_blk, rowres, colpart);
    } else {
        hipLaunchKernelGGL(mfma_prep_kernel<SFM_METRIC_HAMMING>, dim3(k_pad / 256, n_img),
                           dim3(256), 0, st, desc, n_kp, k_max, k_pad, norm, crow, zero_row,
                           (uint4*)desc_i8);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(mfma_match_kernel<256>, dim3(grid), dim3(512), 0, st,
                           desc_i8, n_kp, k_max, k_pad, norm, crow, zero_row, pairs, n_qblk,
                           pair_order, n_blk, rowres, colpart);
    }
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(l2_finalize_kernel, dim3(n_pairs), dim3(256),
                       prm->cross_check == SFM_XC_OPENCV ? (size_t)k_pad * 8 : 0, st, n_kp, k_max,
                       k_pad, norm, pairs, n_qblk, rowres, colpart, prm->cross_check,
                       prm->ratio_num, prm->ratio_den, (long long)prm->max_dist, l2 ? 1 : 0,
                       out_count, out_match, out_dist);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

// Mutual (any ratio) or OpenCV cross check, both metrics: value-only row side + column winners
// (mutual), or the column side alone (OpenCV rule).
static int mfma_mutual_launch(sfm_ctx* ctx, int metric, const uint8_t* desc, const int32_t* n_kp,
                              int32_t n_img, int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                              const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                              int32_t* out_dist) {
    hipStream_t st = ctx->stream;
    if (k_max == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_pairs, st));
        return SFM_OK;
    }
    const bool l2 = metric == SFM_METRIC_L2;
    const bool rows = prm->cross_check == SFM_XC_MUTUAL;
    const int D = l2 ? 128 : 256;
    const int QB = l2 ? mu_qb<128>() : mu_qb<256>();
    const int k_pad = (int)sfm::align_up((size_t)k_max, KALIGN);
    SFM_REQUIRE(k_pad <= KMAX_MU, "sfm_match_batch: cross-check matcher needs k_max <= 8192");
    if (k_pad * 8 > 65536 - 1024) {  // the column state past 64 KB of dynamic LDS (k_max > 8064)
        // The attribute applies to the current device only, so it is set on every launch that needs
        // it (cheap) rather than once per process (a process may drive several GPUs).
        const int want = KMAX_MU * 8;
        const void* fns[] = {(const void*)mfma_mutual_kernel<128, true>,
                             (const void*)mfma_mutual_kernel<128, false>,
                             (const void*)mfma_mutual_kernel<256, true>,
                             (const void*)mfma_mutual_kernel<256, false>,
                             (const void*)mutual_finalize_kernel<128>,
                             (const void*)mutual_finalize_kernel<256>,
                             (const void*)opencv_finalize_kernel};
        for (const void* f : fns)
            SFM_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, want));
    }
    const int n_qblk = (k_max + QB - 1) / QB;
    const size_t tab = (size_t)n_img * k_pad * sizeof(int32_t);
    const size_t rowb = (size_t)n_pairs * k_pad * sizeof(int2);   // (e1, e2) per query
    const size_t colb = (size_t)n_pairs * n_qblk * k_pad * sizeof(unsigned long long);
    const size_t descb = sfm::align_up((size_t)n_img * k_max * D, 256);
    const size_t ordb = sfm::align_up(sizeof(int32_t) * ((size_t)n_pairs + n_img), 256);
    char* ws = (char*)sfm::workspace(ctx, 256 + 2 * tab + rowb + colb + descb + ordb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    uint8_t* zero_row = (uint8_t*)ws;
    int32_t* norm = (int32_t*)(ws + 256);
    int32_t* cinit = (int32_t*)(ws + 256 + tab);
    int4* rowres = (int4*)(ws + 256 + 2 * tab);
    unsigned long long* colpart = (unsigned long long*)(ws + 256 + 2 * tab + rowb);
    uint8_t* desc_i8 = (uint8_t*)(ws + 256 + 2 * tab + rowb + colb);
    int32_t* pair_order = (int32_t*)(ws + 256 + 2 * tab + rowb + colb + descb);
    const int n_blk = n_pairs * n_qblk;
    // column winners merged by atomics (default) or as per-query-block partials the finalize
    // reduces (SFM_MU_COLPART=1); DESIGN.md 4.1
    static const int col_atomic = [] {
        const char* e = getenv("SFM_MU_COLPART");
        return (e && e[0] == '1') ? 0 : 1;
    }();
    // whole pairs per XCD (blocks of one pair never straddle two XCDs' ranges)
    const int grid = 8 * ((n_pairs + 7) / 8) * n_qblk;
    const int fin_qblk = col_atomic ? 1 : n_qblk;
    if (col_atomic)
        SFM_HIP_CHECK(hipMemsetAsync(colpart, 0, sizeof(unsigned long long) * (size_t)n_pairs * k_pad, st));
    hipLaunchKernelGGL(pair_order_kernel, dim3(1), dim3(1024), sizeof(int) * (size_t)n_img, st,
                       pairs, n_pairs, n_img, pair_order, pair_order + n_pairs);
    SFM_HIP_CHECK(hipGetLastError());
    if (l2)
        hipLaunchKernelGGL((mfma_prep_kernel<SFM_METRIC_L2, true>), dim3(k_pad / 256, n_img),
                           dim3(256), 0, st, desc, n_kp, k_max, k_pad, norm, cinit, zero_row,
                           (uint4*)desc_i8);
    else
        hipLaunchKernelGGL((mfma_prep_kernel<SFM_METRIC_HAMMING, true>), dim3(k_pad / 256, n_img),
                           dim3(256), 0, st, desc, n_kp, k_max, k_pad, norm, cinit, zero_row,
                           (uint4*)desc_i8);
    SFM_HIP_CHECK(hipGetLastError());
#define SFM_MU_SCAN(DD, RR)                                                                       \
    hipLaunchKernelGGL((mfma_mutual_kernel<DD, RR>), dim3(grid), dim3(64 * MU_WAVES),             \
                       (size_t)k_pad * 8, st, desc_i8, n_kp,                                      \
                       k_max, k_pad, norm, cinit, zero_row, pairs, n_qblk, pair_order, n_blk,     \
                       rowres, colpart, col_atomic)
    if (l2 && rows) SFM_MU_SCAN(128, true);
    else if (l2) SFM_MU_SCAN(128, false);
    else if (rows) SFM_MU_SCAN(256, true);
    else SFM_MU_SCAN(256, false);
#undef SFM_MU_SCAN
    SFM_HIP_CHECK(hipGetLastError());
    if (rows) {
        if (l2)
            hipLaunchKernelGGL(mutual_finalize_kernel<128>, dim3(n_pairs), dim3(MU_FT),
                               (size_t)k_pad * 8, st, desc_i8, n_kp, k_max, k_pad, norm, pairs,
                               fin_qblk, rowres, colpart, prm->ratio_num, prm->ratio_den,
                               (long long)prm->max_dist, out_count, out_match, out_dist);
        else
            hipLaunchKernelGGL(mutual_finalize_kernel<256>, dim3(n_pairs), dim3(MU_FT),
                               (size_t)k_pad * 8, st, desc_i8, n_kp, k_max, k_pad, norm, pairs,
                               fin_qblk, rowres, colpart, prm->ratio_num, prm->ratio_den,
                               (long long)prm->max_dist, out_count, out_match, out_dist);
    } else {
        hipLaunchKernelGGL(opencv_finalize_kernel, dim3(n_pairs), dim3(256), (size_t)k_pad * 8, st,
                           n_kp, k_max, k_pad, norm, pairs, fin_qblk, colpart,
                           (long long)prm->max_dist, out_count, out_match, out_dist);
    }
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

// Both directions of every (unordered) pair from one tile (n_dirs = 2; no ratio test): Hamming on
// the key-in-the-accumulator kernel, L2 on the fused key kernel with TOP2 off.  n_dirs = 1 (Hamming
// only): the single-order call of sfm_match_batch on the same kernel (rows only when the rule
// needs them: not for the OpenCV rule).
static int match_tile_launch(sfm_ctx* ctx, int metric, const uint8_t* desc, const int32_t* n_kp,
                             int32_t n_img, int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                             const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                             int32_t* out_dist, int n_dirs) {
    hipStream_t st = ctx->stream;
    if (k_max == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_dirs * (size_t)n_pairs, st));
        return SFM_OK;
    }
    const bool rows = n_dirs == 2 || prm->cross_check != SFM_XC_OPENCV;
    const bool l2 = metric == SFM_METRIC_L2;
    // Hamming: the key-in-the-accumulator kernel (ham_key_kernel); SFM_HAM_BOTH=fused keeps the
    // fused key kernel (A/B only)
    static const bool ham_fused = [] {
        const char* e = getenv("SFM_HAM_BOTH");
        return e && strcmp(e, "fused") == 0;
    }();
    if (l2 && n_dirs != 2) {
        sfm::set_error("match_tile_launch: the single-order tile path is Hamming only");
        return SFM_ERR_INVALID;
    }
    const bool hkey = !l2 && (n_dirs == 1 || !ham_fused);
    const int D = l2 ? 128 : 256;
    const int QB = l2 ? Geo<128>::QB : (hkey ? mu_qb<256>() : Geo<256>::QB);
    const int k_pad = (int)sfm::align_up((size_t)k_max, KALIGN);
    SFM_REQUIRE(k_pad <= KMAX_L2, "sfm_match_batch_both: k_max <= 4096 required");
    const int n_qblk = (k_max + QB - 1) / QB;
    const size_t tab = (size_t)n_img * k_pad * sizeof(int32_t);
    const size_t rowb = (size_t)n_pairs * k_pad * sizeof(int4);
    const size_t colb = (size_t)n_pairs * n_qblk * k_pad * sizeof(unsigned long long);
    const size_t descb = sfm::align_up((size_t)n_img * k_max * D, 256);
    const size_t ordb = sfm::align_up(sizeof(int32_t) * ((size_t)n_pairs + n_img), 256);
    char* ws = (char*)sfm::workspace(ctx, 256 + 2 * tab + rowb + colb + descb + ordb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    uint8_t* zero_row = (uint8_t*)ws;
    int32_t* norm = (int32_t*)(ws + 256);
    int32_t* crow = (int32_t*)(ws + 256 + tab);
    int4* rowres = (int4*)(ws + 256 + 2 * tab);
    unsigned long long* colpart = (unsigned long long*)(ws + 256 + 2 * tab + rowb);
    uint8_t* desc_i8 = (uint8_t*)(ws + 256 + 2 * tab + rowb + colb);
    int32_t* pair_order = (int32_t*)(ws + 256 + 2 * tab + rowb + colb + descb);
    const int n_blk = n_pairs * n_qblk;
    const int grid = 8 * ((n_blk + 7) / 8);
    hipLaunchKernelGGL(pair_order_kernel, dim3(1), dim3(1024), sizeof(int) * (size_t)n_img, st,
                       pairs, n_pairs, n_img, pair_order, pair_order + n_pairs);
    SFM_HIP_CHECK(hipGetLastError());
    if (hkey) {
        SFM_HIP_CHECK(hipMemsetAsync(colpart, 0, sizeof(unsigned long long) * (size_t)n_pairs * k_pad, st));
        hipLaunchKernelGGL((mfma_prep_kernel<SFM_METRIC_HAMMING, false, 16>), dim3(k_pad / 256, n_img),
                           dim3(256), 0, st, desc, n_kp, k_max, k_pad, norm, crow, zero_row,
                           (uint4*)desc_i8);
        SFM_HIP_CHECK(hipGetLastError());
        // whole pairs per XCD (the column merge of a pair stays in one L2), as the mutual kernel
        const int hgrid = 8 * ((n_pairs + 7) / 8) * n_qblk;
        if (rows)
            hipLaunchKernelGGL(ham_key_kernel<true>, dim3(hgrid), dim3(64 * MU_WAVES),
                               (size_t)k_pad * 8, st, desc_i8, n_kp, k_max, k_pad, norm, crow,
                               zero_row, pairs, n_qblk, pair_order, n_blk, rowres, colpart);
        else
            hipLaunchKernelGGL(ham_key_kernel<false>, dim3(hgrid), dim3(64 * MU_WAVES),
                               (size_t)k_pad * 8, st, desc_i8, n_kp, k_max, k_pad, norm, crow,
                               zero_row, pairs, n_qblk, pair_order, n_blk, rowres, colpart);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(both_finalize_kernel, dim3(n_pairs), dim3(256), (size_t)k_pad * 8, st,
                           n_kp, k_max, k_pad, norm, pairs, n_pairs, 1, rowres, colpart,
                           prm->cross_check, (long long)prm->max_dist, out_count, out_match,
                           out_dist, n_dirs);
        SFM_HIP_CHECK(hipGetLastError());
        return SFM_OK;
    }
    if (l2) {
        hipLaunchKernelGGL(mfma_prep_kernel<SFM_METRIC_L2>, dim3(k_pad / 256, n_img), dim3(256), 0,
                           st, desc, n_kp, k_max, k_pad, norm, crow, zero_row, (uint4*)desc_i8);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL((mfma_match_kernel<128, false>), dim3(grid), dim3(512), 0, st, desc_i8,
                           n_kp, k_max, k_pad, norm, crow, zero_row, pairs, n_qblk, pair_order,
                           n_blk, rowres, colpart);
    } else {
        hipLaunchKernelGGL(mfma_prep_kernel<SFM_METRIC_HAMMING>, dim3(k_pad / 256, n_img),
                           dim3(256), 0, st, desc, n_kp, k_max, k_pad, norm, crow, zero_row,
                           (uint4*)desc_i8);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL((mfma_match_kernel<256, false>), dim3(grid), dim3(512), 0, st, desc_i8,
                           n_kp, k_max, k_pad, norm, crow, zero_row, pairs, n_qblk, pair_order,
                           n_blk, rowres, colpart);
    }
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(both_finalize_kernel, dim3(n_pairs), dim3(256), (size_t)k_pad * 8, st, n_kp,
                       k_max, k_pad, norm, pairs, n_pairs, n_qblk, rowres, colpart,
                       prm->cross_check, (long long)prm->max_dist, out_count, out_match, out_dist,
                       2);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

int sfm_match_both_launch(sfm_ctx* ctx, int metric, const uint8_t* desc, const int32_t* n_kp,
                          int32_t n_img, int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                          const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                          int32_t* out_dist) {
    return match_tile_launch(ctx, metric, desc, n_kp, n_img, k_max, pairs, n_pairs, prm, out_count,
                             out_match, out_dist, 2);
}

int sfm_match_l2_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                        int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                        const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                        int32_t* out_dist) {
    // Path per rule (cfg3, 1225 pairs x 2048): mutual or OpenCV cross check ->
    // the value-only-row / column-only kernel; ratio test without cross check -> the forward/
    // reverse path (match_l2fr.hip); no cross check and no ratio -> the fused key kernel.
    // SFM_L2_PATH=mutual|fr|fused overrides where the rule allows it.
    const char* pe = getenv("SFM_L2_PATH");
    const bool ratio = prm->ratio_den > 0;
    if (pe && strcmp(pe, "fused") == 0)
        return mfma_match_launch(ctx, SFM_METRIC_L2, desc, n_kp, n_img, k_max, pairs, n_pairs, prm,
                                 out_count, out_match, out_dist);
    if (pe && strcmp(pe, "fr") == 0 && ratio && prm->cross_check != SFM_XC_OPENCV)
        return sfm_match_l2fr_launch(ctx, desc, n_kp, n_img, k_max, pairs, n_pairs, prm,
                                     out_count, out_match, out_dist);
    if (prm->cross_check != SFM_XC_NONE)
        return mfma_mutual_launch(ctx, SFM_METRIC_L2, desc, n_kp, n_img, k_max, pairs, n_pairs,
                                  prm, out_count, out_match, out_dist);
    if (ratio)
        return sfm_match_l2fr_launch(ctx, desc, n_kp, n_img, k_max, pairs, n_pairs, prm,
                                     out_count, out_match, out_dist);
    return mfma_match_launch(ctx, SFM_METRIC_L2, desc, n_kp, n_img, k_max, pairs, n_pairs, prm,
                             out_count, out_match, out_dist);
}

int sfm_match_hamming_mfma_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp,
                                  int32_t n_img, int32_t k_max, const int32_t* pairs,
                                  int32_t n_pairs, const sfm_match_params* prm,
                                  int32_t* out_count, int32_t* out_match, int32_t* out_dist) {
    // Without a ratio test (the reference's rules) every cross-check rule runs on the
    // key-in-the-accumulator kernel (ham_key_kernel: no VALU key build; the row side only for the
    // mutual / no rule).  With a ratio test: the OpenCV rule on the column-winner
    // kernel, the others on the fused key kernel — with Hamming distances (0..256) ties in e are
    // the rule, and every tie would cost the value-only row side an exact row scan.
    // SFM_HAMMING_PATH=mutual|fused selects the round-3 kernels (A/B only).
    const char* pe = getenv("SFM_HAMMING_PATH");
    if (prm->ratio_den == 0 && !(pe && (strcmp(pe, "mutual") == 0 || strcmp(pe, "fused") == 0)))
        return match_tile_launch(ctx, SFM_METRIC_HAMMING, desc, n_kp, n_img, k_max, pairs, n_pairs,
                                 prm, out_count, out_match, out_dist, 1);
    const bool col = pe && strcmp(pe, "mutual") == 0 ? prm->cross_check != SFM_XC_NONE
                                                    : prm->cross_check == SFM_XC_OPENCV;
    if (col && !(pe && strcmp(pe, "fused") == 0))
        return mfma_mutual_launch(ctx, SFM_METRIC_HAMMING, desc, n_kp, n_img, k_max, pairs,
                                  n_pairs, prm, out_count, out_match, out_dist);
    return mfma_match_launch(ctx, SFM_METRIC_HAMMING, desc, n_kp, n_img, k_max, pairs, n_pairs,
                             prm, out_count, out_match, out_dist);
}

#ifdef MU_CLOCK
// Diagnostic build only (tools/build_variant.sh clock -DMU_CLOCK): the per-block (memtime start,
// realtime start, memtime end, realtime end) stamps of the last mfma_mutual_kernel launch.
extern "C" int sfm_debug_clock_stamps(unsigned long long* host, int32_t n_blocks) {
    const size_t n = MU_CLOCK_W * (size_t)std::min(n_blocks, MU_CLOCK_SLOTS);
    SFM_HIP_CHECK(hipDeviceSynchronize());
    SFM_HIP_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mu_clock), n * sizeof(unsigned long long)));
    return SFM_OK;
}
#endif
