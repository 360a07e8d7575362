// All-pairs L2 descriptor matching on MFMA (K1, SURVEY.md §8a a1/a3').
//
// Replaces the arithmetic behind cv2.BFMatcher(...).match (code/feature_matching.py:48-50) for
// 128-byte SIFT-like descriptors, fused with the Lowe ratio test and the cross check.
//
// Exact integer formulation.  With x' = x - 128 (u8 -> i8, a free XOR 0x80):
//     d^2(i,j) = |x'_i|^2 + |y'_j|^2 - 2 x'_i.y'_j
// The dot products run on v_mfma_i32_32x32x32_i8 (exact int32).  For a fixed query i the best
// train maximises  vr = 2 dot - |y'_j|^2  (= |x'_i|^2 - d^2);  for a fixed train j the best
// query maximises  vc = 2 dot - |x'_i|^2  (= |y'_j|^2 - d^2).
//
// Tile geometry: MFMA output tile D[32 trains][32 queries]; the column (query) is the lane, the
// 16 accumulator registers of a lane are 16 of the 32 train rows (the other 16 are in lane^32).
//  * row direction (per query, top-2 over trains): lane-local.  Each register becomes the packed
//    key vr*32 + (31 - row) with ONE v_mad_i32_i24 (dot*64 + (31 - row - 32|y'|^2)); a
//    max3/med3 network keeps the tile top-2; the running (best, argbest, second) per query is
//    merged once per tile.
//  * column direction (per train, best query): the key vc*128 + (127 - q) (q = query slot in the
//    wave) is one more v_mad_i32_i24 and a v_max per element, reduced over the wave's 4 query
//    tiles in registers, then across the 32 lanes of each half with DPP, then across waves with
//    64-bit LDS atomics; one slab per workgroup is written to HBM and merged in the finalize.
// Every wave holds 4 query tiles (128 queries, B operand, 64 VGPRs); a 512-thread workgroup
// covers 1024 queries of one pair and streams all train tiles of the other image.
#include <algorithm>
#include <climits>

#include "match_common.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int QT = 4;                 // query tiles (32 each) per wave
constexpr int WAVES = 8;              // waves per workgroup
constexpr int QB = WAVES * QT * 32;   // queries per workgroup
constexpr int SENT_ROW = -1073741824; // Crow of padded trains: never wins (DESIGN.md §4.1 ranges)
constexpr int SENT_COL = -1476395008; // Ccol of padded queries
constexpr int COL_VALID_MIN = -940000000;  // col keys below come from padded queries only
constexpr int ROW_VALID_MIN = -(1 << 24);  // row values below come from padded trains only

__device__ __forceinline__ int imax3(int a, int b, int c) { return max(a, max(b, c)); }
__device__ __forceinline__ int imed3(int a, int b, int c) {
    return max(min(a, b), min(max(a, b), c));
}
__device__ __forceinline__ int mad24(int a, int b, int c) { return __mul24(a, b) + c; }

template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}

// max over the 32 lanes of each wave half (lanes 0-31 and 32-63 independently)
__device__ __forceinline__ int half_max32(int x) {
    x = max(x, dpp<0x121>(x));  // row_ror:1
    x = max(x, dpp<0x122>(x));  // row_ror:2
    x = max(x, dpp<0x124>(x));  // row_ror:4
    x = max(x, dpp<0x128>(x));  // row_ror:8
    int y = __builtin_amdgcn_ds_swizzle(x, 0x401F);  // lane ^ 16 within 32
    return max(x, y);
}

__device__ __forceinline__ v4i xor80(v4i v) {
    const int m = (int)0x80808080u;
    return v4i{v.x ^ m, v.y ^ m, v.z ^ m, v.w ^ m};
}

// |x'|^2 and the row constant per descriptor, padded to k_pad (multiple of 32).
__global__ void l2_prep_kernel(const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp,
                               int k_max, int k_pad, int32_t* __restrict__ norm,
                               int32_t* __restrict__ crow) {
    const int img = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k_pad) return;
    int nv = 0;
    if (j < k_max) {
        const uint4* p = (const uint4*)(desc + ((size_t)img * k_max + j) * 128);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            uint4 v = p[q];
            unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    int x = (int)((w[e] >> (8 * b)) & 0xFF) - 128;
                    nv += x * x;
                }
        }
    }
    const size_t o = (size_t)img * k_pad + j;
    norm[o] = nv;
    crow[o] = (j < n_kp[img]) ? (-32 * nv + 31 - (j & 31)) : SENT_ROW;
}

__global__ __launch_bounds__(512, 2) void l2_match_kernel(
    const uint8_t* __restrict__ desc, const int32_t* __restrict__ n_kp, int k_max, int k_pad,
    const int32_t* __restrict__ norm, const int32_t* __restrict__ crow_tab,
    const int32_t* __restrict__ pairs, int n_qblk, int4* __restrict__ rowres,
    unsigned long long* __restrict__ colpart) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_col[];
    const int p = blockIdx.x / n_qblk, qb = blockIdx.x - p * n_qblk;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
    for (int j = tid; j < k_pad; j += 512) lds_col[j] = 0ull;
    __syncthreads();

    const int qbase = qb * QB + wave * QT * 32;
    if (qbase < na) {
        const uint8_t* da = desc + (size_t)a * k_max * 128;
        const uint8_t* db = desc + (size_t)b * k_max * 128;
        const int32_t* crb = crow_tab + (size_t)b * k_pad;
        v4i bq[QT][4];
        int ccol[QT], B1[QT], J1[QT], B2[QT];
#pragma unroll
        for (int c = 0; c < QT; ++c) {
            const int q = qbase + c * 32 + r32;
            const int qq = min(q, k_max - 1);
            const v4i* src = (const v4i*)(da + (size_t)qq * 128 + 64 * h);
#pragma unroll
            for (int s = 0; s < 4; ++s) bq[c][s] = xor80(src[s]);
            ccol[c] = (q < na) ? (-128 * norm[(size_t)a * k_pad + q] + 127 - (c * 32 + r32))
                               : SENT_COL;
            B1[c] = INT_MIN; J1[c] = -1; B2[c] = INT_MIN;
        }
        const int nt = (nb + 31) >> 5;
        for (int t = 0; t < nt; ++t) {
            const int jj = min(t * 32 + r32, k_max - 1);
            const v4i* srcb = (const v4i*)(db + (size_t)jj * 128 + 64 * h);
            v4i af[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) af[s] = xor80(srcb[s]);
            int crow[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                v4i cv = *(const v4i*)(crb + t * 32 + 8 * g + 4 * h);
                crow[4 * g + 0] = cv.x; crow[4 * g + 1] = cv.y;
                crow[4 * g + 2] = cv.z; crow[4 * g + 3] = cv.w;
            }
            int colacc[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) colacc[r] = INT_MIN;
#pragma unroll
            for (int c = 0; c < QT; ++c) {
                v16i acc = {0};
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[c][s], acc, 0, 0, 0);
                // row direction: tile top-2 of packed keys
                int k0 = mad24(acc[0], 64, crow[0]), k1 = mad24(acc[1], 64, crow[1]);
                int tb = max(k0, k1), ts = min(k0, k1);
#pragma unroll
                for (int r = 2; r < 16; r += 2) {
                    int x = mad24(acc[r], 64, crow[r]);
                    int y = mad24(acc[r + 1], 64, crow[r + 1]);
                    ts = max(ts, imed3(tb, x, y));
                    tb = imax3(tb, x, y);
                }
                const int v1 = tb >> 5, v2 = ts >> 5;
                const int j1 = t * 32 + 31 - (tb & 31);
                const bool up = v1 > B1[c];
                B2[c] = up ? max(B1[c], v2) : max(B2[c], v1);
                J1[c] = up ? j1 : J1[c];
                B1[c] = max(B1[c], v1);
                // column direction
#pragma unroll
                for (int r = 0; r < 16; ++r) colacc[r] = max(colacc[r], mad24(acc[r], 256, ccol[c]));
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) colacc[r] = half_max32(colacc[r]);
            if (r32 == 0) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = colacc[r];
                    if (key > COL_VALID_MIN) {
                        const int row = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const unsigned vb = (unsigned)(key >> 7) ^ 0x80000000u;
                        const unsigned gq = (unsigned)(qbase + 127 - (key & 127));
                        const unsigned long long k64 =
                            ((unsigned long long)vb << 32) | (unsigned long long)(0xFFFFFFFFu - gq);
                        atomicMax(&lds_col[row], k64);
                    }
                }
            }
        }
        // merge the two halves' row state (same queries, complementary train rows)
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
    __syncthreads();
    unsigned long long* dst = colpart + ((size_t)p * n_qblk + qb) * k_pad;
    for (int j = tid; j < k_pad; j += 512) dst[j] = lds_col[j];
}

// Finalize: cross check + ratio + max distance, ordered compaction (one 256-thread block / pair).
__global__ __launch_bounds__(256) void l2_finalize_kernel(
    const int32_t* __restrict__ n_kp, int k_max, int k_pad, const int32_t* __restrict__ norm,
    const int32_t* __restrict__ pairs, int n_qblk, const int4* __restrict__ rowres,
    const unsigned long long* __restrict__ colpart, int xc, int rnum, int rden,
    long long max_dist, int32_t* __restrict__ out_count, int32_t* __restrict__ out_match,
    int32_t* __restrict__ out_dist) {
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
            const int v = (int)((unsigned)(best >> 32) ^ 0x80000000u);
            const int gq = (int)(0xFFFFFFFFu - (unsigned)best);
            const long long d = (long long)norm[(size_t)b * k_pad + j] - v;
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
                if (j >= 0) {
                    const long long nx = norm[(size_t)a * k_pad + i];
                    d1 = nx - rr.x;
                    const long long d2 = (rr.z > ROW_VALID_MIN) ? nx - rr.z : sfm::DIST_INF;
                    keep = true;
                    if (xc == SFM_XC_MUTUAL) {
                        unsigned long long best = 0;
                        for (int q = 0; q < n_qblk; ++q) best = max(best, cp[(size_t)q * k_pad + j]);
                        keep = (int)(0xFFFFFFFFu - (unsigned)best) == i;
                    }
                    keep = keep && sfm::ratio_ok(d1, d2, rnum, rden, true);
                    keep = keep && (max_dist < 0 || d1 < max_dist);
                }
            }
            base = sfm::compact256(keep, i, j, (int)d1, base, wsum, om, od);
        }
    }
    if (tid == 0) out_count[p] = base;
}

}  // namespace

int sfm_match_l2_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                        int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                        const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                        int32_t* out_dist) {
    const int k_pad = (int)sfm::align_up((size_t)std::max(k_max, 1), 32);
    const int n_qblk = (k_max + QB - 1) / QB;
    const size_t tab = (size_t)n_img * k_pad * sizeof(int32_t);
    const size_t rowb = (size_t)n_pairs * k_pad * sizeof(int4);
    const size_t colb = (size_t)n_pairs * n_qblk * k_pad * sizeof(unsigned long long);
    char* ws = (char*)sfm::workspace(ctx, 2 * tab + rowb + colb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    int32_t* norm = (int32_t*)ws;
    int32_t* crow = (int32_t*)(ws + tab);
    int4* rowres = (int4*)(ws + 2 * tab);
    unsigned long long* colpart = (unsigned long long*)(ws + 2 * tab + rowb);
    hipStream_t st = ctx->stream;
    if (k_max == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_pairs, st));
        return SFM_OK;
    }
    hipLaunchKernelGGL(l2_prep_kernel, dim3((k_pad + 255) / 256, n_img), dim3(256), 0, st, desc,
                       n_kp, k_max, k_pad, norm, crow);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(l2_match_kernel, dim3(n_pairs * n_qblk), dim3(512),
                       (size_t)k_pad * sizeof(unsigned long long), st, desc, n_kp, k_max, k_pad,
                       norm, crow, pairs, n_qblk, rowres, colpart);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(l2_finalize_kernel, dim3(n_pairs), dim3(256),
                       prm->cross_check == SFM_XC_OPENCV ? (size_t)k_pad * 8 : 0, st, n_kp, k_max,
                       k_pad, norm, pairs, n_qblk, rowres, colpart, prm->cross_check,
                       prm->ratio_num, prm->ratio_den, (long long)prm->max_dist, out_count,
                       out_match, out_dist);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
