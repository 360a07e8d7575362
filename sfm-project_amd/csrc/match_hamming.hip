// Brute-force Hamming matching of 256-bit ORB descriptors — the reference's own matcher:
// cv2.BFMatcher(cv2.NORM_HAMMING, crossCheck=True).match(des1, des2) at
// code/feature_matching.py:48-50, followed by the `distance < 26` cut of :53-58 (max_dist).
//
// The ORB sets of the reference are small (OpenCV default nfeatures = 500), so this is a plain
// VALU kernel: one 256-thread block per pair, descriptors staged through LDS in 1024-row chunks
// (every lane reads the same LDS row: broadcast), 8 x (xor + popcount) per distance.  Pass 1 keeps
// per-query (d1, argmin, d2); pass 2 swaps roles for the per-train nearest query.  The finalize
// applies the cross-check rule (OpenCV batchDistance semantics or strict mutual), the optional
// ratio test and max_dist, and compacts in ascending query order.
#include <algorithm>
#include <climits>

#include "match_common.h"

namespace {

constexpr int CH = 1024;  // rows per LDS chunk (32 KB)

__device__ __forceinline__ void load_row(const uint8_t* base, int row, unsigned (&v)[8]) {
    const uint4* p = (const uint4*)(base + (size_t)row * 32);
    uint4 x = p[0], y = p[1];
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}

// One direction: for each row of S (n_s rows) find the nearest rows of T (n_t rows):
// best distance, lowest-index argmin and the second smallest distance.
__device__ void nn_pass(const uint8_t* S, int n_s, const uint8_t* T, int n_t, uint4* lds,
                        int4* out) {
    const int tid = threadIdx.x;
    for (int i0 = 0; i0 < n_s; i0 += 256) {
        const int i = i0 + tid;
        unsigned q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i < n_s) load_row(S, i, q);
        int b1 = INT_MAX, b2 = INT_MAX, j1 = -1;
        for (int c0 = 0; c0 < n_t; c0 += CH) {
            const int n = min(CH, n_t - c0);
            __syncthreads();
            for (int e = tid; e < 2 * n; e += 256) lds[e] = ((const uint4*)(T + (size_t)c0 * 32))[e];
            __syncthreads();
            for (int jj = 0; jj < n; ++jj) {
                const uint4 x = lds[2 * jj], y = lds[2 * jj + 1];
                int d = __popc(q[0] ^ x.x) + __popc(q[1] ^ x.y) + __popc(q[2] ^ x.z) +
                        __popc(q[3] ^ x.w) + __popc(q[4] ^ y.x) + __popc(q[5] ^ y.y) +
                        __popc(q[6] ^ y.z) + __popc(q[7] ^ y.w);
                if (d < b1) { b2 = b1; b1 = d; j1 = c0 + jj; }
                else if (d < b2) { b2 = d; }
            }
        }
        if (i < n_s) out[i] = make_int4(b1, j1, b2, 0);
    }
}

__global__ __launch_bounds__(256) void hamming_nn_kernel(const uint8_t* __restrict__ desc,
                                                         const int32_t* __restrict__ n_kp,
                                                         int k_max, const int32_t* __restrict__ pairs,
                                                         int4* __restrict__ rowtab,
                                                         int4* __restrict__ coltab) {
    __shared__ uint4 lds[2 * CH];
    const int p = blockIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const uint8_t* A = desc + (size_t)a * k_max * 32;
    const uint8_t* B = desc + (size_t)b * k_max * 32;
    nn_pass(A, na, B, nb, lds, rowtab + (size_t)p * k_max);
    nn_pass(B, nb, A, na, lds, coltab + (size_t)p * k_max);
}

__global__ __launch_bounds__(256) void hamming_finalize_kernel(
    const int32_t* __restrict__ n_kp, int k_max, const int32_t* __restrict__ pairs,
    const int4* __restrict__ rowtab, const int4* __restrict__ coltab, int xc, int rnum, int rden,
    long long max_dist, int32_t* __restrict__ out_count, int32_t* __restrict__ out_match,
    int32_t* __restrict__ out_dist) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_best[];
    __shared__ int wsum[8];
    const int p = blockIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int na = n_kp[a], nb = n_kp[b];
    const int tid = threadIdx.x;
    const int4* rt = rowtab + (size_t)p * k_max;
    const int4* ct = coltab + (size_t)p * k_max;
    int32_t* om = out_match + (size_t)p * k_max * 2;
    int32_t* od = out_dist + (size_t)p * k_max;
    int base = 0;
    if (na <= 0 || nb <= 0) {
        if (tid == 0) out_count[p] = 0;
        return;
    }
    if (xc == SFM_XC_OPENCV) {
        // OpenCV batchDistance crosscheck: train j (ascending) claims its nearest query if its
        // distance is strictly smaller than the best claim so far -> min (d, j) per query.
        for (int i = tid; i < na; i += 256) lds_best[i] = ~0ull;
        __syncthreads();
        for (int j = tid; j < nb; j += 256) {
            const int4 c = ct[j];
            atomicMin(&lds_best[c.y], ((unsigned long long)(unsigned)c.x << 32) | (unsigned)j);
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
            int j = 0, d1 = 0;
            if (i < na) {
                const int4 r = rt[i];
                j = r.y;
                d1 = r.x;
                if (j >= 0) {
                    keep = (xc != SFM_XC_MUTUAL) || (ct[j].y == i);
                    const long long d2 = (r.z == INT_MAX) ? sfm::DIST_INF : (long long)r.z;
                    keep = keep && sfm::ratio_ok(d1, d2, rnum, rden, false);
                    keep = keep && (max_dist < 0 || (long long)d1 < max_dist);
                }
            }
            base = sfm::compact256(keep, i, j, d1, base, wsum, om, od);
        }
    }
    if (tid == 0) out_count[p] = base;
}

}  // namespace

int sfm_match_hamming_launch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp,
                             int32_t n_img, int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                             const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                             int32_t* out_dist) {
    (void)n_img;
    hipStream_t st = ctx->stream;
    if (k_max == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_pairs, st));
        return SFM_OK;
    }
    const size_t tb = (size_t)n_pairs * k_max * sizeof(int4);
    char* ws = (char*)sfm::workspace(ctx, 2 * tb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    int4* rowtab = (int4*)ws;
    int4* coltab = (int4*)(ws + tb);
    hipLaunchKernelGGL(hamming_nn_kernel, dim3(n_pairs), dim3(256), 0, st, desc, n_kp, k_max,
                       pairs, rowtab, coltab);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(hamming_finalize_kernel, dim3(n_pairs), dim3(256),
                       prm->cross_check == SFM_XC_OPENCV ? (size_t)k_max * 8 : 0, st, n_kp, k_max,
                       pairs, rowtab, coltab, prm->cross_check, prm->ratio_num, prm->ratio_den,
                       (long long)prm->max_dist, out_count, out_match, out_dist);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
