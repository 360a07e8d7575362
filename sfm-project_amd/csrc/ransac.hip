// 8-point fundamental-matrix RANSAC (K2).
//
// Fills the empty reference module code/geometric_verification.py (placeholder at
// code/pipeline.py:60).  Three kernels per batch of pairs:
//   ransac_prep   one wave per pair: gathers the tentative-match pixel coordinates, Hartley-
//                 normalises each side with a fixed-order wave reduction, writes float4
//                 (x1,y1,x2,y2) normalised per match and the (cx,cy,s) of both sides.
//   ransac_hyp    one LANE per hypothesis (256 per block): counter-based Philox sample of 8 distinct
//                 matches (Floyd), Householder-QR null space of the 8x9 epipolar system, rank-2
//                 projection (5 Jacobi sweeps on F^T F), then a sweep over all M matches held in LDS
//                 (every lane reads the same float4: LDS broadcast) counting Sampson inliers.  The
//                 block argmax (max count, lowest h) is a wave shuffle reduction, then one 64-bit
//                 atomicMax per block into the pair's slot.
//   ransac_final  one block per pair: recomputes the winner, writes the inlier mask, F and count.
// Every float expression follows oracle/sfm_oracle.c op for op (explicit fmaf, -ffp-contract=off),
// so inlier sets are bit-identical to the CPU path at a fixed seed.
#include <algorithm>
#include <climits>

#include "sfm_internal.h"

namespace {

__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__device__ __forceinline__ void sample8(uint64_t seed, uint32_t pa, uint32_t pb, uint32_t h, int M,
                                        int idx[8]) {
    uint32_t r[8];
    philox4x32_10(h, 0u, pa, pb, (uint32_t)seed, (uint32_t)(seed >> 32), r);
    philox4x32_10(h, 1u, pa, pb, (uint32_t)seed, (uint32_t)(seed >> 32), r + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t jmax = (uint32_t)(M - 8 + k);
        uint32_t t = __umulhi(r[k], jmax + 1u);
        bool dup = false;
#pragma unroll
        for (int q = 0; q < k; ++q) dup = dup || ((uint32_t)idx[q] == t);
        idx[k] = (int)(dup ? jmax : t);
    }
}

// Mirrors oracle_fit_f8.  Returns false if degenerate.  V[k][r] (r > k) lives in Mt[r][k].
__device__ __forceinline__ bool fit_f8(const float4 s[8], float F[9]) {
    float Mt[9][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float x1 = s[k].x, y1 = s[k].y, x2 = s[k].z, y2 = s[k].w;
        Mt[0][k] = x2 * x1; Mt[1][k] = x2 * y1; Mt[2][k] = x2;
        Mt[3][k] = y2 * x1; Mt[4][k] = y2 * y1; Mt[5][k] = y2;
        Mt[6][k] = x1;      Mt[7][k] = y1;      Mt[8][k] = 1.0f;
    }
    float vkk[8], beta[8];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float nrm2 = 0.0f;
#pragma unroll
        for (int r = k; r < 9; ++r) nrm2 = fmaf(Mt[r][k], Mt[r][k], nrm2);
        ok = ok && (nrm2 > 0.0f);
        const float nrm = sqrtf(nrm2);
        const float alpha = (Mt[k][k] > 0.0f) ? -nrm : nrm;
        vkk[k] = Mt[k][k] - alpha;
        float vn2 = fmaf(vkk[k], vkk[k], 0.0f);
#pragma unroll
        for (int r = k + 1; r < 9; ++r) vn2 = fmaf(Mt[r][k], Mt[r][k], vn2);
        ok = ok && (vn2 > 0.0f);
        beta[k] = 2.0f / vn2;
        Mt[k][k] = alpha;
#pragma unroll
        for (int c = k + 1; c < 8; ++c) {
            float dot = fmaf(vkk[k], Mt[k][c], 0.0f);
#pragma unroll
            for (int r = k + 1; r < 9; ++r) dot = fmaf(Mt[r][k], Mt[r][c], dot);
            const float f = beta[k] * dot;
            Mt[k][c] = fmaf(-f, vkk[k], Mt[k][c]);
#pragma unroll
            for (int r = k + 1; r < 9; ++r) Mt[r][c] = fmaf(-f, Mt[r][k], Mt[r][c]);
        }
    }
    float z[9] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f};
#pragma unroll
    for (int k = 7; k >= 0; --k) {
        float dot = fmaf(vkk[k], z[k], 0.0f);
#pragma unroll
        for (int r = k + 1; r < 9; ++r) dot = fmaf(Mt[r][k], z[r], dot);
        const float f = beta[k] * dot;
        z[k] = fmaf(-f, vkk[k], z[k]);
#pragma unroll
        for (int r = k + 1; r < 9; ++r) z[r] = fmaf(-f, Mt[r][k], z[r]);
    }
    float G[3][3], E[3][3] = {{1.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f}, {0.0f, 0.0f, 1.0f}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float g = 0.0f;
#pragma unroll
            for (int r = 0; r < 3; ++r) g = fmaf(z[3 * r + i], z[3 * r + j], g);
            G[i][j] = g;
        }
#pragma unroll
    for (int sweep = 0; sweep < 5; ++sweep) {
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            const int p = (e == 2) ? 1 : 0, q = (e == 0) ? 1 : 2;
            const float gpq = G[p][q];
            const bool rot = (gpq != 0.0f);
            const float theta = (G[q][q] - G[p][p]) / (2.0f * gpq);
            const float at = fabsf(theta);
            float t = 1.0f / (at + sqrtf(fmaf(theta, theta, 1.0f)));
            if (theta < 0.0f) t = -t;
            const float c = 1.0f / sqrtf(fmaf(t, t, 1.0f));
            const float sn = t * c;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const float gp = G[r][p], gq = G[r][q];
                G[r][p] = rot ? c * gp - sn * gq : gp;
                G[r][q] = rot ? fmaf(sn, gp, c * gq) : gq;
            }
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const float gp = G[p][r], gq = G[q][r];
                G[p][r] = rot ? c * gp - sn * gq : gp;
                G[q][r] = rot ? fmaf(sn, gp, c * gq) : gq;
            }
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const float ep = E[r][p], eq = E[r][q];
                E[r][p] = rot ? c * ep - sn * eq : ep;
                E[r][q] = rot ? fmaf(sn, ep, c * eq) : eq;
            }
        }
    }
    int kmin = 0;
    float gmin = G[0][0];
    if (G[1][1] < gmin) { kmin = 1; gmin = G[1][1]; }
    if (G[2][2] < gmin) { kmin = 2; }
    const float v0 = kmin == 0 ? E[0][0] : (kmin == 1 ? E[0][1] : E[0][2]);
    const float v1 = kmin == 0 ? E[1][0] : (kmin == 1 ? E[1][1] : E[1][2]);
    const float v2 = kmin == 0 ? E[2][0] : (kmin == 1 ? E[2][1] : E[2][2]);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float w = fmaf(z[3 * r + 2], v2, fmaf(z[3 * r + 1], v1, z[3 * r] * v0));
        F[3 * r + 0] = fmaf(-w, v0, z[3 * r + 0]);
        F[3 * r + 1] = fmaf(-w, v1, z[3 * r + 1]);
        F[3 * r + 2] = fmaf(-w, v2, z[3 * r + 2]);
    }
    return ok;
}

// Sampson inlier test (oracle/sfm_oracle.c sampson_inlier): e = t2*g1 + t1*g2 - r^2 > 0.
__device__ __forceinline__ int sampson_inlier(const float F[9], float x1, float y1, float x2,
                                              float y2, float t1, float t2) {
    const float a0 = fmaf(F[0], x1, fmaf(F[1], y1, F[2]));
    const float a1 = fmaf(F[3], x1, fmaf(F[4], y1, F[5]));
    const float a2 = fmaf(F[6], x1, fmaf(F[7], y1, F[8]));
    const float b0 = fmaf(F[0], x2, fmaf(F[3], y2, F[6]));
    const float b1 = fmaf(F[1], x2, fmaf(F[4], y2, F[7]));
    const float r = fmaf(x2, a0, fmaf(y2, a1, a2));
    const float g1 = fmaf(a0, a0, a1 * a1);
    const float g2 = fmaf(b0, b0, b1 * b1);
    const float den = fmaf(t2, g1, t1 * g2);
    const float e = fmaf(-r, r, den);
    return e > 0.0f ? 1 : 0;
}

// The same test on two matches at once: every op is a v_pk_fma_f32 / v_pk_mul_f32 (gfx950 issues
// one packed op per 4 cycles like a scalar one, so this halves the scoring cost).  Each half is an
// IEEE fma/mul exactly like the scalar form, so results are bit-identical.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 sp(float x) { return f2{x, x}; }
__device__ __forceinline__ int sampson_inlier2(const float F[9], f2 x1, f2 y1, f2 x2, f2 y2,
                                               float t1, float t2) {
    const f2 a0 = fma2(sp(F[0]), x1, fma2(sp(F[1]), y1, sp(F[2])));
    const f2 a1 = fma2(sp(F[3]), x1, fma2(sp(F[4]), y1, sp(F[5])));
    const f2 a2 = fma2(sp(F[6]), x1, fma2(sp(F[7]), y1, sp(F[8])));
    const f2 b0 = fma2(sp(F[0]), x2, fma2(sp(F[3]), y2, sp(F[6])));
    const f2 b1 = fma2(sp(F[1]), x2, fma2(sp(F[4]), y2, sp(F[7])));
    const f2 r = fma2(x2, a0, fma2(y2, a1, a2));
    const f2 g1 = fma2(a0, a0, a1 * a1);
    const f2 g2 = fma2(b0, b0, b1 * b1);
    const f2 den = fma2(sp(t2), g1, sp(t1) * g2);
    const f2 e = fma2(-r, r, den);
    return (e.x > 0.0f ? 1 : 0) + (e.y > 0.0f ? 1 : 0);
}

// fixed-order sum: lane l accumulates m = l, l+64, ... then a halving tree (oracle fixed_sum)
__device__ __forceinline__ float wave_fixed_sum(float partial) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) partial = partial + __shfl_down(partial, off, 64);
    return __shfl(partial, 0, 64);
}

__global__ __launch_bounds__(64) void ransac_prep_kernel(
    const float* __restrict__ kps, int k_max, const int32_t* __restrict__ pairs,
    const int32_t* __restrict__ match_count, const int32_t* __restrict__ matches,
    float* __restrict__ nrm_xy, float* __restrict__ out_norm) {
    const int p = blockIdx.x, l = threadIdx.x;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int M = match_count[p];
    const int32_t* mt = matches + (size_t)p * k_max * 2;
    // SoA planes x1 | y1 | x2 | y2, k_max floats each
    float* X1 = nrm_xy + (size_t)p * 4 * k_max;
    float* Y1 = X1 + k_max;
    float* X2 = Y1 + k_max;
    float* Y2 = X2 + k_max;
    if (M < 8) {
        if (l < 6) out_norm[p * 6 + l] = 0.0f;
        return;
    }
    float sx1 = 0.f, sy1 = 0.f, sx2 = 0.f, sy2 = 0.f;
    for (int m = l; m < M; m += 64) {
        const float2 u = *(const float2*)(kps + ((size_t)a * k_max + mt[2 * m]) * 2);
        const float2 v = *(const float2*)(kps + ((size_t)b * k_max + mt[2 * m + 1]) * 2);
        sx1 = sx1 + u.x; sy1 = sy1 + u.y; sx2 = sx2 + v.x; sy2 = sy2 + v.y;
        X1[m] = u.x; Y1[m] = u.y; X2[m] = v.x; Y2[m] = v.y;
    }
    const float fM = (float)M;
    const float mx1 = wave_fixed_sum(sx1) / fM, my1 = wave_fixed_sum(sy1) / fM;
    const float mx2 = wave_fixed_sum(sx2) / fM, my2 = wave_fixed_sum(sy2) / fM;
    float sd1 = 0.f, sd2 = 0.f;
    for (int m = l; m < M; m += 64) {
        const float4 w = make_float4(X1[m], Y1[m], X2[m], Y2[m]);
        float dx = w.x - mx1, dy = w.y - my1;
        float q = dx * dx;
        q = fmaf(dy, dy, q);
        sd1 = sd1 + sqrtf(q);
        dx = w.z - mx2; dy = w.w - my2;
        q = dx * dx;
        q = fmaf(dy, dy, q);
        sd2 = sd2 + sqrtf(q);
    }
    const float mean1 = wave_fixed_sum(sd1) / fM, mean2 = wave_fixed_sum(sd2) / fM;
    const float s1 = (mean1 > 0.0f) ? (1.41421356237309515f / mean1) : 1.0f;
    const float s2 = (mean2 > 0.0f) ? (1.41421356237309515f / mean2) : 1.0f;
    for (int m = l; m < M; m += 64) {
        X1[m] = (X1[m] - mx1) * s1;
        Y1[m] = (Y1[m] - my1) * s1;
        X2[m] = (X2[m] - mx2) * s2;
        Y2[m] = (Y2[m] - my2) * s2;
    }
    if (l == 0) {
        float* o = out_norm + p * 6;
        o[0] = mx1; o[1] = my1; o[2] = s1; o[3] = mx2; o[4] = my2; o[5] = s2;
    }
}

__global__ __launch_bounds__(256) void ransac_hyp_kernel(
    int k_max, const int32_t* __restrict__ pairs, const int32_t* __restrict__ match_count,
    const float* __restrict__ nrm_xy, const float* __restrict__ norm, uint64_t seed, float thr,
    unsigned long long* __restrict__ best) {
    // LDS: the pair's normalised matches as SoA planes x1 | y1 | x2 | y2 (k2 floats each), so a
    // float2 read hands the packed Sampson test two matches in adjacent registers
    extern __shared__ __attribute__((aligned(16))) float lds_m[];
    __shared__ unsigned long long wbest[4];
    const int p = blockIdx.y;
    const int M = match_count[p];
    if (M < 8) return;  // block-uniform
    const int tid = threadIdx.x;
    const int k2 = (k_max + 3) & ~3;
    float* LX1 = lds_m;
    float* LY1 = LX1 + k2;
    float* LX2 = LY1 + k2;
    float* LY2 = LX2 + k2;
    const float* src = nrm_xy + (size_t)p * 4 * k_max;
    for (int m = tid; m < M; m += 256) {
        LX1[m] = src[m];
        LY1[m] = src[k_max + m];
        LX2[m] = src[2 * k_max + m];
        LY2[m] = src[3 * k_max + m];
    }
    __syncthreads();
    const uint32_t pa = (uint32_t)pairs[2 * p], pb = (uint32_t)pairs[2 * p + 1];
    const float s1 = norm[p * 6 + 2], s2 = norm[p * 6 + 5];
    const float t1 = thr * (s1 * s1), t2 = thr * (s2 * s2);
    const uint32_t h = blockIdx.x * 256 + tid;
    int idx[8];
    sample8(seed, pa, pb, h, M, idx);
    float4 smp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        smp[k] = make_float4(LX1[idx[k]], LY1[idx[k]], LX2[idx[k]], LY2[idx[k]]);
    float F[9];
    const bool ok = fit_f8(smp, F);
    // two packed chains (4 matches) per iteration; the count is an integer, so the order of the
    // partial sums does not change the result
    const f2* PX1 = (const f2*)LX1;
    const f2* PY1 = (const f2*)LY1;
    const f2* PX2 = (const f2*)LX2;
    const f2* PY2 = (const f2*)LY2;
    int c0 = 0, c1 = 0;
    int q = 0;
    const int half = M >> 1;
    for (; q + 2 <= half; q += 2) {
        c0 += sampson_inlier2(F, PX1[q], PY1[q], PX2[q], PY2[q], t1, t2);
        c1 += sampson_inlier2(F, PX1[q + 1], PY1[q + 1], PX2[q + 1], PY2[q + 1], t1, t2);
    }
    if (q < half) c0 += sampson_inlier2(F, PX1[q], PY1[q], PX2[q], PY2[q], t1, t2);
    if (M & 1) c1 += sampson_inlier(F, LX1[M - 1], LY1[M - 1], LX2[M - 1], LY2[M - 1], t1, t2);
    int cnt = c0 + c1;
    if (!ok) cnt = -1;
    unsigned long long key = ((unsigned long long)(unsigned)(cnt + 1) << 32) | (0xFFFFFFFFu - h);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = o > key ? o : key;
    }
    if ((tid & 63) == 0) wbest[tid >> 6] = key;
    __syncthreads();
    if (tid == 0) {
        unsigned long long k = wbest[0];
        for (int w = 1; w < 4; ++w) k = wbest[w] > k ? wbest[w] : k;
        atomicMax(&best[p], k);
    }
}

__global__ __launch_bounds__(256) void ransac_final_kernel(
    int k_max, const int32_t* __restrict__ pairs, const int32_t* __restrict__ match_count,
    const float* __restrict__ nrm_xy, const float* __restrict__ norm, uint64_t seed, float thr,
    const unsigned long long* __restrict__ best, int32_t* __restrict__ out_inl_count,
    int32_t* __restrict__ out_best_h, uint8_t* __restrict__ out_mask, float* __restrict__ out_F) {
    __shared__ int wsum[4];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int M = match_count[p];
    uint8_t* mask = out_mask + (size_t)p * k_max;
    if (M < 8) {
        for (int m = tid; m < M; m += 256) mask[m] = 0;
        if (tid < 9) out_F[p * 9 + tid] = 0.0f;
        if (tid == 0) { out_inl_count[p] = -1; out_best_h[p] = -1; }
        return;
    }
    const uint32_t pa = (uint32_t)pairs[2 * p], pb = (uint32_t)pairs[2 * p + 1];
    const uint32_t h = 0xFFFFFFFFu - (uint32_t)best[p];
    const float* X1 = nrm_xy + (size_t)p * 4 * k_max;
    const float* Y1 = X1 + k_max;
    const float* X2 = Y1 + k_max;
    const float* Y2 = X2 + k_max;
    const float s1 = norm[p * 6 + 2], s2 = norm[p * 6 + 5];
    const float t1 = thr * (s1 * s1), t2 = thr * (s2 * s2);
    int idx[8];
    sample8(seed, pa, pb, h, M, idx);
    float4 smp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) smp[k] = make_float4(X1[idx[k]], Y1[idx[k]], X2[idx[k]], Y2[idx[k]]);
    float F[9];
    const bool ok = fit_f8(smp, F);
    int cnt = 0;
    for (int m = tid; m < M; m += 256) {
        const int in = ok ? sampson_inlier(F, X1[m], Y1[m], X2[m], Y2[m], t1, t2) : 0;
        mask[m] = (uint8_t)in;
        cnt += in;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if ((tid & 63) == 0) wsum[tid >> 6] = cnt;
    __syncthreads();
    if (tid == 0) {
        out_inl_count[p] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        out_best_h[p] = (int)h;
    }
    if (tid < 9) out_F[p * 9 + tid] = ok ? F[tid] : 0.0f;
}

}  // namespace

extern "C" int sfm_ransac_f_batch(sfm_ctx* ctx, const float* kps, int32_t n_img, int32_t k_max,
                                  const int32_t* pairs, int32_t n_pairs,
                                  const int32_t* match_count, const int32_t* matches,
                                  const sfm_ransac_params* prm, int32_t* out_inl_count,
                                  int32_t* out_best_h, uint8_t* out_mask, float* out_F,
                                  float* out_norm) {
    SFM_REQUIRE(ctx && prm, "sfm_ransac_f_batch: ctx/prm is NULL");
    SFM_REQUIRE(n_pairs >= 0 && n_img >= 0 && k_max >= 0, "sfm_ransac_f_batch: negative size");
    if (n_pairs == 0) return SFM_OK;
    SFM_REQUIRE(kps && pairs && match_count && matches && out_inl_count && out_best_h &&
                    out_mask && out_F && out_norm,
                "sfm_ransac_f_batch: NULL array");
    SFM_REQUIRE(prm->n_hyp > 0 && prm->n_hyp % 256 == 0,
                "sfm_ransac_f_batch: n_hyp must be a positive multiple of 256");
    SFM_REQUIRE(k_max <= 8192, "sfm_ransac_f_batch: k_max > 8192 not supported");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const size_t xyb = (size_t)n_pairs * 4 * std::max(k_max, 1) * sizeof(float);
    const size_t bb = (size_t)n_pairs * sizeof(unsigned long long);
    char* ws = (char*)sfm::workspace(ctx, xyb + bb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    float* nrm_xy = (float*)ws;
    unsigned long long* best = (unsigned long long*)(ws + xyb);
    SFM_HIP_CHECK(hipMemsetAsync(best, 0, bb, st));
    hipLaunchKernelGGL(ransac_prep_kernel, dim3(n_pairs), dim3(64), 0, st, kps, k_max, pairs,
                       match_count, matches, nrm_xy, out_norm);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ransac_hyp_kernel, dim3(prm->n_hyp / 256, n_pairs), dim3(256),
                       (size_t)4 * ((std::max(k_max, 1) + 3) & ~3) * sizeof(float), st, k_max, pairs,
                       match_count,
                       nrm_xy, out_norm, prm->seed, prm->thr, best);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ransac_final_kernel, dim3(n_pairs), dim3(256), 0, st, k_max, pairs,
                       match_count, nrm_xy, out_norm, prm->seed, prm->thr, best, out_inl_count,
                       out_best_h, out_mask, out_F);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
