// 8-point fundamental-matrix RANSAC (K2).
//
// Fills the empty reference module code/geometric_verification.py (placeholder at
// code/pipeline.py:60).  Default schedule (SFM_RANSAC_MODE 0, "ordered"; described above
// ransac_fit_kernel): ransac_prep -> ransac_fit (sample, fit, 64-match preview, one 48-byte record
// per hypothesis) -> ransac_order (per-pair sort by preview) -> ransac_score (pruned scoring in
// preview order; an XCD's pairs in groups, hb-major inside a group, xcd_pair_block) ->
// ransac_final.  The single-pass schedules (modes 1, 2) use three kernels per batch of pairs:
//   ransac_prep   one wave per pair: gathers the tentative-match pixel coordinates, Hartley-
//                 normalises each side with a fixed-order wave reduction and writes 8 planes per
//                 pair: the normalised x1|y1|x2|y2 (fits) and the Sampson-scaled X1|Y1|X2|Y2
//                 (scoring, X = k * x_normalised, k = 1/(s*sqrt(thr))), plus (cx,cy,s) per side.
//   ransac_hyp    one LANE per hypothesis (256 per block): counter-based Philox sample of 8 distinct
//                 matches (Floyd), Householder-QR null space of the 8x9 epipolar system, rank-2
//                 projection (squarings of adj(F^T F)), then a sweep over all M matches counting
//                 Sampson inliers (17 flops + compare per match).  The match coordinates are
//                 wave-uniform, so they are read with scalar loads into SGPRs and fed to packed
//                 FMAs as SGPR-pair operands.  Exact pruning: every 64 matches a wave reads
//                 the pair's best count so far (published by finished waves) and stops when no lane
//                 can still reach it (count + remaining < best: strictly cannot win, so the result
//                 is unchanged).  Each wave publishes its argmax (max count, lowest h) with one
//                 64-bit atomicMax.  Grid x = pair, so the first hypothesis block of every pair runs
//                 first and later blocks start with a bound.
//   ransac_final  one block per pair: recomputes the winner, writes the inlier mask, F and count.
// Every float expression follows oracle/sfm_oracle.c op for op (explicit fmaf, -ffp-contract=off),
// so inlier sets are bit-identical to the CPU path at a fixed seed.
#include <algorithm>
#include <climits>

#include "sfm_internal.h"

namespace {

constexpr int RANK2_SQUARINGS = 8;  // oracle_fit_f8 (round 3; was 4 power iterations)

__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of mul_hi + mul_lo
        const uint64_t m0 = (uint64_t)0xD2511F53u * c0, m1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(m0 >> 32), lo0 = (uint32_t)m0;
        const uint32_t hi1 = (uint32_t)(m1 >> 32), lo1 = (uint32_t)m1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Scalar-type helpers: the f32 spec (default) and its fp64 mode (sfm_ransac_f_batch_f64) run the
// same op sequence; these pick the fmaf / fma families (oracle/sfm_oracle_ransac.inc).
__device__ __forceinline__ float fmaT(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fmaT(double a, double b, double c) { return fma(a, b, c); }
__device__ __forceinline__ float sqrtT(float a) { return sqrtf(a); }
__device__ __forceinline__ double sqrtT(double a) { return sqrt(a); }
__device__ __forceinline__ float fabsT(float a) { return fabsf(a); }
__device__ __forceinline__ double fabsT(double a) { return fabs(a); }
__device__ __forceinline__ float fmaxT(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ double fmaxT(double a, double b) { return fmax(a, b); }
__device__ __forceinline__ float frexpT(float a, int* e) { return frexpf(a, e); }
__device__ __forceinline__ double frexpT(double a, int* e) { return frexp(a, e); }
__device__ __forceinline__ float ldexpT(float a, int e) { return ldexpf(a, e); }
__device__ __forceinline__ double ldexpT(double a, int e) { return ldexp(a, e); }
template <typename T> struct V4 { T x, y, z, w; };
template <typename T> struct alignas(2 * sizeof(T)) V2 { T x, y; };
// the preview count rides in a record slot of the scalar type (its bit pattern)
__device__ __forceinline__ float pc_bits(int pc, float) { return __int_as_float(pc); }
__device__ __forceinline__ double pc_bits(int pc, double) { return __longlong_as_double((long long)pc); }
__device__ __forceinline__ int pc_of(float v) { return __float_as_int(v); }
__device__ __forceinline__ int pc_of(double v) { return (int)__double_as_longlong(v); }

// pl[i] through a 32-bit byte offset (the plane block of a pair is < 4 GB): the load takes the
// pair's uniform base in SGPRs and no per-lane 64-bit address arithmetic
template <typename T>
__device__ __forceinline__ T ldT(const T* __restrict__ pl, int i) {
    return *(const T*)((const char*)pl + (uint32_t)i * (uint32_t)sizeof(T));
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
template <typename T>
__device__ __forceinline__ bool fit_f8(const V4<T> s[8], T F[9]) {
    T Mt[9][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const T x1 = s[k].x, y1 = s[k].y, x2 = s[k].z, y2 = s[k].w;
        Mt[0][k] = x2 * x1; Mt[1][k] = x2 * y1; Mt[2][k] = x2;
        Mt[3][k] = y2 * x1; Mt[4][k] = y2 * y1; Mt[5][k] = y2;
        Mt[6][k] = x1;      Mt[7][k] = y1;      Mt[8][k] = T(1.0);
    }
    T vkk[8], beta[8];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        T nrm2 = T(0.0);
#pragma unroll
        for (int r = k; r < 9; ++r) nrm2 = fmaT(Mt[r][k], Mt[r][k], nrm2);
        ok = ok && (nrm2 > T(0.0));
        const T nrm = sqrtT(nrm2);
        const T alpha = (Mt[k][k] > T(0.0)) ? -nrm : nrm;
        vkk[k] = Mt[k][k] - alpha;
        T vn2 = fmaT(vkk[k], vkk[k], T(0.0));
#pragma unroll
        for (int r = k + 1; r < 9; ++r) vn2 = fmaT(Mt[r][k], Mt[r][k], vn2);
        ok = ok && (vn2 > T(0.0));
        beta[k] = T(2.0) / vn2;
        Mt[k][k] = alpha;
#pragma unroll
        for (int c = k + 1; c < 8; ++c) {
            T dot = fmaT(vkk[k], Mt[k][c], T(0.0));
#pragma unroll
            for (int r = k + 1; r < 9; ++r) dot = fmaT(Mt[r][k], Mt[r][c], dot);
            const T f = beta[k] * dot;
            Mt[k][c] = fmaT(-f, vkk[k], Mt[k][c]);
#pragma unroll
            for (int r = k + 1; r < 9; ++r) Mt[r][c] = fmaT(-f, Mt[r][k], Mt[r][c]);
        }
    }
    T z[9] = {T(0.0), T(0.0), T(0.0), T(0.0), T(0.0), T(0.0), T(0.0), T(0.0), T(1.0)};
#pragma unroll
    for (int k = 7; k >= 0; --k) {
        T dot = fmaT(vkk[k], z[k], T(0.0));
#pragma unroll
        for (int r = k + 1; r < 9; ++r) dot = fmaT(Mt[r][k], z[r], dot);
        const T f = beta[k] * dot;
        z[k] = fmaT(-f, vkk[k], z[k]);
#pragma unroll
        for (int r = k + 1; r < 9; ++r) z[r] = fmaT(-f, Mt[r][k], z[r]);
    }
#ifdef RANSAC_ABL_NORANK2  // ablation: no rank-2 step (timing only; results invalid)
#pragma unroll
    for (int i = 0; i < 9; ++i) F[i] = z[i];
    return ok;
#endif
    // rank 2 (oracle_fit_f8): smallest eigen-direction of G = F^T F by power iteration on adj(G)
    T G[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            T g = T(0.0);
#pragma unroll
            for (int r = 0; r < 3; ++r) g = fmaT(z[3 * r + i], z[3 * r + j], g);
            G[i][j] = g;
        }
    T A[3][3];
    A[0][0] = fmaT(G[1][1], G[2][2], -(G[1][2] * G[1][2]));
    A[1][1] = fmaT(G[0][0], G[2][2], -(G[0][2] * G[0][2]));
    A[2][2] = fmaT(G[0][0], G[1][1], -(G[0][1] * G[0][1]));
    A[0][1] = A[1][0] = fmaT(G[0][2], G[1][2], -(G[0][1] * G[2][2]));
    A[0][2] = A[2][0] = fmaT(G[0][1], G[1][2], -(G[0][2] * G[1][1]));
    A[1][2] = A[2][1] = fmaT(G[0][1], G[0][2], -(G[0][0] * G[1][2]));
    // rescaled squarings of adj(G) (oracle square3_sym): the max-diagonal column of
    // adj(G)^(2^RANK2_SQUARINGS) is the removed direction to (s3/s2)^512
    T a00 = A[0][0], a11 = A[1][1], a22 = A[2][2], a01 = A[0][1], a02 = A[0][2], a12 = A[1][2];
#pragma unroll
    for (int it = 0; it < RANK2_SQUARINGS; ++it) {
        const T m = fmaxT(fmaxT(fmaxT(fabsT(a00), fabsT(a11)), fmaxT(fabsT(a22), fabsT(a01))),
                              fmaxT(fabsT(a02), fabsT(a12)));
        if (m > T(0.0) && isfinite(m)) {
            int e;
            frexpT(m, &e);
            a00 = ldexpT(a00, -e); a11 = ldexpT(a11, -e); a22 = ldexpT(a22, -e);
            a01 = ldexpT(a01, -e); a02 = ldexpT(a02, -e); a12 = ldexpT(a12, -e);
        }
        const T b00 = fmaT(a02, a02, fmaT(a01, a01, a00 * a00));
        const T b11 = fmaT(a12, a12, fmaT(a11, a11, a01 * a01));
        const T b22 = fmaT(a22, a22, fmaT(a12, a12, a02 * a02));
        const T b01 = fmaT(a02, a12, fmaT(a01, a11, a00 * a01));
        const T b02 = fmaT(a02, a22, fmaT(a01, a12, a00 * a02));
        const T b12 = fmaT(a12, a22, fmaT(a11, a12, a01 * a02));
        a00 = b00; a11 = b11; a22 = b22; a01 = b01; a02 = b02; a12 = b12;
    }
    int kk = 0;
    T amax = a00;
    if (a11 > amax) { kk = 1; amax = a11; }
    if (a22 > amax) kk = 2;
    T v0 = kk == 0 ? a00 : (kk == 1 ? a01 : a02);
    T v1 = kk == 0 ? a01 : (kk == 1 ? a11 : a12);
    T v2 = kk == 0 ? a02 : (kk == 1 ? a12 : a22);
    {   // exact power-of-two rescale by the exponent of max|v| (oracle rescale3_pow2)
        const T m = fmaxT(fabsT(v0), fmaxT(fabsT(v1), fabsT(v2)));
        if (m > T(0.0) && isfinite(m)) {
            int e;
            frexpT(m, &e);
            v0 = ldexpT(v0, -e); v1 = ldexpT(v1, -e); v2 = ldexpT(v2, -e);
        }
    }
    const T n2 = fmaT(v2, v2, fmaT(v1, v1, v0 * v0));
    if (n2 > T(0.0)) {
        const T inv = T(1.0) / sqrtT(n2);
        v0 = v0 * inv; v1 = v1 * inv; v2 = v2 * inv;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const T w = fmaT(z[3 * r + 2], v2, fmaT(z[3 * r + 1], v1, z[3 * r] * v0));
            F[3 * r + 0] = fmaT(-w, v0, z[3 * r + 0]);
            F[3 * r + 1] = fmaT(-w, v1, z[3 * r + 1]);
            F[3 * r + 2] = fmaT(-w, v2, z[3 * r + 2]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) F[i] = z[i];
    }
    return ok;
}

// Sampson inlier test, oracle/sfm_oracle.c sampson_prep / sampson_inlier: G = F with the
// homogeneous scales folded in, coordinates pre-scaled; inlier iff |a|^2 + |b|^2 - r^2 > 0.
template <typename T>
__device__ __forceinline__ void sampson_prep(const T F[9], T k1, T k2, T G[9]) {
#pragma unroll
    for (int i = 0; i < 9; ++i) G[i] = F[i];
    G[2] = F[2] * k1;
    G[5] = F[5] * k1;
    G[6] = F[6] * k2;
    G[7] = F[7] * k2;
    G[8] = (F[8] * k1) * k2;
}

template <typename T>
__device__ __forceinline__ int sampson_inlier(const T G[9], T x1, T y1, T x2, T y2) {
    const T a0 = fmaT(G[0], x1, fmaT(G[1], y1, G[2]));
    const T a1 = fmaT(G[3], x1, fmaT(G[4], y1, G[5]));
    const T c2 = fmaT(G[6], x1, fmaT(G[7], y1, G[8]));
    const T b0 = fmaT(G[0], x2, fmaT(G[3], y2, G[6]));
    const T b1 = fmaT(G[1], x2, fmaT(G[4], y2, G[7]));
    const T r = fmaT(x2, a0, fmaT(y2, a1, c2));
    const T den = fmaT(a0, a0, fmaT(a1, a1, fmaT(b0, b0, b1 * b1)));
    const T e = fmaT(-r, r, den);
    return e > T(0.0) ? 1 : 0;
}

// per-pair scales of the scoring coordinates (oracle sampson_scales)
template <typename T>
__device__ __forceinline__ void sampson_scales(T s1, T s2, T thr, T& k1, T& k2) {
    const T rt = sqrtT(thr);
    k1 = T(1.0) / (s1 * rt);
    k2 = T(1.0) / (s2 * rt);
}

// fixed-order sum: lane l accumulates m = l, l+64, ... then a halving tree (oracle fixed_sum)
template <typename T>
__device__ __forceinline__ T wave_fixed_sum(T partial) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) partial = partial + __shfl_down(partial, off, 64);
    return __shfl(partial, 0, 64);
}

// plane stride per pair: 8 planes of k_pl floats (k_pl multiple of 16: 64-B aligned planes)
__host__ __device__ __forceinline__ int plane_len(int k_max) { return (k_max + 15) & ~15; }

// One 256-thread block per pair.  The four waves share the dependent gathers (match index ->
// keypoint) and the final scaling; wave 0 alone forms the sums, lane l accumulating m = l, l+64,
// ... in order then the halving tree (the oracle's fixed_sum), so the bits do not depend on the
// block width.  (One wave per pair spent its life on the gather chain: 28 us at cfg3.)
constexpr int PREP_T = 256;
template <typename T>
__global__ __launch_bounds__(PREP_T) void ransac_prep_kernel(
    const T* __restrict__ kps, int k_max, const int32_t* __restrict__ pairs,
    const int32_t* __restrict__ match_count, const int32_t* __restrict__ matches, T thr,
    T* __restrict__ planes, T* __restrict__ out_norm) {
    __shared__ T par[8];  // mx1, my1, s1, mx2, my2, s2, k1, k2
    const int p = blockIdx.x, tid = threadIdx.x, l = tid & 63;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int M = match_count[p];
    const int32_t* mt = matches + (size_t)p * k_max * 2;
    const int kp = plane_len(k_max);
    T* X1 = planes + (size_t)p * 8 * kp;  // normalised x1 | y1 | x2 | y2
    T* Y1 = X1 + kp;
    T* X2 = Y1 + kp;
    T* Y2 = X2 + kp;
    T* S = Y2 + kp;                        // scaled X1 | Y1 | X2 | Y2
    if (M < 8) {
        if (tid < 6) out_norm[p * 6 + tid] = T(0.0);
        return;
    }
    // gathers: four matches per thread in flight, raw coordinates to the planes
    for (int m0 = tid; m0 < M; m0 += 4 * PREP_T) {
        int2 id[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int m = m0 + PREP_T * t;
            id[t] = m < M ? *(const int2*)(mt + 2 * m) : make_int2(0, 0);
        }
        V2<T> u[4], v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            u[t] = *(const V2<T>*)(kps + ((size_t)a * k_max + id[t].x) * 2);
            v[t] = *(const V2<T>*)(kps + ((size_t)b * k_max + id[t].y) * 2);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int m = m0 + PREP_T * t;
            if (m < M) { X1[m] = u[t].x; Y1[m] = u[t].y; X2[m] = v[t].x; Y2[m] = v[t].y; }
        }
    }
    __syncthreads();  // the raw planes are visible to the block
    if (tid < 64) {
        T sx1 = 0.f, sy1 = 0.f, sx2 = 0.f, sy2 = 0.f;
#pragma unroll 4
        for (int m = l; m < M; m += 64) {
            sx1 = sx1 + X1[m]; sy1 = sy1 + Y1[m]; sx2 = sx2 + X2[m]; sy2 = sy2 + Y2[m];
        }
        const T fM = (T)M;
        const T mx1 = wave_fixed_sum(sx1) / fM, my1 = wave_fixed_sum(sy1) / fM;
        const T mx2 = wave_fixed_sum(sx2) / fM, my2 = wave_fixed_sum(sy2) / fM;
        T sd1 = 0.f, sd2 = 0.f;
#pragma unroll 4
        for (int m = l; m < M; m += 64) {
            const V4<T> w = {X1[m], Y1[m], X2[m], Y2[m]};
            T dx = w.x - mx1, dy = w.y - my1;
            T q = dx * dx;
            q = fmaT(dy, dy, q);
            sd1 = sd1 + sqrtT(q);
            dx = w.z - mx2; dy = w.w - my2;
            q = dx * dx;
            q = fmaT(dy, dy, q);
            sd2 = sd2 + sqrtT(q);
        }
        const T mean1 = wave_fixed_sum(sd1) / fM, mean2 = wave_fixed_sum(sd2) / fM;
        const T s1 = (mean1 > T(0.0)) ? (T(1.41421356237309515) / mean1) : T(1.0);
        const T s2 = (mean2 > T(0.0)) ? (T(1.41421356237309515) / mean2) : T(1.0);
        T k1, k2;
        sampson_scales(s1, s2, thr, k1, k2);
        if (l == 0) {
            par[0] = mx1; par[1] = my1; par[2] = s1; par[3] = mx2; par[4] = my2; par[5] = s2;
            par[6] = k1; par[7] = k2;
            T* o = out_norm + p * 6;
            o[0] = mx1; o[1] = my1; o[2] = s1; o[3] = mx2; o[4] = my2; o[5] = s2;
        }
    }
    __syncthreads();
    const T mx1 = par[0], my1 = par[1], s1 = par[2], mx2 = par[3], my2 = par[4], s2 = par[5];
    const T k1 = par[6], k2 = par[7];
#pragma unroll 4
    for (int m = tid; m < M; m += PREP_T) {
        const T x1 = (X1[m] - mx1) * s1, y1 = (Y1[m] - my1) * s1;
        const T x2 = (X2[m] - mx2) * s2, y2 = (Y2[m] - my2) * s2;
        X1[m] = x1; Y1[m] = y1; X2[m] = x2; Y2[m] = y2;
        S[m] = x1 * k1;
        S[kp + m] = y1 * k1;
        S[2 * kp + m] = x2 * k2;
        S[3 * kp + m] = y2 * k2;
    }
}

typedef const __attribute__((address_space(4))) float* cfloat_p;  // scalar (constant) loads
typedef const __attribute__((address_space(4))) double* cdouble_p;
template <typename T> struct CPtr { typedef cfloat_p type; };
template <> struct CPtr<double> { typedef cdouble_p type; };

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 sp(float x) { return f2{x, x}; }
// two matches per call with v_pk_fma_f32 / v_pk_mul_f32; each half is the scalar op sequence
__device__ __forceinline__ int sampson_inlier2(const float G[9], f2 x1, f2 y1, f2 x2, f2 y2) {
    const f2 a0 = fma2(sp(G[0]), x1, fma2(sp(G[1]), y1, sp(G[2])));
    const f2 a1 = fma2(sp(G[3]), x1, fma2(sp(G[4]), y1, sp(G[5])));
    const f2 c2 = fma2(sp(G[6]), x1, fma2(sp(G[7]), y1, sp(G[8])));
    const f2 b0 = fma2(sp(G[0]), x2, fma2(sp(G[3]), y2, sp(G[6])));
    const f2 b1 = fma2(sp(G[1]), x2, fma2(sp(G[4]), y2, sp(G[7])));
    const f2 r = fma2(x2, a0, fma2(y2, a1, c2));
    const f2 den = fma2(a0, a0, fma2(a1, a1, fma2(b0, b0, b1 * b1)));
    const f2 e = fma2(-r, r, den);
    return (e.x > 0.0f ? 1 : 0) + (e.y > 0.0f ? 1 : 0);
}

// XCD-aware block mapping of the [pair][hypothesis block] grids (fit, score).  Workgroups are
// dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), each XCD with its own 4 MB L2:
// XCD x gets the contiguous pair range [x*Q, (x+1)*Q) and walks it hypothesis-block-major, so a
// pair's scoring planes are read through ONE L2 (with grid (P, H/256) and P = 1 mod 8, as at
// cfg3, every pair's 16 blocks landed on all 8 XCDs) and every pair's first (best-previewed)
// block still runs before any second block.  Returns false for the padding blocks.
__device__ __forceinline__ bool xcd_pair_block(int n_pairs, int n_hb, int gp, int& p, int& hb) {
    const int Q = (n_pairs + 7) >> 3;
    const int x = (int)(blockIdx.x & 7), j = (int)(blockIdx.x >> 3);
    // the XCD's pairs in groups of gp, hb-major inside a group: the best-previewed block of a pair
    // still runs first, and the group's match planes stay in the XCD's L2 while its blocks run
    const int g = j / (gp * n_hb), r = j - g * gp * n_hb;
    const int gsz = min(gp, Q - g * gp);
    hb = r / gsz;
    p = x * Q + g * gp + (r - hb * gsz);
    return p < n_pairs;
}
static inline unsigned xcd_grid(int n_pairs, int n_hb) { return 8u * (unsigned)((n_pairs + 7) >> 3) * (unsigned)n_hb; }

constexpr int CH = 16;         // matches per scalar-load chunk (4 x s_load_dwordx16)
#ifndef RANSAC_PRUNE_EVERY
#define RANSAC_PRUNE_EVERY 32  // K2 at cfg4 vs 32: 16 and 64 +0.8 %, 128 +2.5 % (ransac_prune_every_ab.txt)
#endif
constexpr int PRUNE_EVERY = RANSAC_PRUNE_EVERY;  // matches between bound checks (multiple of CH)
static_assert(PRUNE_EVERY % CH == 0, "prune period");

// One lane = one hypothesis; see the file comment.  The scoring coordinates are wave-uniform, so
// they come through the scalar cache into SGPRs (no LDS traffic; the packed FMAs take them as
// SGPR-pair operands).  Measured on cfg3 (tools/ransac_variants.py): LDS broadcast source
// 1.93 ms, SGPR source 1.86 ms, SGPR + pruning 1.45 ms per 1225-pair launch.
template <bool PRUNE>
__global__ __launch_bounds__(256) void ransac_hyp_kernel(
    int k_max, const int32_t* __restrict__ pairs, const int32_t* __restrict__ match_count,
    const float* __restrict__ planes, const float* __restrict__ norm, uint64_t seed, float thr,
    unsigned long long* __restrict__ best) {
    const int p = blockIdx.x;
    const int M = match_count[p];
    if (M < 8) return;  // block-uniform
    const int tid = threadIdx.x;
    const int kp = plane_len(k_max);
    const float* pl = planes + (size_t)p * 8 * kp;
    const cfloat_p S = (cfloat_p)(pl + 4 * kp);
    const uint32_t pa = (uint32_t)pairs[2 * p], pb = (uint32_t)pairs[2 * p + 1];
    const float s1 = norm[p * 6 + 2], s2 = norm[p * 6 + 5];
    float k1, k2;
    sampson_scales(s1, s2, thr, k1, k2);
    const uint32_t h = blockIdx.y * 256 + tid;
    int idx[8];
    sample8(seed, pa, pb, h, M, idx);
    V4<float> smp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        smp[k] = {ldT(pl, idx[k]), ldT(pl, kp + idx[k]), ldT(pl, 2 * kp + idx[k]),
                  ldT(pl, 3 * kp + idx[k])};
    float F[9], G[9];
    const bool ok = fit_f8(smp, F);
    sampson_prep(F, k1, k2, G);

    int cnt = 0;
    const int Mc = M & ~(CH - 1);
    int m = 0;
#pragma unroll 1
    for (; m < Mc; m += CH) {
        float x1[CH], y1[CH], x2[CH], y2[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            x1[j] = S[m + j];
            y1[j] = S[kp + m + j];
            x2[j] = S[2 * kp + m + j];
            y2[j] = S[3 * kp + m + j];
        }
#pragma unroll
        for (int j = 0; j < CH; j += 2)
            cnt += sampson_inlier2(G, f2{x1[j], x1[j + 1]}, f2{y1[j], y1[j + 1]},
                                   f2{x2[j], x2[j + 1]}, f2{y2[j], y2[j + 1]});
        if (PRUNE && ((m + CH) % PRUNE_EVERY) == 0) {
            // Exact pruning: best[p] only grows and every published key is a real hypothesis's
            // (count, id), so (key >> 32) - 1 is a lower bound on the winning count.  A wave
            // whose lanes all satisfy count + remaining < bound holds no possible winner.
            const unsigned long long bk =
                __hip_atomic_load(&best[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int bound = (int)(bk >> 32) - 1;
            if (__all(cnt + (M - m - CH) < bound)) return;  // wave-uniform exit
        }
    }
#pragma unroll 1
    for (; m < M; ++m) cnt += sampson_inlier(G, S[m], S[kp + m], S[2 * kp + m], S[3 * kp + m]);
    if (!ok) cnt = -1;
    unsigned long long key = ((unsigned long long)(unsigned)(cnt + 1) << 32) | (0xFFFFFFFFu - h);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = o > key ? o : key;
    }
    if ((tid & 63) == 0) atomicMax(&best[p], key);  // per wave: later waves prune sooner
}

// ---- ordered variant: fit + preview, per-pair ordering, ordered scoring --------------------------
//
// Exact pruning only removes a wave once every lane is provably beaten, so it pays most when the
// strong hypotheses are scored first and the weak ones end up together in the same waves.
//   ransac_fit_kernel    lane per hypothesis: sample + fit, Sampson count over the first PV matches
//                        (the "preview", same op sequence), G + preview to a [pair][H] record table.
//   ransac_order_kernel  block per pair: counting sort of the hypotheses by preview count,
//                        descending (order within a bucket is irrelevant: the winner key carries h).
//   ransac_score_kernel  rank r of pair p scores hypothesis order[p][r] from match PV on, starting
//                        from its preview count, with the same exact pruning; grid x = pair so the
//                        best-previewed block of every pair runs first and publishes a strong bound.
// PV = 128: interleaved A/B at cfg4 (profiles/r04/ransac_preview_ab_r6i.txt, _r6j.txt): 32 206.5,
// 64 202.2, 96 200.7, 128 199.7 ms; second box 64 207.0-207.6 vs 128-224 a plateau at 204.3-205.2;
// cfg3 within noise, outputs identical.  (hist[PV + 2] in 256 threads: PV <= 240, multiple of 16.)
#ifndef RANSAC_PV
#define RANSAC_PV 128
#endif
constexpr int PV = RANSAC_PV;  // preview matches (multiple of CH and of 8)
constexpr int HREC = 12;  // hypothesis record: G[9], preview count (int bits), 2 pad floats

// counts inliers of G over matches [m, mend) into cnt; with PRUNE checks the published bound every
// PRUNE_EVERY matches and returns false (wave-uniform) when no lane can still win.
// `mstop` (if given) receives the match index where the wave stopped (mend when it finished).
// f32: two matches per packed op (sampson_inlier2); fp64: the scalar test per match.
template <bool PRUNE, int C = CH, typename T = float>
__device__ __forceinline__ bool score_matches(typename CPtr<T>::type S, int kp, const T G[9], int m,
                                              int mend, int M, int& cnt,
                                              const unsigned long long* __restrict__ bestp,
                                              int* mstop = nullptr) {
    const int mc = m + ((mend - m) & ~(C - 1));
#pragma unroll 1
    for (; m < mc; m += C) {
        T x1[C], y1[C], x2[C], y2[C];
#pragma unroll
        for (int j = 0; j < C; ++j) {
            x1[j] = S[m + j];
            y1[j] = S[kp + m + j];
            x2[j] = S[2 * kp + m + j];
            y2[j] = S[3 * kp + m + j];
        }
        if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int j = 0; j < C; j += 2)
                cnt += sampson_inlier2(G, f2{x1[j], x1[j + 1]}, f2{y1[j], y1[j + 1]},
                                       f2{x2[j], x2[j + 1]}, f2{y2[j], y2[j + 1]});
        } else {
#pragma unroll
            for (int j = 0; j < C; ++j) cnt += sampson_inlier(G, x1[j], y1[j], x2[j], y2[j]);
        }
        if (PRUNE && ((m + C) % PRUNE_EVERY) == 0) {
            const unsigned long long bk =
                __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int bound = (int)(bk >> 32) - 1;
            if (__all(cnt + (M - m - C) < bound)) {
                if (mstop) *mstop = m + C;
                return false;
            }
        }
    }
#pragma unroll 1
    for (; m < mend; ++m) cnt += sampson_inlier(G, S[m], S[kp + m], S[2 * kp + m], S[3 * kp + m]);
    if (mstop) *mstop = mend;
    return true;
}

#ifdef RANSAC_FIT_MINW  // build knob: minimum waves per SIMD for the fit kernel (caps its VGPRs)
#define RANSAC_FIT_ATTR __attribute__((amdgpu_waves_per_eu(RANSAC_FIT_MINW, 8)))
#else
#define RANSAC_FIT_ATTR
#endif
template <typename T>
__global__ __launch_bounds__(256) RANSAC_FIT_ATTR void ransac_fit_kernel(
    int n_pairs, int k_max, const int32_t* __restrict__ pairs, const int32_t* __restrict__ match_count,
    const T* __restrict__ planes, const T* __restrict__ norm, uint64_t seed, T thr,
    int n_hyp, int gp, T* __restrict__ hypG, int32_t* __restrict__ prev,
    float* __restrict__ out_hyp_F = nullptr) {
    int p, hb;
    if (!xcd_pair_block(n_pairs, n_hyp >> 8, gp, p, hb)) return;
    const int M = match_count[p];
    if (M < 8) return;  // block-uniform
    const int kp = plane_len(k_max);
    const T* pl = planes + (size_t)p * 8 * kp;
    const typename CPtr<T>::type S = (typename CPtr<T>::type)(pl + 4 * kp);
    const uint32_t pa = (uint32_t)pairs[2 * p], pb = (uint32_t)pairs[2 * p + 1];
    const T s1 = norm[p * 6 + 2], s2 = norm[p * 6 + 5];
    T k1, k2;
    sampson_scales(s1, s2, thr, k1, k2);
    const uint32_t h = hb * 256 + threadIdx.x;
    int idx[8];
#ifdef RANSAC_ABL_NOSAMPLE  // ablation: no Philox / Floyd sampling (timing only; results invalid)
#pragma unroll
    for (int k = 0; k < 8; ++k) idx[k] = (int)((h * 8u + (uint32_t)k) % (uint32_t)M);
#else
    sample8(seed, pa, pb, h, M, idx);
#endif
    V4<T> smp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        smp[k] = {ldT(pl, idx[k]), ldT(pl, kp + idx[k]), ldT(pl, 2 * kp + idx[k]),
                  ldT(pl, 3 * kp + idx[k])};
    T F[9], G[9];
#ifdef RANSAC_ABL_NOFIT  // ablation: no 8-point fit (timing only; results invalid)
    const bool ok = true;
#pragma unroll
    for (int k = 0; k < 9; ++k) F[k] = smp[k & 7].x * (T)(k + 1) + smp[(k + 3) & 7].w;
#else
    const bool ok = fit_f8(smp, F);
#endif
    if (out_hyp_F) {  // diagnostic (sfm_ransac_counts): F of every hypothesis, normalised frame
        float* o = out_hyp_F + ((size_t)p * n_hyp + h) * 9;
#pragma unroll
        for (int k = 0; k < 9; ++k) o[k] = (float)F[k];
    }
    sampson_prep(F, k1, k2, G);
    int cnt = 0;
#ifndef RANSAC_ABL_NOPREVIEW  // ablation: no preview (timing only; order degenerates)
    score_matches<false, 8, T>(S, kp, G, 0, min(PV, M), M, cnt, nullptr);  // 8-match chunks: fewer VGPRs beside the fit
#endif
    const int pc = ok ? cnt : -1;
    V4<T>* rec = (V4<T>*)(hypG + ((size_t)p * n_hyp + h) * HREC);
    rec[0] = {G[0], G[1], G[2], G[3]};
    rec[1] = {G[4], G[5], G[6], G[7]};
    rec[2] = {G[8], pc_bits(pc, T(0)), T(0), T(0)};
    prev[(size_t)p * n_hyp + h] = pc;  // also dense, for the order kernel's coalesced read
}

// 256 threads per pair: every block of a launch is resident at once (the kernel is latency-bound)
__global__ __launch_bounds__(256) void ransac_order_kernel(int n_hyp,
                                                           const int32_t* __restrict__ match_count,
                                                           const int32_t* __restrict__ prev,
                                                           uint16_t* __restrict__ order) {
    __shared__ int hist[PV + 2];  // bucket = preview count + 1 (degenerate -1 -> 0)
    const int p = blockIdx.x, tid = threadIdx.x;
    if (match_count[p] < 8) return;
    const int32_t* pv = prev + (size_t)p * n_hyp;
    if (tid < PV + 2) hist[tid] = 0;
    __syncthreads();
    for (int h = tid; h < n_hyp; h += 256) atomicAdd(&hist[pv[h] + 1], 1);
    __syncthreads();
    if (tid == 0) {  // descending exclusive offsets
        int off = 0;
        for (int b = PV + 1; b >= 0; --b) {
            const int c = hist[b];
            hist[b] = off;
            off += c;
        }
    }
    __syncthreads();
    for (int h = tid; h < n_hyp; h += 256)
        order[(size_t)p * n_hyp + atomicAdd(&hist[pv[h] + 1], 1)] = (uint16_t)h;
}

// COUNTS: no pruning; every hypothesis's count to out_counts[p][h] (sfm_ransac_counts)
template <typename T, bool PRUNE, bool COUNTS = false>
__global__ __launch_bounds__(256) void ransac_score_kernel(
    int n_pairs, int k_max, const int32_t* __restrict__ match_count,
    const T* __restrict__ planes, int n_hyp, int gp, const T* __restrict__ hypG,
    const uint16_t* __restrict__ order, unsigned long long* __restrict__ best, int32_t* __restrict__ out_counts = nullptr,
    uint32_t* __restrict__ exec_w = nullptr) {
    int p, hb;
    if (!xcd_pair_block(n_pairs, n_hyp >> 8, gp, p, hb)) return;
    const int M = match_count[p];
    if (M < 8) return;  // block-uniform
    const int kp = plane_len(k_max);
    const typename CPtr<T>::type S = (typename CPtr<T>::type)(planes + (size_t)p * 8 * kp + 4 * kp);
    const uint32_t h = order[(size_t)p * n_hyp + hb * 256 + threadIdx.x];
    // h is a permutation of the pair's hypotheses: one 48-byte record per hypothesis keeps the
    // lane's fetch to 1-2 cache lines (a [9][H] table scattered it over 9; PMC)
    const V4<T>* rec = (const V4<T>*)(hypG + ((size_t)p * n_hyp + h) * HREC);
    const V4<T> r0 = rec[0], r1 = rec[1], r2 = rec[2];
    const T G[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
    const int pc = pc_of(r2.y);
    int cnt = max(pc, 0);
    int mstop = PV;
    const bool alive = M <= PV || score_matches<PRUNE, CH, T>(S, kp, G, PV, M, M, cnt, best + p, &mstop);
    if (exec_w && (threadIdx.x & 63) == 0)  // sfm_ransac_stats: matches this wave scored past the preview
        exec_w[(size_t)p * (n_hyp >> 6) + hb * 4 + (threadIdx.x >> 6)] = (uint32_t)max(mstop - PV, 0);
    if (!alive) return;
    if (pc < 0) cnt = -1;
    if (COUNTS) {
        out_counts[(size_t)p * n_hyp + h] = cnt;
        return;
    }
    unsigned long long key = ((unsigned long long)(unsigned)(cnt + 1) << 32) | (0xFFFFFFFFu - h);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = o > key ? o : key;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(&best[p], key);
}

template <typename T>
__global__ __launch_bounds__(256) void ransac_final_kernel(
    int k_max, const int32_t* __restrict__ pairs, const int32_t* __restrict__ match_count,
    const T* __restrict__ planes, const T* __restrict__ norm, uint64_t seed, T thr,
    const unsigned long long* __restrict__ best, int32_t* __restrict__ out_inl_count,
    int32_t* __restrict__ out_best_h, uint8_t* __restrict__ out_mask, T* __restrict__ out_F) {
    __shared__ int wsum[4];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int M = match_count[p];
    uint8_t* mask = out_mask + (size_t)p * k_max;
    if (M < 8) {
        for (int m = tid; m < M; m += 256) mask[m] = 0;
        if (tid < 9) out_F[p * 9 + tid] = T(0);
        if (tid == 0) { out_inl_count[p] = -1; out_best_h[p] = -1; }
        return;
    }
    const uint32_t pa = (uint32_t)pairs[2 * p], pb = (uint32_t)pairs[2 * p + 1];
    const uint32_t h = 0xFFFFFFFFu - (uint32_t)best[p];
    const int kp = plane_len(k_max);
    const T* pl = planes + (size_t)p * 8 * kp;
    const T* S = pl + 4 * kp;
    const T s1 = norm[p * 6 + 2], s2 = norm[p * 6 + 5];
    T k1, k2;
    sampson_scales(s1, s2, thr, k1, k2);
    int idx[8];
    sample8(seed, pa, pb, h, M, idx);
    V4<T> smp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        smp[k] = {ldT(pl, idx[k]), ldT(pl, kp + idx[k]), ldT(pl, 2 * kp + idx[k]),
                  ldT(pl, 3 * kp + idx[k])};
    T F[9], G[9];
    const bool ok = fit_f8(smp, F);
    sampson_prep(F, k1, k2, G);
    int cnt = 0;
    for (int m = tid; m < M; m += 256) {
        const int in = ok ? sampson_inlier(G, S[m], S[kp + m], S[2 * kp + m], S[3 * kp + m]) : 0;
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
    if (tid < 9) out_F[p * 9 + tid] = ok ? F[tid] : T(0);
}

// Diagnostic (sfm_ransac_counts out_hyp_mask): every hypothesis's inlier decision on every match,
// lane per hypothesis, from the fit kernel's G record (the same scalar Sampson test).
__global__ __launch_bounds__(256) void ransac_hyp_mask_kernel(
    int k_max, const int32_t* __restrict__ match_count, const float* __restrict__ planes, int n_hyp,
    const float* __restrict__ hypG, uint8_t* __restrict__ out_mask) {
    const int p = blockIdx.x;
    const int M = match_count[p];
    if (M < 8) return;
    const int h = blockIdx.y * 256 + threadIdx.x;
    const int kp = plane_len(k_max);
    const float* S = planes + (size_t)p * 8 * kp + 4 * kp;
    const float4* rec = (const float4*)(hypG + ((size_t)p * n_hyp + h) * HREC);
    const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2];
    const float G[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
    uint8_t* o = out_mask + ((size_t)p * n_hyp + h) * k_max;
    for (int m = 0; m < M; ++m)
        o[m] = (uint8_t)sampson_inlier(G, S[m], S[kp + m], S[2 * kp + m], S[3 * kp + m]);
}

// sfm_ransac_stats: (executed, algorithmic) Sampson evaluations of a batch and its pairs with >= 8
// matches.  executed = issued lane-slots: every hypothesis's preview (min(PV, M)) + 64 x the matches
// each score wave scored past the preview (a wave runs until its last live lane stops, so lanes
// already pruned count as masked slots) + the final kernel's M; algorithmic = H x M.  Identity
// (tests/test_gpu_ransac.py, sfm_ransac_wave_stops): executed = sum over pairs with M >= 8 of
// H min(PV, M) + 64 sum_w stop_w + M, and H min(PV, M) + M <= executed <= H M + M.
__global__ __launch_bounds__(256) void ransac_stats_kernel(int n_pairs, int n_hyp,
                                                           const int32_t* __restrict__ match_count,
                                                           const uint32_t* __restrict__ exec_w,
                                                           unsigned long long* __restrict__ acc) {
    // wave per pair, grid-stride over the pairs (a few hundred blocks: three 64-bit atomics per
    // block instead of per four pairs, which serialised on one L2 line)
    __shared__ unsigned long long se[4], sa[4], sn[4];
    const int lane = threadIdx.x & 63;
    unsigned long long ex = 0, al = 0, np = 0;
    for (int p = blockIdx.x * 4 + (threadIdx.x >> 6); p < n_pairs; p += gridDim.x * 4) {
        const int M = match_count[p];
        if (M >= 8) {
            const int nw = n_hyp >> 6;
            for (int w = lane; w < nw; w += 64) ex += 64ull * exec_w[(size_t)p * nw + w];
            if (lane == 0) {
                ex += (unsigned long long)n_hyp * (unsigned)min(PV, M) + (unsigned)M;
                al += (unsigned long long)n_hyp * (unsigned)M;
                np += 1;
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ex += __shfl_xor(ex, off, 64);
    if (lane == 0) { se[threadIdx.x >> 6] = ex; sa[threadIdx.x >> 6] = al; sn[threadIdx.x >> 6] = np; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(acc, se[0] + se[1] + se[2] + se[3]);
        atomicAdd(acc + 1, sa[0] + sa[1] + sa[2] + sa[3]);
        atomicAdd(acc + 2, sn[0] + sn[1] + sn[2] + sn[3]);
    }
}

}  // namespace

// SFM_RANSAC_MODE (same results in every mode; for measuring the schedules):
//   0 ordered (fit + preview, per-pair ordering, ordered pruned scoring) — default
//   1 single pass with pruning, 2 single pass without pruning (lane per hypothesis)
// (A certified f16-MFMA scorer, exact but 4.5x slower, was mode 3 at commit 8912e00)
static int ransac_mode() {
    const char* e = getenv("SFM_RANSAC_MODE");
    const int v = e ? atoi(e) : 0;
    return (v < 0 || v > 2) ? 0 : v;
}

// Pairs per XCD group of the ordered schedule (xcd_pair_block).  Measured (profiles/r02/
// ransac_group_ab.txt): groups of 64 -3.9 % K2 at cfg4 (244 pairs per XCD per launch; the group's
// planes stay in L2), +1-2 % at cfg3 (154 per XCD; bounds publish later) -> 64 above 192 pairs
// per XCD, one group below.  SFM_RANSAC_GROUP overrides (A/B only).
static int ransac_group(int n_pairs) {
    const int q = std::max((n_pairs + 7) >> 3, 1);
    const char* e = getenv("SFM_RANSAC_GROUP");
    const int v = e ? atoi(e) : (q > 192 ? 64 : q);
    return (v <= 0 || v > q) ? q : v;
}

namespace {
struct RansacWs {
    void* planes;
    unsigned long long* best;
    void* hypG;
    int32_t* prev;
    uint16_t* order;
    uint32_t* exec_w;  // sfm_ransac_stats: per-wave scored-match counts (nullptr when off)
};
// Workspace of one batch (scalar size `rs`: 4 = f32 spec, 8 = fp64 mode).  ordered: hypothesis
// table, previews, order, and with sfm_ransac_stats on the per-wave execution counts (inside the
// one workspace, so enabling the counters never allocates on the launch path by itself).
int ransac_ws(sfm_ctx* ctx, int n_pairs, int kp, int H, bool ordered, RansacWs& w, size_t rs = 4) {
    const size_t plb = sfm::align_up((size_t)n_pairs * 8 * kp * rs, 256);
    const size_t bb = sfm::align_up((size_t)n_pairs * sizeof(unsigned long long), 256);
    const size_t gb = ordered ? sfm::align_up((size_t)n_pairs * HREC * H * rs, 256) : 0;
    const size_t vb = ordered ? sfm::align_up((size_t)n_pairs * H * sizeof(int32_t), 256) : 0;
    const size_t ob = ordered ? sfm::align_up((size_t)n_pairs * H * sizeof(uint16_t), 256) : 0;
    const bool stats = ordered && ctx->ransac_stats;
    const size_t eb = stats ? sfm::align_up((size_t)n_pairs * (H / 64) * sizeof(uint32_t), 256) : 0;
    char* ws = (char*)sfm::workspace(ctx, plb + bb + gb + vb + ob + eb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    w.exec_w = stats ? (uint32_t*)(ws + plb + bb + gb + vb + ob) : nullptr;
    w.planes = (void*)ws;
    w.best = (unsigned long long*)(ws + plb);
    w.hypG = (void*)(ws + plb + bb);
    w.prev = (int32_t*)(ws + plb + bb + gb);
    w.order = (uint16_t*)(ws + plb + bb + gb + vb);
    return SFM_OK;
}
}  // namespace

#define RANSAC_CHECK_ARGS(NAME)                                                                    \
    SFM_REQUIRE(ctx && prm, NAME ": ctx/prm is NULL");                                             \
    SFM_REQUIRE(n_pairs >= 0 && n_img >= 0 && k_max >= 0, NAME ": negative size");                 \
    if (n_pairs == 0) return SFM_OK;                                                               \
    SFM_REQUIRE(kps && pairs && match_count && matches, NAME ": NULL array");                      \
    SFM_REQUIRE(prm->n_hyp > 0 && prm->n_hyp % 256 == 0,                                           \
                NAME ": n_hyp must be a positive multiple of 256");                                \
    SFM_REQUIRE(prm->thr > 0.0f, NAME ": thr must be > 0");                                        \
    SFM_REQUIRE(k_max <= 8192, NAME ": k_max > 8192 not supported");                               \
    SFM_REQUIRE(prm->n_hyp / 256 <= 65535, NAME ": n_hyp too large")

// One batch in the scalar type T: f32 (the spec; every schedule) or f64 (the fp64 mode; the
// ordered schedule).
template <typename T>
static int ransac_batch(sfm_ctx* ctx, const T* kps, int32_t k_max, const int32_t* pairs,
                        int32_t n_pairs, const int32_t* match_count, const int32_t* matches,
                        const sfm_ransac_params* prm, int32_t* out_inl_count, int32_t* out_best_h,
                        uint8_t* out_mask, T* out_F, T* out_norm) {
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int kp = plane_len(std::max(k_max, 1));
    const int H = prm->n_hyp;
    const int mode = sizeof(T) == 4 ? ransac_mode() : 0;
    const bool ordered = mode == 0;
    SFM_REQUIRE(!ordered || H <= 65536, "sfm_ransac_f_batch: n_hyp > 65536");
    const T thr = (T)prm->thr;
    RansacWs w;
    const int rc = ransac_ws(ctx, n_pairs, kp, H, ordered, w, sizeof(T));
    if (rc != SFM_OK) return rc;
    T* planes = (T*)w.planes;
    T* hypG = (T*)w.hypG;
    SFM_HIP_CHECK(hipMemsetAsync(w.best, 0, (size_t)n_pairs * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(ransac_prep_kernel<T>, dim3(n_pairs), dim3(PREP_T), 0, st, kps, k_max,
                       pairs, match_count, matches, thr, planes, out_norm);
    SFM_HIP_CHECK(hipGetLastError());
    const dim3 grid(n_pairs, H / 256);
    uint32_t* exec_w = w.exec_w;  // sfm_ransac_stats (ordered schedule only)
    if (ordered) {
        const dim3 xgrid(xcd_grid(n_pairs, H / 256));
        const int gp = ransac_group(n_pairs);
        hipLaunchKernelGGL(ransac_fit_kernel<T>, xgrid, dim3(256), 0, st, n_pairs, k_max, pairs,
                           match_count, planes, out_norm, prm->seed, thr, H, gp, hypG, w.prev,
                           (float*)nullptr);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(ransac_order_kernel, dim3(n_pairs), dim3(256), 0, st, H, match_count,
                           w.prev, w.order);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL((ransac_score_kernel<T, true>), xgrid, dim3(256), 0, st, n_pairs, k_max,
                           match_count, planes, H, gp, hypG, w.order, w.best, (int32_t*)nullptr,
                           exec_w);
        if (exec_w) {
            SFM_HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(ransac_stats_kernel, dim3(std::min((n_pairs + 3) / 4, 512)),
                               dim3(256), 0, st, n_pairs, H, match_count, exec_w, ctx->rs_acc);
            ctx->rs_last_w = exec_w;
            ctx->rs_last_pairs = n_pairs;
            ctx->rs_last_hyp = H;
        }
    } else if constexpr (sizeof(T) == 4) {
        if (mode == 1)
            hipLaunchKernelGGL(ransac_hyp_kernel<true>, grid, dim3(256), 0, st, k_max, pairs,
                               match_count, planes, out_norm, prm->seed, prm->thr, w.best);
        else
            hipLaunchKernelGGL(ransac_hyp_kernel<false>, grid, dim3(256), 0, st, k_max, pairs,
                               match_count, planes, out_norm, prm->seed, prm->thr, w.best);
    }
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ransac_final_kernel<T>, dim3(n_pairs), dim3(256), 0, st, k_max, pairs,
                       match_count, planes, out_norm, prm->seed, thr, w.best, out_inl_count,
                       out_best_h, out_mask, out_F);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

extern "C" int sfm_ransac_f_batch(sfm_ctx* ctx, const float* kps, int32_t n_img, int32_t k_max,
                                  const int32_t* pairs, int32_t n_pairs,
                                  const int32_t* match_count, const int32_t* matches,
                                  const sfm_ransac_params* prm, int32_t* out_inl_count,
                                  int32_t* out_best_h, uint8_t* out_mask, float* out_F,
                                  float* out_norm) {
    RANSAC_CHECK_ARGS("sfm_ransac_f_batch");
    SFM_REQUIRE(out_inl_count && out_best_h && out_mask && out_F && out_norm,
                "sfm_ransac_f_batch: NULL output");
    return ransac_batch<float>(ctx, kps, k_max, pairs, n_pairs, match_count, matches, prm,
                               out_inl_count, out_best_h, out_mask, out_F, out_norm);
}

extern "C" int sfm_ransac_f_batch_f64(sfm_ctx* ctx, const double* kps, int32_t n_img,
                                      int32_t k_max, const int32_t* pairs, int32_t n_pairs,
                                      const int32_t* match_count, const int32_t* matches,
                                      const sfm_ransac_params* prm, int32_t* out_inl_count,
                                      int32_t* out_best_h, uint8_t* out_mask, double* out_F,
                                      double* out_norm) {
    RANSAC_CHECK_ARGS("sfm_ransac_f_batch_f64");
    SFM_REQUIRE(out_inl_count && out_best_h && out_mask && out_F && out_norm,
                "sfm_ransac_f_batch_f64: NULL output");
    return ransac_batch<double>(ctx, kps, k_max, pairs, n_pairs, match_count, matches, prm,
                                out_inl_count, out_best_h, out_mask, out_F, out_norm);
}

extern "C" int sfm_ransac_counts(sfm_ctx* ctx, const float* kps, int32_t n_img, int32_t k_max,
                                 const int32_t* pairs, int32_t n_pairs, const int32_t* match_count,
                                 const int32_t* matches, const sfm_ransac_params* prm,
                                 int32_t* out_counts, float* out_norm, float* out_hyp_F,
                                 uint8_t* out_hyp_mask) {
    RANSAC_CHECK_ARGS("sfm_ransac_counts");
    SFM_REQUIRE(out_counts && out_norm, "sfm_ransac_counts: NULL output");
    SFM_REQUIRE(prm->n_hyp <= 65536, "sfm_ransac_counts: n_hyp > 65536");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int kp = plane_len(std::max(k_max, 1));
    const int H = prm->n_hyp;
    RansacWs w;
    const int rc = ransac_ws(ctx, n_pairs, kp, H, true, w);
    if (rc != SFM_OK) return rc;
    // pairs with fewer than 8 matches: every count -1
    SFM_HIP_CHECK(hipMemsetAsync(out_counts, 0xFF, (size_t)n_pairs * H * sizeof(int32_t), st));
    float* planes = (float*)w.planes;
    float* hypG = (float*)w.hypG;
    hipLaunchKernelGGL(ransac_prep_kernel<float>, dim3(n_pairs), dim3(PREP_T), 0, st, kps, k_max,
                       pairs, match_count, matches, prm->thr, planes, out_norm);
    SFM_HIP_CHECK(hipGetLastError());
    const dim3 xgrid(xcd_grid(n_pairs, H / 256));
    const int gp = ransac_group(n_pairs);
    hipLaunchKernelGGL(ransac_fit_kernel<float>, xgrid, dim3(256), 0, st, n_pairs, k_max, pairs,
                       match_count, planes, out_norm, prm->seed, prm->thr, H, gp, hypG, w.prev,
                       out_hyp_F);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ransac_order_kernel, dim3(n_pairs), dim3(256), 0, st, H, match_count,
                       w.prev, w.order);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL((ransac_score_kernel<float, false, true>), xgrid, dim3(256), 0, st,
                       n_pairs, k_max, match_count, planes, H, gp, hypG, w.order, w.best,
                       out_counts, (uint32_t*)nullptr);
    SFM_HIP_CHECK(hipGetLastError());
    if (out_hyp_mask) {
        hipLaunchKernelGGL(ransac_hyp_mask_kernel, dim3(n_pairs, H / 256), dim3(256), 0, st, k_max,
                           match_count, planes, H, hypG, out_hyp_mask);
        SFM_HIP_CHECK(hipGetLastError());
    }
    return SFM_OK;
}

extern "C" int sfm_ransac_wave_stops(sfm_ctx* ctx, int32_t n_pairs, int32_t n_hyp,
                                     uint32_t* out) {
    SFM_REQUIRE(ctx && out, "sfm_ransac_wave_stops: ctx/out is NULL");
    SFM_REQUIRE(ctx->rs_last_w && n_pairs == ctx->rs_last_pairs && n_hyp == ctx->rs_last_hyp,
                "sfm_ransac_wave_stops: no counted batch of this shape (enable sfm_ransac_stats "
                "and run sfm_ransac_f_batch first; no other call on ctx in between)");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    SFM_HIP_CHECK(hipMemcpyAsync(out, ctx->rs_last_w, (size_t)n_pairs * (n_hyp / 64) * sizeof(uint32_t),
                                 hipMemcpyDeviceToHost, ctx->stream));
    SFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return SFM_OK;
}

extern "C" int sfm_ransac_stats(sfm_ctx* ctx, int32_t enable, uint64_t* out) {
    SFM_REQUIRE(ctx, "sfm_ransac_stats: ctx is NULL");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    if (!ctx->rs_acc) {
        SFM_HIP_CHECK(hipMalloc(&ctx->rs_acc, 3 * sizeof(unsigned long long)));
        SFM_HIP_CHECK(hipMemsetAsync(ctx->rs_acc, 0, 3 * sizeof(unsigned long long), ctx->stream));
    }
    if (out) {  // read and reset the counters (synchronises the context's stream)
        unsigned long long h[3];
        SFM_HIP_CHECK(hipMemcpyAsync(h, ctx->rs_acc, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
        SFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
        out[0] = h[0]; out[1] = h[1]; out[2] = h[2];
        SFM_HIP_CHECK(hipMemsetAsync(ctx->rs_acc, 0, 3 * sizeof(unsigned long long), ctx->stream));
    }
    ctx->ransac_stats = enable ? 1 : 0;
    return SFM_OK;
}
