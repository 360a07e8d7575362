// Next-view registration: P3P RANSAC + Gauss-Newton pose refinement (SURVEY.md §8f item 3,
// DESIGN.md §4.8).  Registers a batch of images against already-triangulated points: for each
// image, 2-D keypoints xy (pixels) with their 3-D points X (tracks), known intrinsics (f, k1, c).
//
// Spec: oracle/sfm_oracle_reg.c header (mirrored op-for-op here; only +, -, *, /, sqrt in the
// RANSAC part and no FMA contraction on either side, so counts, the winning hypothesis and the
// inlier mask are bit-identical to the CPU).  Kernels:
//   reg_hyp_kernel    lane per (hypothesis, correspondence slice) (grid: hypothesis blocks x
//                     slices x images): Philox sample of 3 correspondences, Grunert P3P (Durand-
//                     Kerner quartic roots), every pose scored over the slice; integer counts
//                     summed per hypothesis by atomics
//   reg_key_kernel    lane per hypothesis: 64-bit key (count+1) << 32 | ~(4h + root) -> wave max
//                     -> atomicMax per image
//   reg_final_kernel  block per image: the winner's pose again, inlier mask and count, then 10
//                     Gauss-Newton steps on the inliers (left rotation increment, as the BA
//                     Jacobians; fixed-order sums; 6x6 Cholesky), pose -> (angle-axis, t, f, k1)
#include "camera_model.h"
#include "sfm_internal.h"

namespace {

constexpr int REG_UNDISTORT = 10;
constexpr int REG_DK_ITERS = 48;
constexpr int REG_GN_ITERS = 10;
// Correspondence slices per hypothesis (reg_hyp_kernel): 1024 hypotheses x the candidate images
// are fewer waves than the chip has SIMDs, so every hypothesis' correspondences are cut into
// REG_SPLIT slices scored by REG_SPLIT lanes (each solves the P3P again) and the integer counts
// are summed by atomics — exact in any order — before the key kernel picks the winner.
#ifndef REG_SPLIT
#define REG_SPLIT 4
#endif

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

__device__ __forceinline__ void sample3(uint64_t seed, uint32_t img, uint32_t h, int n, int idx[3]) {
    uint32_t r[4];
    philox4x32_10(h, 2u, img, 0x52454731u, (uint32_t)seed, (uint32_t)(seed >> 32), r);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t jmax = (uint32_t)(n - 3 + k);
        uint32_t t = __umulhi(r[k], jmax + 1u);
        bool dup = false;
#pragma unroll
        for (int q = 0; q < k; ++q) dup = dup || ((uint32_t)idx[q] == t);
        idx[k] = (int)(dup ? jmax : t);
    }
}

__device__ __forceinline__ void bearing(double x, double y, const double* intr, double b[3]) {
    const double f = intr[0], k1 = intr[1];
    const double xd0 = (x - intr[2]) / f, xd1 = (y - intr[3]) / f;
    double x0 = xd0, x1 = xd1;
    for (int it = 0; it < REG_UNDISTORT; ++it) {
        const double s = 1.0 + k1 * (x0 * x0 + x1 * x1);
        x0 = xd0 / s;
        x1 = xd1 / s;
    }
    const double n = sqrt(x0 * x0 + x1 * x1 + 1.0);
    b[0] = x0 / n; b[1] = x1 / n; b[2] = 1.0 / n;
}

__device__ __forceinline__ void cmul(double a, double b, double c, double d, double& re, double& im) {
    re = a * c - b * d;
    im = a * d + b * c;
}
__device__ __forceinline__ void cdiv(double a, double b, double c, double d, double& re, double& im) {
    const double den = c * c + d * d;
    re = (a * c + b * d) / den;
    im = (b * c - a * d) / den;
}

__device__ void dk_roots(const double c[4], double re[4], double im[4]) {
    double R = 1.0;
    for (int i = 0; i < 4; ++i) R = fmax(R, 1.0 + fabs(c[i]));
    double wr = 1.0, wi = 0.0;
    for (int k = 0; k < 4; ++k) {
        re[k] = R * wr; im[k] = R * wi;
        double tr, ti;
        cmul(wr, wi, 0.4, 0.9, tr, ti);
        wr = tr; wi = ti;
    }
    for (int it = 0; it < REG_DK_ITERS; ++it) {
        for (int k = 0; k < 4; ++k) {
            double pr = 1.0, pi = 0.0;
            for (int i = 3; i >= 0; --i) {
                double tr, ti;
                cmul(pr, pi, re[k], im[k], tr, ti);
                pr = tr + c[i]; pi = ti;
            }
            double qr = 1.0, qi = 0.0;
            for (int j = 0; j < 4; ++j) {
                if (j == k) continue;
                double tr, ti;
                cmul(qr, qi, re[k] - re[j], im[k] - im[j], tr, ti);
                qr = tr; qi = ti;
            }
            if (qr == 0.0 && qi == 0.0) continue;
            double dr, di;
            cdiv(pr, pi, qr, qi, dr, di);
            re[k] = re[k] - dr;
            im[k] = im[k] - di;
        }
    }
}

__device__ bool tri_frame(const double X[3][3], double F[9]) {
    double e1[3] = {X[1][0] - X[0][0], X[1][1] - X[0][1], X[1][2] - X[0][2]};
    const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    if (!(n1 > 0.0)) return false;
    e1[0] = e1[0] / n1; e1[1] = e1[1] / n1; e1[2] = e1[2] / n1;
    const double d[3] = {X[2][0] - X[0][0], X[2][1] - X[0][1], X[2][2] - X[0][2]};
    double e3[3] = {e1[1] * d[2] - e1[2] * d[1], e1[2] * d[0] - e1[0] * d[2],
                    e1[0] * d[1] - e1[1] * d[0]};
    const double n3 = sqrt(e3[0] * e3[0] + e3[1] * e3[1] + e3[2] * e3[2]);
    if (!(n3 > 0.0)) return false;
    e3[0] = e3[0] / n3; e3[1] = e3[1] / n3; e3[2] = e3[2] / n3;
    const double e2[3] = {e3[1] * e1[2] - e3[2] * e1[1], e3[2] * e1[0] - e3[0] * e1[2],
                          e3[0] * e1[1] - e3[1] * e1[0]};
    for (int i = 0; i < 3; ++i) { F[3 * i] = e1[i]; F[3 * i + 1] = e2[i]; F[3 * i + 2] = e3[i]; }
    return true;
}

// Grunert P3P; ok[k] marks valid root slots (mirrors oracle_reg_p3p).
__device__ void p3p(const double b[3][3], const double X[3][3], double Rs[4][9], double ts[4][3],
                    bool ok[4]) {
    for (int k = 0; k < 4; ++k) ok[k] = false;
    double dx, dy, dz;
    dx = X[1][0] - X[2][0]; dy = X[1][1] - X[2][1]; dz = X[1][2] - X[2][2];
    const double a2 = dx * dx + dy * dy + dz * dz;
    dx = X[0][0] - X[2][0]; dy = X[0][1] - X[2][1]; dz = X[0][2] - X[2][2];
    const double b2 = dx * dx + dy * dy + dz * dz;
    dx = X[0][0] - X[1][0]; dy = X[0][1] - X[1][1]; dz = X[0][2] - X[1][2];
    const double c2 = dx * dx + dy * dy + dz * dz;
    if (!(b2 > 0.0)) return;
    const double ca = b[1][0] * b[2][0] + b[1][1] * b[2][1] + b[1][2] * b[2][2];
    const double cb = b[0][0] * b[2][0] + b[0][1] * b[2][1] + b[0][2] * b[2][2];
    const double cg = b[0][0] * b[1][0] + b[0][1] * b[1][1] + b[0][2] * b[1][2];
    const double p = (a2 - c2) / b2, q = (a2 + c2) / b2;
    const double cb2 = c2 / b2, ab2 = a2 / b2, bc2 = (b2 - c2) / b2, ba2 = (b2 - a2) / b2;
    const double A4 = (p - 1.0) * (p - 1.0) - 4.0 * cb2 * ca * ca;
    const double A3 = 4.0 * (p * (1.0 - p) * cb - (1.0 - q) * ca * cg + 2.0 * cb2 * ca * ca * cb);
    const double A2 = 2.0 * (p * p - 1.0 + 2.0 * p * p * cb * cb + 2.0 * bc2 * ca * ca
                             - 4.0 * q * ca * cb * cg + 2.0 * ba2 * cg * cg);
    const double A1 = 4.0 * (-p * (1.0 + p) * cb + 2.0 * ab2 * cg * cg * cb - (1.0 - q) * ca * cg);
    const double A0 = (1.0 + p) * (1.0 + p) - 4.0 * ab2 * cg * cg;
    const double amax = fmax(fmax(fabs(A3), fabs(A2)), fmax(fabs(A1), fabs(A0)));
    if (!(fabs(A4) > 1e-12 * amax)) return;
    const double c[4] = {A0 / A4, A1 / A4, A2 / A4, A3 / A4};
    double re[4], im[4];
    dk_roots(c, re, im);
    double FP[9];
    if (!tri_frame(X, FP)) return;
    for (int k = 0; k < 4; ++k) {
        if (!(fabs(im[k]) <= 1e-7 * (1.0 + fabs(re[k])))) continue;
        double v = re[k];
        for (int it = 0; it < 2; ++it) {
            const double pv = (((v + c[3]) * v + c[2]) * v + c[1]) * v + c[0];
            const double dv = ((4.0 * v + 3.0 * c[3]) * v + 2.0 * c[2]) * v + c[1];
            if (dv != 0.0) v = v - pv / dv;
        }
        const double den_u = 2.0 * (cg - v * ca);
        if (den_u == 0.0) continue;
        const double u = ((-1.0 + p) * v * v - 2.0 * p * cb * v + 1.0 + p) / den_u;
        const double den = 1.0 + u * u - 2.0 * u * cg;
        if (!(den > 0.0)) continue;
        const double s1 = sqrt(c2 / den), s2 = u * s1, s3 = v * s1;
        if (!(s1 > 0.0 && s2 > 0.0 && s3 > 0.0)) continue;
        double Q[3][3];
        for (int i = 0; i < 3; ++i) {
            Q[0][i] = s1 * b[0][i]; Q[1][i] = s2 * b[1][i]; Q[2][i] = s3 * b[2][i];
        }
        double FQ[9];
        if (!tri_frame(Q, FQ)) continue;
        double* R = Rs[k];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                R[3 * i + j] = FQ[3 * i] * FP[3 * j] + FQ[3 * i + 1] * FP[3 * j + 1]
                               + FQ[3 * i + 2] * FP[3 * j + 2];
        for (int i = 0; i < 3; ++i)
            ts[k][i] = Q[0][i] - (R[3 * i] * X[0][0] + R[3 * i + 1] * X[0][1] + R[3 * i + 2] * X[0][2]);
        ok[k] = true;
    }
}

__device__ __forceinline__ bool inlier(const double R[9], const double t[3], const double* intr,
                                       double x, double y, const double* X, double thr2) {
    const double P0 = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
    const double P1 = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
    const double P2 = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
    if (!(P2 > 0.0)) return false;
    const double q0 = P0 / P2, q1 = P1 / P2;
    const double d = 1.0 + intr[1] * (q0 * q0 + q1 * q1);
    const double e0 = intr[0] * d * q0 + intr[2] - x;
    const double e1 = intr[0] * d * q1 + intr[3] - y;
    return (e0 * e0 + e1 * e1) < thr2;
}

// The hypothesis' poses for image `img` (sample + P3P).
__device__ void hypothesis(uint64_t seed, uint32_t img, uint32_t h, int n,
                           const double* __restrict__ xy, const double* __restrict__ X,
                           const double* intr, double Rs[4][9], double ts[4][3], bool ok[4]) {
    int idx[3];
    sample3(seed, img, h, n, idx);
    double b[3][3], Xs[3][3];
    for (int i = 0; i < 3; ++i) {
        bearing(xy[2 * (size_t)idx[i]], xy[2 * (size_t)idx[i] + 1], intr, b[i]);
        for (int j = 0; j < 3; ++j) Xs[i][j] = X[3 * (size_t)idx[i] + j];
    }
    p3p(b, Xs, Rs, ts, ok);
}

__global__ __launch_bounds__(256) void reg_hyp_kernel(
    const int32_t* __restrict__ corr_ptr, const double* __restrict__ xy,
    const double* __restrict__ X, const double* __restrict__ intr_all,
    const int32_t* __restrict__ img_id, uint64_t seed, double thr2, int n_hyp,
    unsigned long long* __restrict__ best, int32_t* __restrict__ cnt_g,
    uint8_t* __restrict__ ok_g) {
    const int im = blockIdx.y;
    const int c0 = corr_ptr[im], n = corr_ptr[im + 1] - c0;
    if (n < 3) return;
    const int sl = (int)blockIdx.x % REG_SPLIT;   // this lane's correspondence slice
    const uint32_t h = (blockIdx.x / REG_SPLIT) * blockDim.x + threadIdx.x;
    const double* intr = intr_all + 4 * (size_t)im;
    const double* xyi = xy + 2 * (size_t)c0;
    const double* Xi = X + 3 * (size_t)c0;
    double Rs[4][9], ts[4][3];
    bool ok[4];
    hypothesis(seed, (uint32_t)img_id[im], h, n, xyi, Xi, intr, Rs, ts, ok);
    // the poses of a hypothesis scored together, one pass over the slice: each correspondence is
    // loaded once and the (up to) four independent division chains overlap (reg_hyp 21.6 ->
    // 17.1 ms per cfg5 reconstruction before the slices).  Per-evaluation arithmetic as the spec.
    const int m0 = (int)((long long)n * sl / REG_SPLIT), m1 = (int)((long long)n * (sl + 1) / REG_SPLIT);
    int cnt[4] = {0, 0, 0, 0};
    const bool any0 = __any(ok[0]), any1 = __any(ok[1]), any2 = __any(ok[2]), any3 = __any(ok[3]);
    for (int m = m0; m < m1; ++m) {  // wave-uniform correspondence loads
        const double x = xyi[2 * m], y = xyi[2 * m + 1];
        const double* Xm = Xi + 3 * m;
        if (any0) cnt[0] += (ok[0] && inlier(Rs[0], ts[0], intr, x, y, Xm, thr2)) ? 1 : 0;
        if (any1) cnt[1] += (ok[1] && inlier(Rs[1], ts[1], intr, x, y, Xm, thr2)) ? 1 : 0;
        if (any2) cnt[2] += (ok[2] && inlier(Rs[2], ts[2], intr, x, y, Xm, thr2)) ? 1 : 0;
        if (any3) cnt[3] += (ok[3] && inlier(Rs[3], ts[3], intr, x, y, Xm, thr2)) ? 1 : 0;
    }
    if (REG_SPLIT > 1) {   // slice counts -> the hypothesis' totals (reg_key_kernel takes over)
        int32_t* cg = cnt_g + ((size_t)im * n_hyp + h) * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (ok[k] && cnt[k]) atomicAdd(cg + k, cnt[k]);
        if (sl == 0)
            ok_g[(size_t)im * n_hyp + h] = (uint8_t)(ok[0] | (ok[1] << 1) | (ok[2] << 2) | (ok[3] << 3));
        return;
    }
    unsigned long long key = 0ull;
    for (int k = 0; k < 4; ++k) {
        if (!ok[k]) continue;
        const unsigned long long kk = ((unsigned long long)(cnt[k] + 1) << 32) |
                                      (unsigned long long)(0xFFFFFFFFu - (4u * h + k));
        key = key > kk ? key : kk;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = key > o ? key : o;
    }
    if ((threadIdx.x & 63) == 0 && key) atomicMax(best + im, key);
}

// REG_SPLIT > 1: the winner key per image from the summed slice counts (lane per hypothesis).
__global__ __launch_bounds__(256) void reg_key_kernel(const int32_t* __restrict__ corr_ptr,
                                                      int n_hyp, const int32_t* __restrict__ cnt_g,
                                                      const uint8_t* __restrict__ ok_g,
                                                      unsigned long long* __restrict__ best) {
    const int im = blockIdx.y;
    if (corr_ptr[im + 1] - corr_ptr[im] < 3) return;
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    const int okb = ok_g[(size_t)im * n_hyp + h];
    const int32_t* cg = cnt_g + ((size_t)im * n_hyp + h) * 4;
    unsigned long long key = 0ull;
    for (int k = 0; k < 4; ++k) {
        if (!((okb >> k) & 1)) continue;
        const unsigned long long kk = ((unsigned long long)(cg[k] + 1) << 32) |
                                      (unsigned long long)(0xFFFFFFFFu - (4u * h + k));
        key = key > kk ? key : kk;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = key > o ? key : o;
    }
    if ((threadIdx.x & 63) == 0 && key) atomicMax(best + im, key);
}

// 6x6 SPD solve by Cholesky (one thread).  Returns false if not SPD.
__device__ bool chol6_solve(double A[36], double b[6], double x[6]) {
    double L[36];
    for (int k = 0; k < 36; ++k) L[k] = 0.0;
    for (int j = 0; j < 6; ++j) {
        double s = A[6 * j + j];
        for (int k = 0; k < j; ++k) s -= L[6 * j + k] * L[6 * j + k];
        if (!(s > 0.0)) return false;
        L[6 * j + j] = sqrt(s);
        for (int i = j + 1; i < 6; ++i) {
            double t = A[6 * i + j];
            for (int k = 0; k < j; ++k) t -= L[6 * i + k] * L[6 * j + k];
            L[6 * i + j] = t / L[6 * j + j];
        }
    }
    double y[6];
    for (int i = 0; i < 6; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= L[6 * i + k] * y[k];
        y[i] = t / L[6 * i + i];
    }
    for (int i = 5; i >= 0; --i) {
        double t = y[i];
        for (int k = i + 1; k < 6; ++k) t -= L[6 * k + i] * x[k];
        x[i] = t / L[6 * i + i];
    }
    return true;
}

__global__ __launch_bounds__(256) void reg_final_kernel(
    const int32_t* __restrict__ corr_ptr, const double* __restrict__ xy,
    const double* __restrict__ X, const double* __restrict__ intr_all,
    const int32_t* __restrict__ img_id, uint64_t seed, double thr2, int refine,
    const unsigned long long* __restrict__ best, double* __restrict__ cam_out,
    int32_t* __restrict__ count_out, int32_t* __restrict__ key_out, uint8_t* __restrict__ mask) {
    constexpr int N = 27;  // 21 upper-triangle JᵀJ + 6 Jᵀr
    __shared__ double Rsh[9], tsh[3];
    __shared__ double red[4][N];
    __shared__ double tot[N];
    __shared__ int cnt_s[4];
    __shared__ int valid_s;
    const int im = blockIdx.x, tid = threadIdx.x;
    const int c0 = corr_ptr[im], n = corr_ptr[im + 1] - c0;
    const double* intr = intr_all + 4 * (size_t)im;
    const double* xyi = xy + 2 * (size_t)c0;
    const double* Xi = X + 3 * (size_t)c0;
    const unsigned long long key = best[im];
    if (tid == 0) {
        valid_s = 0;
        if (key != 0ull && n >= 3) {
            const uint32_t hk = 0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull);
            double Rs[4][9], ts[4][3];
            bool ok[4];
            hypothesis(seed, (uint32_t)img_id[im], hk >> 2, n, xyi, Xi, intr, Rs, ts, ok);
            const int k = hk & 3;
            if (ok[k]) {
                for (int i = 0; i < 9; ++i) Rsh[i] = Rs[k][i];
                for (int i = 0; i < 3; ++i) tsh[i] = ts[k][i];
                valid_s = 1;
            }
            key_out[im] = (int32_t)hk;
        } else {
            key_out[im] = -1;
        }
    }
    __syncthreads();
    if (!valid_s) {
        for (int m = tid; m < n; m += 256) mask[c0 + m] = 0;
        if (tid == 0) {
            count_out[im] = -1;
            for (int i = 0; i < 8; ++i) cam_out[8 * (size_t)im + i] = 0.0;
        }
        return;
    }
    // inlier mask and count of the RANSAC winner
    double R[9], t[3];
    for (int i = 0; i < 9; ++i) R[i] = Rsh[i];
    for (int i = 0; i < 3; ++i) t[i] = tsh[i];
    int c = 0;
    for (int m = tid; m < n; m += 256) {
        const bool in = inlier(R, t, intr, xyi[2 * m], xyi[2 * m + 1], Xi + 3 * m, thr2);
        mask[c0 + m] = in ? 1 : 0;
        c += in ? 1 : 0;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_down(c, off, 64);
    if ((tid & 63) == 0) cnt_s[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) count_out[im] = cnt_s[0] + cnt_s[1] + cnt_s[2] + cnt_s[3];
    // Gauss-Newton on the inliers: residual e = pred - xy, J = d pred / d(δr, t)
    for (int it = 0; refine && it < REG_GN_ITERS; ++it) {
        double acc[N];
        for (int i = 0; i < N; ++i) acc[i] = 0.0;
        for (int m = tid; m < n; m += 256) {
            if (!mask[c0 + m]) continue;
            const double* Xm = Xi + 3 * m;
            const double Y0 = R[0] * Xm[0] + R[1] * Xm[1] + R[2] * Xm[2];
            const double Y1 = R[3] * Xm[0] + R[4] * Xm[1] + R[5] * Xm[2];
            const double Y2 = R[6] * Xm[0] + R[7] * Xm[1] + R[8] * Xm[2];
            const double P0 = Y0 + t[0], P1 = Y1 + t[1], P2 = Y2 + t[2];
            const double iz = 1.0 / P2, p0 = P0 * iz, p1 = P1 * iz;
            const double f = intr[0], k1 = intr[1], rho2 = p0 * p0 + p1 * p1, d = 1.0 + k1 * rho2;
            const double e0 = f * d * p0 + intr[2] - xyi[2 * m];
            const double e1 = f * d * p1 + intr[3] - xyi[2 * m + 1];
            const double m00 = f * (d + 2.0 * k1 * p0 * p0), m01 = f * (2.0 * k1 * p0 * p1);
            const double m11 = f * (d + 2.0 * k1 * p1 * p1);
            const double D[2][3] = {{iz, 0.0, -p0 * iz}, {0.0, iz, -p1 * iz}};
            double A[2][3];
            for (int j = 0; j < 3; ++j) {
                A[0][j] = m00 * D[0][j] + m01 * D[1][j];
                A[1][j] = m01 * D[0][j] + m11 * D[1][j];
            }
            const double S[3][3] = {{0.0, Y2, -Y1}, {-Y2, 0.0, Y0}, {Y1, -Y0, 0.0}};
            double J[2][6];
            for (int a = 0; a < 2; ++a)
                for (int j = 0; j < 3; ++j) {
                    J[a][j] = A[a][0] * S[0][j] + A[a][1] * S[1][j] + A[a][2] * S[2][j];
                    J[a][3 + j] = A[a][j];
                }
            int q = 0;
            for (int i = 0; i < 6; ++i)
                for (int j = i; j < 6; ++j) acc[q++] += J[0][i] * J[0][j] + J[1][i] * J[1][j];
            for (int i = 0; i < 6; ++i) acc[21 + i] += J[0][i] * e0 + J[1][i] * e1;
        }
        for (int i = 0; i < N; ++i) {
            double v = acc[i];
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_down(v, off, 64);
            acc[i] = v;
        }
        if ((tid & 63) == 0)
            for (int i = 0; i < N; ++i) red[tid >> 6][i] = acc[i];
        __syncthreads();
        if (tid < N) tot[tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
        __syncthreads();
        if (tid == 0) {
            double H[36], g[6], dx[6];
            int q = 0;
            for (int i = 0; i < 6; ++i)
                for (int j = i; j < 6; ++j) { H[6 * i + j] = tot[q]; H[6 * j + i] = tot[q]; ++q; }
            for (int i = 0; i < 6; ++i) g[i] = -tot[21 + i];
            if (chol6_solve(H, g, dx)) {
                double Ad[9], Rn[9];
                rotmat(dx[0], dx[1], dx[2], Ad);
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k)
                        Rn[3 * r + k] = Ad[3 * r] * R[k] + Ad[3 * r + 1] * R[3 + k] + Ad[3 * r + 2] * R[6 + k];
                for (int i = 0; i < 9; ++i) Rsh[i] = Rn[i];
                for (int i = 0; i < 3; ++i) tsh[i] = t[i] + dx[3 + i];
            }
        }
        __syncthreads();
        for (int i = 0; i < 9; ++i) R[i] = Rsh[i];
        for (int i = 0; i < 3; ++i) t[i] = tsh[i];
        __syncthreads();
    }
    if (tid == 0) {
        // pose -> angle-axis (log map, stable near 0 and pi), t, f, k1
        const double cs = fmin(fmax(0.5 * ((R[0] + R[4] + R[8]) - 1.0), -1.0), 1.0);
        const double w0 = R[7] - R[5], w1 = R[2] - R[6], w2 = R[3] - R[1];
        const double sn = 0.5 * sqrt(w0 * w0 + w1 * w1 + w2 * w2);
        const double th = atan2(sn, cs);
        double o0, o1, o2;
        if (sn > 1e-7) {
            const double k = th / (2.0 * sn);
            o0 = w0 * k; o1 = w1 * k; o2 = w2 * k;
        } else if (cs > 0.0) {
            o0 = 0.5 * w0; o1 = 0.5 * w1; o2 = 0.5 * w2;
        } else {
            const double B0 = 0.5 * (R[0] + 1.0), B4 = 0.5 * (R[4] + 1.0), B8 = 0.5 * (R[8] + 1.0);
            const int j = (B0 >= B4 && B0 >= B8) ? 0 : (B4 >= B8 ? 1 : 2);
            const double bjj = j == 0 ? B0 : (j == 1 ? B4 : B8);
            const double sq = sqrt(bjj);
            double a0 = (j == 0 ? B0 : 0.5 * R[j]) / sq;
            double a1 = (j == 1 ? B4 : 0.5 * R[3 + j]) / sq;
            double a2 = (j == 2 ? B8 : 0.5 * R[6 + j]) / sq;
            if (a0 * w0 + a1 * w1 + a2 * w2 < 0.0) { a0 = -a0; a1 = -a1; a2 = -a2; }
            const double nn = sqrt(a0 * a0 + a1 * a1 + a2 * a2);
            o0 = th * a0 / nn; o1 = th * a1 / nn; o2 = th * a2 / nn;
        }
        double* out = cam_out + 8 * (size_t)im;
        out[0] = o0; out[1] = o1; out[2] = o2;
        out[3] = t[0]; out[4] = t[1]; out[5] = t[2];
        out[6] = intr[0]; out[7] = intr[1];
    }
}

}  // namespace

extern "C" int sfm_register_batch(sfm_ctx* ctx, int32_t n_img, const int32_t* corr_ptr,
                                  const double* xy, const double* X, const double* intr,
                                  const int32_t* img_id, const sfm_register_params* prm,
                                  double* out_cams, int32_t* out_count, int32_t* out_key,
                                  uint8_t* out_mask) {
    SFM_REQUIRE(ctx != nullptr && prm != nullptr, "sfm_register_batch: ctx/prm is NULL");
    SFM_REQUIRE(n_img >= 0, "sfm_register_batch: negative size");
    SFM_REQUIRE(prm->n_hyp > 0 && prm->n_hyp % 256 == 0 && prm->n_hyp <= (1 << 28),
                "sfm_register_batch: n_hyp must be a positive multiple of 256");
    SFM_REQUIRE(prm->thr > 0.0, "sfm_register_batch: thr must be > 0");
    if (n_img == 0) return SFM_OK;
    SFM_REQUIRE(corr_ptr && xy && X && intr && img_id && out_cams && out_count && out_key &&
                    out_mask,
                "sfm_register_batch: NULL array");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // workspace: best keys [n_img] u64, then (REG_SPLIT > 1) slice-count sums [n_img][n_hyp][4]
    // i32 and pose flags [n_img][n_hyp] u8; keys and sums zeroed in one memset
    const size_t bb = sfm::align_up(sizeof(unsigned long long) * (size_t)n_img, 256);
    const size_t cb = REG_SPLIT > 1 ? sizeof(int32_t) * 4 * (size_t)n_img * prm->n_hyp : 0;
    const size_t ob = REG_SPLIT > 1 ? (size_t)n_img * prm->n_hyp : 0;
    char* ws = (char*)sfm::workspace(ctx, bb + cb + ob);
    if (!ws) return SFM_ERR_NOMEM;
    unsigned long long* best = (unsigned long long*)ws;
    int32_t* cnt_g = (int32_t*)(ws + bb);
    uint8_t* ok_g = (uint8_t*)(ws + bb + cb);
    SFM_HIP_CHECK(hipMemsetAsync(ws, 0, bb + cb, st));
    const double thr2 = prm->thr * prm->thr;
    hipLaunchKernelGGL(reg_hyp_kernel, dim3(prm->n_hyp / 256 * REG_SPLIT, n_img), dim3(256), 0, st,
                       corr_ptr, xy, X, intr, img_id, (uint64_t)prm->seed, thr2, prm->n_hyp, best,
                       cnt_g, ok_g);
    SFM_HIP_CHECK(hipGetLastError());
    if (REG_SPLIT > 1) {
        hipLaunchKernelGGL(reg_key_kernel, dim3(prm->n_hyp / 256, n_img), dim3(256), 0, st,
                           corr_ptr, prm->n_hyp, cnt_g, ok_g, best);
        SFM_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(reg_final_kernel, dim3(n_img), dim3(256), 0, st, corr_ptr, xy, X, intr,
                       img_id, (uint64_t)prm->seed, thr2, prm->refine, best, out_cams, out_count,
                       out_key, out_mask);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
