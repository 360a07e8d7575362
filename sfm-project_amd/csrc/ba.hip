// Bundle-adjustment linearisation: residuals, Jacobians and the J^TJ blocks (K3, SURVEY.md §8a a7,
// DESIGN.md §4.3).  Fills the empty reference module code/3d_reconstruction.py.
//
// fp64 throughout.  Deterministic (no float atomics): every accumulation has a fixed order.
//   ba_obs_kernel          one thread per observation (enough waves to stream HBM): residual,
//                          J_c (2x8), J_p (2x3) -> res, W = w J_c^T J_p, and the observation's
//                          point terms (w J_p^T J_p upper triangle, w J_p^T r, rho/2) to a scratch.
//   ba_point_kernel        one thread per point: sums its observations' terms in order (pt_ptr
//                          CSR) -> V_p, g_p; fixed-tree block sum of the cost shares.
//   ba_camera_kernel       block (camera, split): recomputes J_c (cheaper than storing it: HBM is
//                          the bound) over a contiguous share of the camera's observations
//                          (cam_ptr/cam_obs CSR), fixed lane-strided order + shuffle tree.
//   ba_camera_final_kernel sums the splits in order -> U_c = sum w J_c^T J_c, g_c = sum w J_c^T r.
//   ba_cost_kernel         fixed-order sum of the block cost shares.
// Algorithmic HBM traffic ~300 B/observation; this is an HBM-bound stage.
#include <algorithm>

#include "sfm_internal.h"

namespace {

struct ObsLin {
    double r[2];
    double Jc[16];  // row-major 2x8
    double Jp[6];   // row-major 2x3
    double w, rho;
};

// Mirrors oracle_ba_obs (oracle/sfm_oracle_ba.c).
__device__ __forceinline__ void linearize(const double* __restrict__ cam, const double* __restrict__ pp,
                                          const double X[3], double u, double v, double loss_s,
                                          bool want_jp, ObsLin& o) {
    const double r0v = cam[0], r1v = cam[1], r2v = cam[2];
    const double th2 = r0v * r0v + r1v * r1v + r2v * r2v;
    double R[9];
    if (th2 > 1e-20) {
        const double th = sqrt(th2);
        double s, c;
        sincos(th, &s, &c);
        const double C = 1.0 - c;
        const double kx = r0v / th, ky = r1v / th, kz = r2v / th;
        R[0] = c + C * kx * kx;      R[1] = C * kx * ky - s * kz; R[2] = C * kx * kz + s * ky;
        R[3] = C * ky * kx + s * kz; R[4] = c + C * ky * ky;      R[5] = C * ky * kz - s * kx;
        R[6] = C * kz * kx - s * ky; R[7] = C * kz * ky + s * kx; R[8] = c + C * kz * kz;
    } else {
        R[0] = 1.0;  R[1] = -r2v; R[2] = r1v;
        R[3] = r2v;  R[4] = 1.0;  R[5] = -r0v;
        R[6] = -r1v; R[7] = r0v;  R[8] = 1.0;
    }
    double Y[3], P[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        Y[i] = R[3 * i] * X[0] + R[3 * i + 1] * X[1] + R[3 * i + 2] * X[2];
        P[i] = Y[i] + cam[3 + i];
    }
    const double iz = 1.0 / P[2];
    const double p0 = P[0] * iz, p1 = P[1] * iz;
    const double f = cam[6], k1 = cam[7];
    const double rho2 = p0 * p0 + p1 * p1;
    const double d = 1.0 + k1 * rho2;
    const double e0 = f * d * p0 + pp[0] - u;
    const double e1 = f * d * p1 + pp[1] - v;
    const double e = e0 * e0 + e1 * e1;
    double w = 1.0, rho = e;
    if (loss_s > 0.0) {
        const double s2 = loss_s * loss_s;
        w = 1.0 / (1.0 + e / s2);
        rho = s2 * log1p(e / s2);
    }
    const double m00 = f * (d + 2.0 * k1 * p0 * p0), m01 = f * (2.0 * k1 * p0 * p1);
    const double m11 = f * (d + 2.0 * k1 * p1 * p1);
    const double D[2][3] = {{iz, 0.0, -p0 * iz}, {0.0, iz, -p1 * iz}};
    double A[2][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        A[0][j] = m00 * D[0][j] + m01 * D[1][j];
        A[1][j] = m01 * D[0][j] + m11 * D[1][j];
    }
    const double S[3][3] = {{0.0, Y[2], -Y[1]}, {-Y[2], 0.0, Y[0]}, {Y[1], -Y[0], 0.0}};
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            o.Jc[8 * a + j] = A[a][0] * S[0][j] + A[a][1] * S[1][j] + A[a][2] * S[2][j];
            o.Jc[8 * a + 3 + j] = A[a][j];
            if (want_jp) o.Jp[3 * a + j] = A[a][0] * R[j] + A[a][1] * R[3 + j] + A[a][2] * R[6 + j];
        }
    o.Jc[6] = d * p0;        o.Jc[14] = d * p1;
    o.Jc[7] = f * rho2 * p0; o.Jc[15] = f * rho2 * p1;
    o.r[0] = e0; o.r[1] = e1;
    o.w = w; o.rho = rho;
}

constexpr int NV = 10;      // per-observation point terms: V upper triangle (6), g_p (3), 0.5 rho
constexpr int NU = 36 + 8;  // upper triangle of U_c (8x8) + g_c

// One thread per observation: residual, W = w J_c^T J_p, and the observation's point terms.
__global__ __launch_bounds__(256) void ba_obs_kernel(
    int n_obs, const double* __restrict__ cams, const double* __restrict__ pp,
    const double* __restrict__ pts, const int32_t* __restrict__ cam_idx,
    const int32_t* __restrict__ pt_idx, const double* __restrict__ uv, double loss_s,
    double* __restrict__ W, double* __restrict__ res, double* __restrict__ terms) {
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_obs) return;
    const int c = cam_idx[o], p = pt_idx[o];
    const double X[3] = {pts[3 * (size_t)p], pts[3 * (size_t)p + 1], pts[3 * (size_t)p + 2]};
    const double2 z = *(const double2*)(uv + 2 * (size_t)o);
    ObsLin L;
    linearize(cams + 8 * (size_t)c, pp + 2 * (size_t)c, X, z.x, z.y, loss_s, true, L);
    *(double2*)(res + 2 * (size_t)o) = make_double2(L.r[0], L.r[1]);
    double2* Wo = (double2*)(W + 24 * (size_t)o);
#pragma unroll
    for (int q = 0; q < 12; ++q) {
        const int i0 = (2 * q) / 3, j0 = (2 * q) % 3, i1 = (2 * q + 1) / 3, j1 = (2 * q + 1) % 3;
        Wo[q] = make_double2(L.w * (L.Jc[i0] * L.Jp[j0] + L.Jc[8 + i0] * L.Jp[3 + j0]),
                             L.w * (L.Jc[i1] * L.Jp[j1] + L.Jc[8 + i1] * L.Jp[3 + j1]));
    }
    double t[NV];
    int k = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i; j < 3; ++j) t[k++] = L.w * (L.Jp[i] * L.Jp[j] + L.Jp[3 + i] * L.Jp[3 + j]);
#pragma unroll
    for (int i = 0; i < 3; ++i) t[6 + i] = L.w * (L.Jp[i] * L.r[0] + L.Jp[3 + i] * L.r[1]);
    t[9] = 0.5 * L.rho;
    double2* To = (double2*)(terms + NV * (size_t)o);
#pragma unroll
    for (int q = 0; q < NV / 2; ++q) To[q] = make_double2(t[2 * q], t[2 * q + 1]);
}

// One thread per point: V_p, g_p and the cost share, summed over its observations in order; then a
// fixed-order block reduction of the cost shares.
__global__ __launch_bounds__(256) void ba_point_kernel(int n_pt, const int32_t* __restrict__ pt_ptr,
                                                       const double* __restrict__ terms,
                                                       double* __restrict__ V,
                                                       double* __restrict__ gp,
                                                       double* __restrict__ cost_blk) {
    __shared__ double red[4];
    const int p = blockIdx.x * blockDim.x + threadIdx.x, tid = threadIdx.x;
    double cost = 0.0;
    if (p < n_pt) {
        double a[NV - 1];
#pragma unroll
        for (int i = 0; i < NV - 1; ++i) a[i] = 0.0;
        const int o0 = pt_ptr[p], o1 = pt_ptr[p + 1];
        for (int o = o0; o < o1; ++o) {
            const double2* T = (const double2*)(terms + NV * (size_t)o);
#pragma unroll
            for (int q = 0; q < NV / 2; ++q) {
                const double2 v = T[q];
                if (2 * q < NV - 1) a[2 * q] += v.x; else cost += v.x;
                if (2 * q + 1 < NV - 1) a[2 * q + 1] += v.y; else cost += v.y;
            }
        }
        double* Vo = V + 9 * (size_t)p;
        Vo[0] = a[0]; Vo[1] = a[1]; Vo[2] = a[2];
        Vo[3] = a[1]; Vo[4] = a[3]; Vo[5] = a[4];
        Vo[6] = a[2]; Vo[7] = a[4]; Vo[8] = a[5];
        gp[3 * (size_t)p] = a[6]; gp[3 * (size_t)p + 1] = a[7]; gp[3 * (size_t)p + 2] = a[8];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cost += __shfl_down(cost, off, 64);
    if ((tid & 63) == 0) red[tid >> 6] = cost;
    __syncthreads();
    if (tid == 0) cost_blk[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// Block (camera c, split s): fixed-order partial U_c / g_c over its share of the camera's
// observations (J_c recomputed: cheaper than storing it, HBM is the bound).
__global__ __launch_bounds__(256) void ba_camera_kernel(
    const double* __restrict__ cams, const double* __restrict__ pp, const double* __restrict__ pts,
    const int32_t* __restrict__ pt_idx, const double* __restrict__ uv,
    const int32_t* __restrict__ cam_ptr, const int32_t* __restrict__ cam_obs, double loss_s,
    int splits, double* __restrict__ part) {
    __shared__ double red[4][NU];
    const int c = blockIdx.x, s = blockIdx.y, tid = threadIdx.x;
    double acc[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) acc[i] = 0.0;
    const double* cam = cams + 8 * (size_t)c;
    const int c0 = cam_ptr[c], c1 = cam_ptr[c + 1];
    const int len = (c1 - c0 + splits - 1) / splits;
    const int e0 = c0 + s * len, e1 = min(c1, e0 + len);
    for (int e = e0 + tid; e < e1; e += 256) {
        const int o = cam_obs[e];
        const int p = pt_idx[o];
        const double X[3] = {pts[3 * (size_t)p], pts[3 * (size_t)p + 1], pts[3 * (size_t)p + 2]};
        ObsLin L;
        linearize(cam, pp + 2 * (size_t)c, X, uv[2 * (size_t)o], uv[2 * (size_t)o + 1], loss_s,
                  false, L);
        int t = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = i; j < 8; ++j) acc[t++] += L.w * (L.Jc[i] * L.Jc[j] + L.Jc[8 + i] * L.Jc[8 + j]);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[36 + i] += L.w * (L.Jc[i] * L.r[0] + L.Jc[8 + i] * L.r[1]);
    }
#pragma unroll
    for (int i = 0; i < NU; ++i) {
        double v = acc[i];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_down(v, off, 64);
        acc[i] = v;
    }
    if ((tid & 63) == 0) {
#pragma unroll
        for (int i = 0; i < NU; ++i) red[tid >> 6][i] = acc[i];
    }
    __syncthreads();
    if (tid < NU)
        part[((size_t)c * splits + s) * NU + tid] =
            ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

// One thread per (camera, component): sum of the split partials in order -> U_c (both triangles),
// g_c.
__global__ __launch_bounds__(256) void ba_camera_final_kernel(int n_cam, int splits,
                                                              const double* __restrict__ part,
                                                              double* __restrict__ U,
                                                              double* __restrict__ gc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_cam * NU) return;
    const int c = g / NU, k = g - c * NU;
    double v = 0.0;
    for (int s = 0; s < splits; ++s) v += part[((size_t)c * splits + s) * NU + k];
    if (k >= 36) {
        gc[8 * (size_t)c + k - 36] = v;
    } else {
        int i = 0, t = k;
        while (t >= 8 - i) { t -= 8 - i; ++i; }
        const int j = i + t;
        U[64 * (size_t)c + 8 * i + j] = v;
        U[64 * (size_t)c + 8 * j + i] = v;
    }
}

__global__ __launch_bounds__(256) void ba_cost_kernel(int n, const double* __restrict__ cost_blk,
                                                      double* __restrict__ cost) {
    __shared__ double red[4];
    const int tid = threadIdx.x;
    double s = 0.0;
    for (int p = tid; p < n; p += 256) s += cost_blk[p];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_down(s, off, 64);
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) cost[0] = ((red[0] + red[1]) + red[2]) + red[3];
}

}  // namespace

extern "C" int sfm_ba_jtj(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* pp,
                          int32_t n_pt, const double* pts, int32_t n_obs, const int32_t* cam_idx,
                          const int32_t* pt_idx, const double* uv, const int32_t* pt_ptr,
                          const int32_t* cam_ptr, const int32_t* cam_obs, double loss_s,
                          double* U, double* V, double* W, double* gc, double* gp, double* res,
                          double* cost) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ba_jtj: ctx is NULL");
    SFM_REQUIRE(n_cam >= 0 && n_pt >= 0 && n_obs >= 0, "sfm_ba_jtj: negative size");
    SFM_REQUIRE(cost != nullptr, "sfm_ba_jtj: cost is NULL");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (n_pt == 0 || n_cam == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(cost, 0, sizeof(double), st));
        if (n_cam > 0) {
            SFM_HIP_CHECK(hipMemsetAsync(U, 0, sizeof(double) * 64 * n_cam, st));
            SFM_HIP_CHECK(hipMemsetAsync(gc, 0, sizeof(double) * 8 * n_cam, st));
        }
        if (n_pt > 0) {
            SFM_HIP_CHECK(hipMemsetAsync(V, 0, sizeof(double) * 9 * n_pt, st));
            SFM_HIP_CHECK(hipMemsetAsync(gp, 0, sizeof(double) * 3 * n_pt, st));
        }
        return SFM_OK;
    }
    SFM_REQUIRE(cams && pp && pts && cam_idx && pt_idx && uv && pt_ptr && cam_ptr && cam_obs && U &&
                    V && W && gc && gp && res,
                "sfm_ba_jtj: NULL array");
    // workspace: per-observation point terms | cost per point block | camera split partials
    const int n_pblk = (n_pt + 255) / 256;
    // few cameras: split each camera's observations so the grid still fills the chip
    const int splits = std::max(1, std::min(16, (256 + n_cam - 1) / n_cam));
    const size_t tb = sfm::align_up(sizeof(double) * NV * (size_t)n_obs, 256);
    const size_t cb = sfm::align_up(sizeof(double) * (size_t)n_pblk, 256);
    const size_t pb = sizeof(double) * NU * (size_t)n_cam * splits;
    char* ws = (char*)sfm::workspace(ctx, tb + cb + pb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    double* terms = (double*)ws;
    double* cost_blk = (double*)(ws + tb);
    double* part = (double*)(ws + tb + cb);
    // The observation kernel streams every input once (HBM-bound); afterwards the camera
    // reduction (latency-bound gathers of points / uv, now L2-warm) and the point reduction are
    // independent: they run concurrently on two streams.
    if (n_obs > 0) {
        hipLaunchKernelGGL(ba_obs_kernel, dim3((n_obs + 255) / 256), dim3(256), 0, st, n_obs,
                           cams, pp, pts, cam_idx, pt_idx, uv, loss_s, W, res, terms);
        SFM_HIP_CHECK(hipGetLastError());
    }
    hipStream_t aux = nullptr;
    if (sfm::aux_stream(ctx, &aux) != SFM_OK) return SFM_ERR_HIP;
    SFM_HIP_CHECK(hipEventRecord(ctx->ev_fork, st));
    SFM_HIP_CHECK(hipStreamWaitEvent(aux, ctx->ev_fork, 0));
    hipLaunchKernelGGL(ba_camera_kernel, dim3(n_cam, splits), dim3(256), 0, aux, cams, pp, pts,
                       pt_idx, uv, cam_ptr, cam_obs, loss_s, splits, part);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ba_camera_final_kernel, dim3((n_cam * NU + 255) / 256), dim3(256), 0, aux,
                       n_cam, splits, part, U, gc);
    SFM_HIP_CHECK(hipGetLastError());
    SFM_HIP_CHECK(hipEventRecord(ctx->ev_join, aux));
    hipLaunchKernelGGL(ba_point_kernel, dim3(n_pblk), dim3(256), 0, st, n_pt, pt_ptr, terms, V,
                       gp, cost_blk);
    SFM_HIP_CHECK(hipGetLastError());
    SFM_HIP_CHECK(hipStreamWaitEvent(st, ctx->ev_join, 0));
    hipLaunchKernelGGL(ba_cost_kernel, dim3(1), dim3(256), 0, st, n_pblk, cost_blk, cost);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
