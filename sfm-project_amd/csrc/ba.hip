// Bundle-adjustment linearisation: residuals, Jacobians and the J^TJ blocks (K3, SURVEY.md §8a a7,
// DESIGN.md §4.3).  Fills the empty reference module code/3d_reconstruction.py.
//
// fp64 throughout.  Deterministic (no float atomics): every accumulation has a fixed order.
//   ba_point_kernel   one thread per point, its observations are contiguous (pt_ptr CSR):
//                     residual, J_c (2x8), J_p (2x3) per observation -> res, W = w J_c^T J_p,
//                     V_p = sum w J_p^T J_p, g_p = sum w J_p^T r, the point's cost share.
//   ba_camera_kernel  one 256-thread block per camera over its observation list (cam_ptr/cam_obs
//                     CSR): recomputes J_c (cheaper than storing it: HBM is the bound) and reduces
//                     U_c = sum w J_c^T J_c and g_c = sum w J_c^T r with a fixed lane-strided order
//                     plus a fixed shuffle tree.
//   ba_cost_kernel    one block: fixed-order sum of the per-point cost shares.
// Algorithmic HBM traffic ~300 B/observation; this is an HBM-bound stage.
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

__global__ __launch_bounds__(256) void ba_point_kernel(
    int n_pt, const double* __restrict__ cams, const double* __restrict__ pp,
    const double* __restrict__ pts, const int32_t* __restrict__ cam_idx,
    const double* __restrict__ uv, const int32_t* __restrict__ pt_ptr, double loss_s,
    double* __restrict__ V, double* __restrict__ W, double* __restrict__ gp,
    double* __restrict__ res, double* __restrict__ cost_pt) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pt) return;
    const double X[3] = {pts[3 * (size_t)p], pts[3 * (size_t)p + 1], pts[3 * (size_t)p + 2]};
    double Vp[6] = {0, 0, 0, 0, 0, 0};  // upper triangle 00 01 02 11 12 22
    double g[3] = {0, 0, 0};
    double cost = 0.0;
    const int o0 = pt_ptr[p], o1 = pt_ptr[p + 1];
    for (int o = o0; o < o1; ++o) {
        const int c = cam_idx[o];
        ObsLin L;
        linearize(cams + 8 * (size_t)c, pp + 2 * (size_t)c, X, uv[2 * (size_t)o],
                  uv[2 * (size_t)o + 1], loss_s, true, L);
        cost += 0.5 * L.rho;
        res[2 * (size_t)o] = L.r[0];
        res[2 * (size_t)o + 1] = L.r[1];
        double* Wo = W + 24 * (size_t)o;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Wo[3 * i + j] = L.w * (L.Jc[i] * L.Jp[j] + L.Jc[8 + i] * L.Jp[3 + j]);
        int t = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = i; j < 3; ++j) Vp[t++] += L.w * (L.Jp[i] * L.Jp[j] + L.Jp[3 + i] * L.Jp[3 + j]);
            g[i] += L.w * (L.Jp[i] * L.r[0] + L.Jp[3 + i] * L.r[1]);
        }
    }
    double* Vo = V + 9 * (size_t)p;
    Vo[0] = Vp[0]; Vo[1] = Vp[1]; Vo[2] = Vp[2];
    Vo[3] = Vp[1]; Vo[4] = Vp[3]; Vo[5] = Vp[4];
    Vo[6] = Vp[2]; Vo[7] = Vp[4]; Vo[8] = Vp[5];
    gp[3 * (size_t)p] = g[0]; gp[3 * (size_t)p + 1] = g[1]; gp[3 * (size_t)p + 2] = g[2];
    cost_pt[p] = cost;
}

constexpr int NU = 36 + 8;  // upper triangle of U_c (8x8) + g_c

__global__ __launch_bounds__(256) void ba_camera_kernel(
    const double* __restrict__ cams, const double* __restrict__ pp, const double* __restrict__ pts,
    const int32_t* __restrict__ pt_idx, const double* __restrict__ uv,
    const int32_t* __restrict__ cam_ptr, const int32_t* __restrict__ cam_obs, double loss_s,
    double* __restrict__ U, double* __restrict__ gc) {
    __shared__ double red[4][NU];
    const int c = blockIdx.x, tid = threadIdx.x;
    double acc[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) acc[i] = 0.0;
    const double* cam = cams + 8 * (size_t)c;
    const int e0 = cam_ptr[c], e1 = cam_ptr[c + 1];
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
    if (tid < NU) {
        const double v = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
        if (tid >= 36) {
            gc[8 * (size_t)c + tid - 36] = v;
        } else {
            // map upper-triangle index -> (i, j)
            int i = 0, t = tid;
            while (t >= 8 - i) { t -= 8 - i; ++i; }
            const int j = i + t;
            U[64 * (size_t)c + 8 * i + j] = v;
            U[64 * (size_t)c + 8 * j + i] = v;
        }
    }
}

__global__ __launch_bounds__(256) void ba_cost_kernel(int n_pt, const double* __restrict__ cost_pt,
                                                      double* __restrict__ cost) {
    __shared__ double red[4];
    const int tid = threadIdx.x;
    double s = 0.0;
    for (int p = tid; p < n_pt; p += 256) s += cost_pt[p];
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
    double* cost_pt = (double*)sfm::workspace(ctx, sizeof(double) * (size_t)n_pt + 1024);
    if (!cost_pt) return SFM_ERR_NOMEM;
    hipLaunchKernelGGL(ba_point_kernel, dim3((n_pt + 255) / 256), dim3(256), 0, st, n_pt, cams, pp,
                       pts, cam_idx, uv, pt_ptr, loss_s, V, W, gp, res, cost_pt);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ba_camera_kernel, dim3(n_cam), dim3(256), 0, st, cams, pp, pts, pt_idx, uv,
                       cam_ptr, cam_obs, loss_s, U, gc);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ba_cost_kernel, dim3(1), dim3(256), 0, st, n_pt, cost_pt, cost);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
