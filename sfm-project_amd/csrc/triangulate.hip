// Multi-view triangulation of tracks: the 3-D points that
// bundle adjustment starts from.  Restated by oracle/recon.py (triangulate), which the GPU tests
// compare against.
//
// Spec, per point (thread per point; its observations are the CSR range pt_ptr[p]..pt_ptr[p+1]):
//   x_d = (uv - pp) / f;  undistort x (1 + k1 |x|^2) = x_d by 10 fixed-point steps from x = x_d;
//   DLT rows x_0 P_2 - P_0, x_1 P_2 - P_1 per view (P = [R | t]), M = Σ rowsᵀ rows (4x4);
//   X = the eigenvector of M's smallest eigenvalue (cyclic Jacobi, <= 10 sweeps), dehomogenised;
//   stats = {mean reprojection error (px, full camera model), largest angle between two viewing
//            rays (degrees), smallest depth, status}: status 0 ok, 1 fewer than 2 observations,
//            2 point at infinity (|w| <= 1e-12 |X|), 3 behind a camera (depth <= 0).
// fp64; HBM/latency-bound (a few hundred bytes per point).
#include "camera_model.h"
#include "sfm_internal.h"

namespace {

constexpr int UNDISTORT_ITERS = 10;
constexpr int JACOBI_SWEEPS = 10;

// Per-camera table (once per launch): R (9), t (3), centre C = -Rᵀ t (3), f, k1, pp (2) = 20.
constexpr int CAMW = 20;

__global__ __launch_bounds__(256) void tri_cam_setup(int n_cam, const double* __restrict__ cams,
                                                     const double* __restrict__ pp,
                                                     double* __restrict__ tab) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cam) return;
    const double* cam = cams + 8 * (size_t)c;
    double R[9];
    rotmat(cam[0], cam[1], cam[2], R);
    double* o = tab + CAMW * (size_t)c;
#pragma unroll
    for (int k = 0; k < 9; ++k) o[k] = R[k];
    o[9] = cam[3]; o[10] = cam[4]; o[11] = cam[5];
#pragma unroll
    for (int j = 0; j < 3; ++j) o[12 + j] = -(R[j] * cam[3] + R[3 + j] * cam[4] + R[6 + j] * cam[5]);
    o[15] = cam[6]; o[16] = cam[7];
    o[17] = pp[2 * (size_t)c]; o[18] = pp[2 * (size_t)c + 1];
    o[19] = 0.0;
}

struct View {
    double R[9], t[3];
    double x0, x1;  // undistorted normalised coordinates
};

__device__ __forceinline__ void load_view(const double* __restrict__ tab, int c, double u,
                                          double v, View& w) {
    const double* o = tab + CAMW * (size_t)c;
#pragma unroll
    for (int k = 0; k < 9; ++k) w.R[k] = o[k];
    w.t[0] = o[9]; w.t[1] = o[10]; w.t[2] = o[11];
    const double f = o[15], k1 = o[16];
    const double xd0 = (u - o[17]) / f, xd1 = (v - o[18]) / f;
    double x0 = xd0, x1 = xd1;
    for (int it = 0; it < UNDISTORT_ITERS; ++it) {
        const double s = 1.0 + k1 * (x0 * x0 + x1 * x1);
        x0 = xd0 / s;
        x1 = xd1 / s;
    }
    w.x0 = x0; w.x1 = x1;
}

// Cyclic Jacobi on a symmetric 4x4: A is destroyed, V gets the eigenvectors (columns).  Stops
// after the sweep that leaves the off-diagonal below 1e-30 of the trace (a value test: the same
// inputs stop at the same sweep).
__device__ void jacobi4(double (&A)[16], double (&V)[16]) {
#pragma unroll
    for (int k = 0; k < 16; ++k) V[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < JACOBI_SWEEPS; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) off += A[4 * p + q] * A[4 * p + q];
        const double tr = A[0] + A[5] + A[10] + A[15];
        if (off <= 1e-60 * tr * tr) break;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                const double apq = A[4 * p + q];
                if (fabs(apq) <= 1e-300) continue;
                const double app = A[4 * p + p], aqq = A[4 * q + q];
                const double theta = (aqq - app) / (2.0 * apq);
                const double tt = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
                for (int k = 0; k < 4; ++k) {  // A <- Jᵀ A J
                    const double akp = A[4 * k + p], akq = A[4 * k + q];
                    A[4 * k + p] = c * akp - s * akq;
                    A[4 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 4; ++k) {
                    const double apk = A[4 * p + k], aqk = A[4 * q + k];
                    A[4 * p + k] = c * apk - s * aqk;
                    A[4 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 4; ++k) {
                    const double vkp = V[4 * k + p], vkq = V[4 * k + q];
                    V[4 * k + p] = c * vkp - s * vkq;
                    V[4 * k + q] = s * vkp + c * vkq;
                }
            }
    }
}

__global__ __launch_bounds__(256) void triangulate_kernel(
    int n_pt, const int32_t* __restrict__ pt_ptr, const int32_t* __restrict__ cam_idx,
    const double* __restrict__ uv, const double* __restrict__ tab, double* __restrict__ pts,
    double* __restrict__ stats) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pt) return;
    const int o0 = pt_ptr[p], o1 = pt_ptr[p + 1];
    double* X = pts + 3 * (size_t)p;
    double* S = stats + 4 * (size_t)p;
    if (o1 - o0 < 2) {
        X[0] = X[1] = X[2] = 0.0;
        S[0] = 0.0; S[1] = 0.0; S[2] = 0.0; S[3] = 1.0;
        return;
    }
    double M[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) M[k] = 0.0;
    for (int o = o0; o < o1; ++o) {
        View w;
        load_view(tab, cam_idx[o], uv[2 * (size_t)o], uv[2 * (size_t)o + 1], w);
        double r0[4], r1[4];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            r0[j] = w.x0 * w.R[6 + j] - w.R[j];
            r1[j] = w.x1 * w.R[6 + j] - w.R[3 + j];
        }
        r0[3] = w.x0 * w.t[2] - w.t[0];
        r1[3] = w.x1 * w.t[2] - w.t[1];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) M[4 * i + j] += r0[i] * r0[j] + r1[i] * r1[j];
    }
    double V[16];
    jacobi4(M, V);
    int kmin = 0;
    for (int k = 1; k < 4; ++k)
        if (M[5 * k] < M[5 * kmin]) kmin = k;
    const double h0 = V[kmin], h1 = V[4 + kmin], h2 = V[8 + kmin], h3 = V[12 + kmin];
    const double nh = sqrt(h0 * h0 + h1 * h1 + h2 * h2);
    if (!(fabs(h3) > 1e-12 * nh)) {
        X[0] = X[1] = X[2] = 0.0;
        S[0] = 0.0; S[1] = 0.0; S[2] = 0.0; S[3] = 2.0;
        return;
    }
    const double x = h0 / h3, y = h1 / h3, z = h2 / h3;
    X[0] = x; X[1] = y; X[2] = z;
    // stats: reprojection error, depth, largest ray angle (rays in world frame: Rᵀ (x0, x1, 1))
    double err = 0.0, dmin = 1e300, cmax = 1.0;
    for (int o = o0; o < o1; ++o) {
        const int c = cam_idx[o];
        const double* oc = tab + CAMW * (size_t)c;
        View w;
        load_view(tab, c, uv[2 * (size_t)o], uv[2 * (size_t)o + 1], w);
        const double P0 = w.R[0] * x + w.R[1] * y + w.R[2] * z + w.t[0];
        const double P1 = w.R[3] * x + w.R[4] * y + w.R[5] * z + w.t[1];
        const double P2 = w.R[6] * x + w.R[7] * y + w.R[8] * z + w.t[2];
        dmin = fmin(dmin, P2);
        const double q0 = P0 / P2, q1 = P1 / P2;
        const double d = 1.0 + oc[16] * (q0 * q0 + q1 * q1);
        const double e0 = oc[15] * d * q0 + oc[17] - uv[2 * (size_t)o];
        const double e1 = oc[15] * d * q1 + oc[18] - uv[2 * (size_t)o + 1];
        err += sqrt(e0 * e0 + e1 * e1);
        // ray of this view (camera centre -> X) against the rays of the later views
        const double a0 = x - oc[12], a1 = y - oc[13], a2 = z - oc[14];
        const double na = sqrt(a0 * a0 + a1 * a1 + a2 * a2);
        for (int o2 = o + 1; o2 < o1; ++o2) {
            const double* c2 = tab + CAMW * (size_t)cam_idx[o2];
            const double b0 = x - c2[12], b1 = y - c2[13], b2 = z - c2[14];
            const double nb = sqrt(b0 * b0 + b1 * b1 + b2 * b2);
            cmax = fmin(cmax, (a0 * b0 + a1 * b1 + a2 * b2) / (na * nb));
        }
    }
    S[0] = err / (double)(o1 - o0);
    S[1] = acos(fmax(-1.0, fmin(1.0, cmax))) * (180.0 / 3.14159265358979323846);
    S[2] = dmin;
    S[3] = dmin > 0.0 ? 0.0 : 3.0;
}

}  // namespace

extern "C" int sfm_triangulate(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* pp,
                               int32_t n_pt, const int32_t* pt_ptr, const int32_t* cam_idx,
                               const double* uv, double* out_pts, double* out_stats) {
    SFM_REQUIRE(ctx != nullptr, "sfm_triangulate: ctx is NULL");
    SFM_REQUIRE(n_cam >= 0 && n_pt >= 0, "sfm_triangulate: negative size");
    if (n_pt == 0) return SFM_OK;
    SFM_REQUIRE(cams && pp && pt_ptr && cam_idx && uv && out_pts && out_stats,
                "sfm_triangulate: NULL array");
    SFM_REQUIRE(n_cam > 0, "sfm_triangulate: no cameras");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    double* tab = (double*)sfm::workspace(ctx, sizeof(double) * CAMW * (size_t)n_cam);
    if (!tab) return SFM_ERR_NOMEM;
    hipLaunchKernelGGL(tri_cam_setup, dim3((n_cam + 255) / 256), dim3(256), 0, ctx->stream, n_cam,
                       cams, pp, tab);
    hipLaunchKernelGGL(triangulate_kernel, dim3((n_pt + 255) / 256), dim3(256), 0, ctx->stream,
                       n_pt, pt_ptr, cam_idx, uv, tab, out_pts, out_stats);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
