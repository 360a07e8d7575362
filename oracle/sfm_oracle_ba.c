/*
 * sfm_oracle_ba.c — CPU restatement of the bundle-adjustment linearisation (J^TJ build).
 *
 * TEST INFRASTRUCTURE ONLY (see sfm_oracle.c header).  Fills the slot of the empty reference file
 * code/3d_reconstruction.py (import commented out at code/pipeline.py:4) with the objective of the
 * bundled paper papers/schoenberger2016sfm.pdf eq. (1) / §4.4 as specified in SURVEY.md §8a row a7:
 *   camera = angle-axis r (3), translation t (3), focal f, radial k1; principal point fixed;
 *   pred = f * (1 + k1*|p|^2) * p + pp,  p = (P0/P2, P1/P2),  P = R(r) X + t;
 *   residual = pred - uv; optional Cauchy loss rho(e) = s^2 log(1 + e/s^2) applied as an IRLS weight.
 * The rotation Jacobian is taken w.r.t. a left-multiplied increment R <- exp([d]x) R (the tangent
 * space an LM step on SO(3) updates), so dP/dd = -[R X]x.
 * Accumulates U_c = sum w J_c^T J_c (8x8), V_p = sum w J_p^T J_p (3x3), W_o = w J_c^T J_p (8x3),
 * g_c = sum w J_c^T r, g_p = sum w J_p^T r, cost = 0.5 sum rho(e).
 * fp64 throughout; parity against the GPU is tolerance-based (reduction order differs).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

void oracle_ba_obs(const double* cam, const double* pp, const double* X, const double* uv,
                   double loss_s, double r_out[2], double Jc[16], double Jp[6], double* w_out,
                   double* rho_out) {
    const double* rv = cam;
    double th2 = rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2];
    double R[9];
    if (th2 > 1e-20) {
        double th = sqrt(th2), c = cos(th), s = sin(th), C = 1.0 - c;
        double kx = rv[0] / th, ky = rv[1] / th, kz = rv[2] / th;
        R[0] = c + C * kx * kx;      R[1] = C * kx * ky - s * kz; R[2] = C * kx * kz + s * ky;
        R[3] = C * ky * kx + s * kz; R[4] = c + C * ky * ky;      R[5] = C * ky * kz - s * kx;
        R[6] = C * kz * kx - s * ky; R[7] = C * kz * ky + s * kx; R[8] = c + C * kz * kz;
    } else {
        R[0] = 1.0;    R[1] = -rv[2]; R[2] = rv[1];
        R[3] = rv[2];  R[4] = 1.0;    R[5] = -rv[0];
        R[6] = -rv[1]; R[7] = rv[0];  R[8] = 1.0;
    }
    double Y[3], P[3];
    for (int i = 0; i < 3; ++i) {
        Y[i] = R[3 * i] * X[0] + R[3 * i + 1] * X[1] + R[3 * i + 2] * X[2];
        P[i] = Y[i] + cam[3 + i];
    }
    double iz = 1.0 / P[2];
    double p0 = P[0] * iz, p1 = P[1] * iz;
    double f = cam[6], k1 = cam[7];
    double rho2 = p0 * p0 + p1 * p1;
    double d = 1.0 + k1 * rho2;
    double r0 = f * d * p0 + pp[0] - uv[0];
    double r1 = f * d * p1 + pp[1] - uv[1];
    double e = r0 * r0 + r1 * r1;
    double w = 1.0, rho = e;
    if (loss_s > 0.0) {
        double s2 = loss_s * loss_s;
        w = 1.0 / (1.0 + e / s2);
        rho = s2 * log1p(e / s2);
    }
    /* M = dpred/dp, D = dp/dP, A = M D */
    double m00 = f * (d + 2.0 * k1 * p0 * p0), m01 = f * (2.0 * k1 * p0 * p1);
    double m11 = f * (d + 2.0 * k1 * p1 * p1);
    double D[2][3] = {{iz, 0.0, -p0 * iz}, {0.0, iz, -p1 * iz}};
    double A[2][3];
    for (int j = 0; j < 3; ++j) {
        A[0][j] = m00 * D[0][j] + m01 * D[1][j];
        A[1][j] = m01 * D[0][j] + m11 * D[1][j];
    }
    /* -[Y]x */
    double S[3][3] = {{0.0, Y[2], -Y[1]}, {-Y[2], 0.0, Y[0]}, {Y[1], -Y[0], 0.0}};
    for (int a = 0; a < 2; ++a) {
        for (int j = 0; j < 3; ++j) {
            Jc[8 * a + j] = A[a][0] * S[0][j] + A[a][1] * S[1][j] + A[a][2] * S[2][j];
            Jc[8 * a + 3 + j] = A[a][j];
            Jp[3 * a + j] = A[a][0] * R[j] + A[a][1] * R[3 + j] + A[a][2] * R[6 + j];
        }
    }
    Jc[6] = d * p0;            Jc[14] = d * p1;
    Jc[7] = f * rho2 * p0;     Jc[15] = f * rho2 * p1;
    r_out[0] = r0; r_out[1] = r1;
    *w_out = w; *rho_out = rho;
}

/* Builds U [n_cam][8][8], V [n_pt][3][3], W [n_obs][8][3], gc [n_cam][8], gp [n_pt][3],
 * res [n_obs][2]; returns cost.  Output arrays are overwritten. */
double oracle_ba_jtj(int n_cam, const double* cams, const double* pp, int n_pt, const double* pts,
                     int n_obs, const int32_t* cam_idx, const int32_t* pt_idx, const double* uv,
                     double loss_s, double* U, double* V, double* W, double* gc, double* gp,
                     double* res) {
    memset(U, 0, sizeof(double) * 64 * (size_t)n_cam);
    memset(V, 0, sizeof(double) * 9 * (size_t)n_pt);
    memset(gc, 0, sizeof(double) * 8 * (size_t)n_cam);
    memset(gp, 0, sizeof(double) * 3 * (size_t)n_pt);
    double cost = 0.0;
    for (int o = 0; o < n_obs; ++o) {
        int c = cam_idx[o], p = pt_idx[o];
        double r[2], Jc[16], Jp[6], w, rho;
        oracle_ba_obs(cams + 8 * (size_t)c, pp + 2 * (size_t)c, pts + 3 * (size_t)p,
                      uv + 2 * (size_t)o, loss_s, r, Jc, Jp, &w, &rho);
        cost += 0.5 * rho;
        res[2 * o] = r[0]; res[2 * o + 1] = r[1];
        double* Uc = U + 64 * (size_t)c;
        for (int i = 0; i < 8; ++i) {
            for (int j = 0; j < 8; ++j) Uc[8 * i + j] += w * (Jc[i] * Jc[j] + Jc[8 + i] * Jc[8 + j]);
            gc[8 * (size_t)c + i] += w * (Jc[i] * r[0] + Jc[8 + i] * r[1]);
            for (int j = 0; j < 3; ++j)
                W[24 * (size_t)o + 3 * i + j] = w * (Jc[i] * Jp[j] + Jc[8 + i] * Jp[3 + j]);
        }
        double* Vp = V + 9 * (size_t)p;
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) Vp[3 * i + j] += w * (Jp[i] * Jp[j] + Jp[3 + i] * Jp[3 + j]);
            gp[3 * (size_t)p + i] += w * (Jp[i] * r[0] + Jp[3 + i] * r[1]);
        }
    }
    return cost;
}
