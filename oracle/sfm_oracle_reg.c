/*
 * sfm_oracle_reg.c — CPU restatement of next-view registration (P3P RANSAC), the last step of
 * incremental SfM listed in SURVEY.md §8f item 3.  TEST INFRASTRUCTURE ONLY (see sfm_oracle.c).
 *
 * The reference has no code for it (code/3d_reconstruction.py is empty); this is the build's spec
 * (DESIGN.md §4.8), mirrored op-for-op by sfm-project_amd/csrc/register.hip.  Only +, -, *, /
 * and sqrt (all correctly rounded) appear in the RANSAC part and both sides are built without FMA
 * contraction, so hypotheses, counts, the best hypothesis and the inlier mask are bit-identical.
 *
 *   bearing   x_d = (xy - c) / f; 10 fixed-point undistortion steps x = x_d / (1 + k1 |x|^2);
 *             b = (x0, x1, 1) / |(x0, x1, 1)|
 *   sample    Philox4x32-10, key = seed, counter (h, 2, image, 0x52454731); Floyd, 3 indices
 *   P3P       Grunert's quartic in v = s3/s1 (Haralick et al. 1994), roots by 48 Durand-Kerner
 *             iterations from R (0.4 + 0.9i)^k, R = 1 + max |a_i / a_4|; real if
 *             |Im| <= 1e-7 (1 + |Re|), then 2 Newton steps; per real root k: u, s1..s3 > 0,
 *             camera-frame points s_i b_i, pose by aligning the two point triangles' frames
 *   score     inlier iff depth > 0 and |f (1 + k1 |q|^2) q + c - xy|^2 < thr^2
 *   best      max count, ties -> lowest 4 h + k
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]);

#define REG_UNDISTORT 10
#define REG_DK_ITERS 48

void oracle_reg_bearing(double x, double y, const double intr[4], double b[3]) {
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

void oracle_reg_sample3(uint64_t seed, uint32_t img, uint32_t h, int n, int32_t out[3]) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {h, 2u, img, 0x52454731u}, r[4];
    oracle_philox4x32_10(ctr, key, r);
    for (int k = 0; k < 3; ++k) {
        uint32_t jmax = (uint32_t)(n - 3 + k);
        uint32_t t = (uint32_t)(((uint64_t)r[k] * (uint64_t)(jmax + 1u)) >> 32);
        for (int q = 0; q < k; ++q)
            if ((uint32_t)out[q] == t) { t = jmax; break; }
        out[k] = (int32_t)t;
    }
}

static void cmul(double a, double b, double c, double d, double* re, double* im) {
    *re = a * c - b * d;
    *im = a * d + b * c;
}
static void cdiv(double a, double b, double c, double d, double* re, double* im) {
    const double den = c * c + d * d;
    *re = (a * c + b * d) / den;
    *im = (b * c - a * d) / den;
}

/* Roots of z^4 + c3 z^3 + c2 z^2 + c1 z + c0 (Durand-Kerner); re/im [4]. */
static void dk_roots(const double c[4], double re[4], double im[4]) {
    double R = 1.0;
    for (int i = 0; i < 4; ++i) R = fmax(R, 1.0 + fabs(c[i]));
    double wr = 1.0, wi = 0.0;
    for (int k = 0; k < 4; ++k) {  /* R (0.4 + 0.9i)^k */
        re[k] = R * wr; im[k] = R * wi;
        double tr, ti;
        cmul(wr, wi, 0.4, 0.9, &tr, &ti);
        wr = tr; wi = ti;
    }
    for (int it = 0; it < REG_DK_ITERS; ++it) {
        for (int k = 0; k < 4; ++k) {
            /* p(z) by Horner */
            double pr = 1.0, pi = 0.0;
            for (int i = 3; i >= 0; --i) {
                double tr, ti;
                cmul(pr, pi, re[k], im[k], &tr, &ti);
                pr = tr + c[i]; pi = ti;
            }
            double qr = 1.0, qi = 0.0;
            for (int j = 0; j < 4; ++j) {
                if (j == k) continue;
                double tr, ti;
                cmul(qr, qi, re[k] - re[j], im[k] - im[j], &tr, &ti);
                qr = tr; qi = ti;
            }
            if (qr == 0.0 && qi == 0.0) continue;
            double dr, di;
            cdiv(pr, pi, qr, qi, &dr, &di);
            re[k] = re[k] - dr;
            im[k] = im[k] - di;
        }
    }
}

/* Orthonormal frame of a point triangle (columns e1, e2, e3), row-major F[3][3]. */
static int tri_frame(const double X[3][3], double F[9]) {
    double e1[3] = {X[1][0] - X[0][0], X[1][1] - X[0][1], X[1][2] - X[0][2]};
    double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    if (!(n1 > 0.0)) return 0;
    e1[0] = e1[0] / n1; e1[1] = e1[1] / n1; e1[2] = e1[2] / n1;
    const double d[3] = {X[2][0] - X[0][0], X[2][1] - X[0][1], X[2][2] - X[0][2]};
    double e3[3] = {e1[1] * d[2] - e1[2] * d[1], e1[2] * d[0] - e1[0] * d[2],
                    e1[0] * d[1] - e1[1] * d[0]};
    double n3 = sqrt(e3[0] * e3[0] + e3[1] * e3[1] + e3[2] * e3[2]);
    if (!(n3 > 0.0)) return 0;
    e3[0] = e3[0] / n3; e3[1] = e3[1] / n3; e3[2] = e3[2] / n3;
    const double e2[3] = {e3[1] * e1[2] - e3[2] * e1[1], e3[2] * e1[0] - e3[0] * e1[2],
                          e3[0] * e1[1] - e3[1] * e1[0]};
    for (int i = 0; i < 3; ++i) { F[3 * i] = e1[i]; F[3 * i + 1] = e2[i]; F[3 * i + 2] = e3[i]; }
    return 1;
}

/* P3P: bearings b[3][3], world points X[3][3] -> up to 4 poses (R row-major, t); ok[k] marks the
 * valid root slots.  Returns the number of valid poses. */
int oracle_reg_p3p(const double b[3][3], const double X[3][3], double Rs[4][9], double ts[4][3],
                   int ok[4]) {
    for (int k = 0; k < 4; ++k) ok[k] = 0;
    double dx, dy, dz;
    dx = X[1][0] - X[2][0]; dy = X[1][1] - X[2][1]; dz = X[1][2] - X[2][2];
    const double a2 = dx * dx + dy * dy + dz * dz;
    dx = X[0][0] - X[2][0]; dy = X[0][1] - X[2][1]; dz = X[0][2] - X[2][2];
    const double b2 = dx * dx + dy * dy + dz * dz;
    dx = X[0][0] - X[1][0]; dy = X[0][1] - X[1][1]; dz = X[0][2] - X[1][2];
    const double c2 = dx * dx + dy * dy + dz * dz;
    if (!(b2 > 0.0)) return 0;
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
    double amax = fmax(fmax(fabs(A3), fabs(A2)), fmax(fabs(A1), fabs(A0)));
    if (!(fabs(A4) > 1e-12 * amax)) return 0;
    const double c[4] = {A0 / A4, A1 / A4, A2 / A4, A3 / A4};
    double re[4], im[4];
    dk_roots(c, re, im);
    double FP[9];
    if (!tri_frame(X, FP)) return 0;
    int n = 0;
    for (int k = 0; k < 4; ++k) {
        if (!(fabs(im[k]) <= 1e-7 * (1.0 + fabs(re[k])))) continue;
        double v = re[k];
        for (int it = 0; it < 2; ++it) {  /* Newton on the real quartic */
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
        ok[k] = 1;
        ++n;
    }
    return n;
}

/* Inlier test of one correspondence under a pose (R row-major, t). */
int oracle_reg_inlier(const double R[9], const double t[3], const double intr[4], double x,
                      double y, const double X[3], double thr2) {
    const double P0 = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
    const double P1 = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
    const double P2 = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
    if (!(P2 > 0.0)) return 0;
    const double q0 = P0 / P2, q1 = P1 / P2;
    const double d = 1.0 + intr[1] * (q0 * q0 + q1 * q1);
    const double e0 = intr[0] * d * q0 + intr[2] - x;
    const double e1 = intr[0] * d * q1 + intr[3] - y;
    return (e0 * e0 + e1 * e1) < thr2;
}

/* RANSAC over n_hyp hypotheses for one image.  Returns the best inlier count (-1: no pose);
 * best_key = 4 h + k of the winner; R, t its pose; mask [n] its inliers. */
int oracle_reg_ransac(int n, const double* xy, const double* X, const double intr[4],
                      uint32_t img, int n_hyp, uint64_t seed, double thr, int32_t* best_key,
                      double R_out[9], double t_out[3], uint8_t* mask) {
    const double thr2 = thr * thr;
    int best = -1;
    int32_t bkey = -1;
    double bR[9] = {0}, bt[3] = {0};
    if (n >= 3) {
        for (int h = 0; h < n_hyp; ++h) {
            int32_t idx[3];
            oracle_reg_sample3(seed, img, (uint32_t)h, n, idx);
            double b[3][3], Xs[3][3];
            for (int i = 0; i < 3; ++i) {
                oracle_reg_bearing(xy[2 * idx[i]], xy[2 * idx[i] + 1], intr, b[i]);
                for (int j = 0; j < 3; ++j) Xs[i][j] = X[3 * idx[i] + j];
            }
            double Rs[4][9], ts[4][3];
            int ok[4];
            oracle_reg_p3p(b, Xs, Rs, ts, ok);
            for (int k = 0; k < 4; ++k) {
                if (!ok[k]) continue;
                int cnt = 0;
                for (int m = 0; m < n; ++m)
                    cnt += oracle_reg_inlier(Rs[k], ts[k], intr, xy[2 * m], xy[2 * m + 1],
                                             X + 3 * m, thr2);
                if (cnt > best) {  /* ascending (h, k): strict > keeps the lowest key on ties */
                    best = cnt;
                    bkey = 4 * h + k;
                    memcpy(bR, Rs[k], sizeof bR);
                    memcpy(bt, ts[k], sizeof bt);
                }
            }
        }
    }
    *best_key = bkey;
    memcpy(R_out, bR, sizeof bR);
    memcpy(t_out, bt, sizeof bt);
    for (int m = 0; m < n; ++m)
        mask[m] = best >= 0 ? (uint8_t)oracle_reg_inlier(bR, bt, intr, xy[2 * m], xy[2 * m + 1],
                                                         X + 3 * m, thr2)
                            : 0;
    return best;
}
