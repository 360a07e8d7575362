// Device camera model shared by the BA and triangulation kernels:
// angle-axis rotation r (3), translation t (3), focal f, radial k1; principal point fixed.
//   pred = f (1 + k1 |p|^2) p + pp,  p = (P0/P2, P1/P2),  P = R(r) X + t.
// Mirrors oracle/sfm_oracle_ba.c (oracle_ba_obs) and oracle/ba_lm.py (_rotmat).
#pragma once
#include <hip/hip_runtime.h>

// Rodrigues; first-order form below |r|^2 = 1e-20 (as the oracle).
__device__ __forceinline__ void rotmat(double r0v, double r1v, double r2v, double (&R)[9]) {
    const double th2 = r0v * r0v + r1v * r1v + r2v * r2v;
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
}
