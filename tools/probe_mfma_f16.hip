// Probe of v_mfma_f32_32x32x16_f16 on gfx950 (the certified MFMA Sampson filter):
//   1. operand layout: lane l supplies A[l%32][8*(l/32) + e] and B[8*(l/32) + e][l%32] (e = 0..7),
//      accumulator register r of lane l is C[8*(r/4) + 4*(l/32) + r%4][l%32];
//   2. f16 subnormal inputs: kept or flushed;
//   3. accumulation error of 16 exact products against an fp64 sum, in units of 2^-24 * sum|p|.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mfma_f16.hip -o tools/probe_mfma_f16
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A, B as [64 lanes][8] f16 in the lane layout; C out as [64 lanes][16]
__global__ void mfma_once(const _Float16* A, const _Float16* B, float* C, int n) {
    const int l = threadIdx.x;
    for (int t = 0; t < n; ++t) {
        h8 a, b;
        for (int e = 0; e < 8; ++e) {
            a[e] = A[(size_t)t * 512 + l * 8 + e];
            b[e] = B[(size_t)t * 512 + l * 8 + e];
        }
        f16v c = {};
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
        for (int r = 0; r < 16; ++r) C[(size_t)t * 1024 + l * 16 + r] = c[r];
    }
}

static void run(std::vector<_Float16>& A, std::vector<_Float16>& B, std::vector<float>& C, int n) {
    _Float16 *dA, *dB;
    float* dC;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, C.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_once, dim3(1), dim3(64), 0, 0, dA, dB, dC, n);
    hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
    hipFree(dA); hipFree(dB); hipFree(dC);
}

// logical A[i][k], B[k][j] -> lane layout
static void pack(const double* Al, const double* Bl, _Float16* A, _Float16* B) {
    for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e) {
            const int k = 8 * (l / 32) + e;
            A[l * 8 + e] = (_Float16)Al[(l % 32) * 16 + k];
            B[l * 8 + e] = (_Float16)Bl[k * 32 + (l % 32)];
        }
}
static double cval(const float* C, int i, int j) {  // register r of lane l holds row 8(r/4)+4(l/32)+r%4
    const int l = j + 32 * ((i / 4) % 2), r = 4 * (i / 8) + i % 4;
    return C[l * 16 + r];
}

int main() {
    // 1. layout: one k slot at a time
    int bad = 0;
    {
        const int n = 16;
        std::vector<_Float16> A(n * 512), B(n * 512);
        std::vector<float> C(n * 1024);
        for (int k0 = 0; k0 < 16; ++k0) {
            double Al[32 * 16] = {}, Bl[16 * 32] = {};
            for (int i = 0; i < 32; ++i) Al[i * 16 + k0] = i + 1;
            for (int j = 0; j < 32; ++j) Bl[k0 * 32 + j] = j + 1;
            pack(Al, Bl, &A[k0 * 512], &B[k0 * 512]);
        }
        run(A, B, C, n);
        for (int k0 = 0; k0 < 16; ++k0)
            for (int i = 0; i < 32; ++i)
                for (int j = 0; j < 32; ++j)
                    if (cval(&C[k0 * 1024], i, j) != (double)(i + 1) * (j + 1)) ++bad;
        printf("{\"layout_mismatches\": %d", bad);
    }
    // 2. subnormal f16 inputs: 2^-20 * 2^10, and a subnormal * subnormal product
    {
        std::vector<_Float16> A(512), B(512);
        std::vector<float> C(1024);
        double Al[32 * 16] = {}, Bl[16 * 32] = {};
        Al[0 * 16 + 0] = std::ldexp(1.0, -20); Bl[0 * 32 + 0] = 1024.0;    // C[0][0] = 2^-10
        Al[1 * 16 + 3] = std::ldexp(3.0, -24); Bl[3 * 32 + 1] = 2048.0;    // C[1][1] = 3*2^-13
        Al[2 * 16 + 5] = 1.0; Bl[5 * 32 + 2] = std::ldexp(5.0, -24);      // C[2][2] = 5*2^-24
        pack(Al, Bl, A.data(), B.data());
        run(A, B, C, 1);
        printf(", \"subnormal_a\": %.9g, \"expect_a\": %.9g, \"subnormal_b\": %.9g, \"expect_b\": %.9g, "
               "\"subnormal_c\": %.9g, \"expect_c\": %.9g",
               cval(C.data(), 0, 0), std::ldexp(1.0, -10), cval(C.data(), 1, 1),
               std::ldexp(3.0, -13), cval(C.data(), 2, 2), std::ldexp(5.0, -24));
    }
    // 3. accumulation error: random f16 operands with mixed exponents and signs
    {
        const int n = 512;
        std::vector<_Float16> A(n * 512), B(n * 512);
        std::vector<float> C(n * 1024);
        std::vector<double> Al(n * 512), Bl(n * 512);
        srand(12345);
        auto rnd = [](int emin, int emax) {
            const double m = 1.0 + (rand() % 1024) / 1024.0;
            const int e = emin + rand() % (emax - emin + 1);
            return (rand() & 1 ? -1.0 : 1.0) * std::ldexp(m, e);
        };
        for (int t = 0; t < n; ++t) {
            const int mode = t % 4;  // 0: wide exponents, 1: narrow, 2: cancelling pairs, 3: hi/lo split
            for (int i = 0; i < 32; ++i)
                for (int k = 0; k < 16; ++k) {
                    double v = mode == 0 ? rnd(-12, 12) : rnd(-2, 2);
                    if (mode == 3) v = (k & 1) ? std::ldexp(rnd(0, 0), -11) : rnd(4, 6);
                    Al[t * 512 + i * 16 + k] = (double)(_Float16)v;
                }
            for (int k = 0; k < 16; ++k)
                for (int j = 0; j < 32; ++j) {
                    double v = mode == 0 ? rnd(-12, 12) : rnd(-2, 2);
                    if (mode == 2 && (k & 1)) v = -Bl[t * 512 + (k - 1) * 32 + j] * (1 + 1.0 / 1024);
                    if (mode == 3) v = (k & 2) ? std::ldexp(rnd(0, 0), -11) : rnd(4, 6);
                    Bl[t * 512 + k * 32 + j] = (double)(_Float16)v;
                }
            pack(&Al[t * 512], &Bl[t * 512], &A[t * 512], &B[t * 512]);
        }
        run(A, B, C, n);
        double worst = 0, worst_rel_sum = 0;
        long exact = 0, total = 0;
        for (int t = 0; t < n; ++t)
            for (int i = 0; i < 32; ++i)
                for (int j = 0; j < 32; ++j) {
                    double s = 0, sa = 0;
                    for (int k = 0; k < 16; ++k) {
                        const double p = Al[t * 512 + i * 16 + k] * Bl[t * 512 + k * 32 + j];
                        s += p;
                        sa += std::fabs(p);
                    }
                    const double c = cval(&C[t * 1024], i, j);
                    const double err = std::fabs(c - s);
                    const double rel = sa > 0 ? err / (sa * std::ldexp(1.0, -24)) : 0;
                    if (rel > worst) worst = rel;
                    if (err == std::fabs((double)(float)s - s)) ++exact;
                    ++total;
                    (void)worst_rel_sum;
                }
        printf(", \"accum_err_max_units_2m24_sumabs\": %.4f, \"correctly_rounded_frac\": %.5f}\n", worst,
               (double)exact / total);
    }
    return bad ? 1 : 0;
}
