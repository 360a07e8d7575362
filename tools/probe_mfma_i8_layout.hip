// Probe of v_mfma_i32_32x32x32_i8 on gfx950 (ham_key_kernel's extra k-step):
//   T1 random operands: which k does byte p of lane l feed, for A and for B (host-side check of
//      the hypothesis lane l supplies A[l%32][16*(l/32) + p] and B[16*(l/32) + p][l%32]);
//   T2 the extra step as ham_key_kernel builds it (A = eight 64s and a 1 in the lane-half-0
//      bytes; B = eight digits of -2 n and 127 - q): D must be -128 n + 127 - q in every row.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mfma_i8_layout.hip -o tools/probe_mfma_i8_layout
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void t1(const int* A, const int* B, int* D) {
    const int l = threadIdx.x;
    v4i a = {A[l * 4], A[l * 4 + 1], A[l * 4 + 2], A[l * 4 + 3]};
    v4i b = {B[l * 4], B[l * 4 + 1], B[l * 4 + 2], B[l * 4 + 3]};
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = c[r];
}

__global__ void t2(int* D) {
    const int l = threadIdx.x, h = l >> 5, q = l & 31;
    const int n = 3 * q + 1;  // a query's popcount
    const int m = 2 * n;
    unsigned w0 = 0, w1 = 0;
    for (int t = 0; t < 8; ++t) {
        const int dgt = -min(max(m - 128 * t, 0), 128);
        const unsigned byte = (unsigned)(dgt & 0xFF);
        if (t < 4) w0 |= byte << (8 * t); else w1 |= byte << (8 * (t - 4));
    }
    const v4i ax = h ? v4i{0, 0, 0, 0} : v4i{0x40404040, 0x40404040, 1, 0};
    const v4i bx = h ? v4i{0, 0, 0, 0} : v4i{(int)w0, (int)w1, 127 - q, 0};
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(ax, bx, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = c[r];
}

int main() {
    std::vector<int> A(256), B(256), D(1024);
    srand(7);
    std::vector<signed char> ab(1024), bb(1024);
    for (int i = 0; i < 1024; ++i) { ab[i] = (signed char)(rand() % 7 - 3); bb[i] = (signed char)(rand() % 7 - 3); }
    memcpy(A.data(), ab.data(), 1024);
    memcpy(B.data(), bb.data(), 1024);
    int *dA, *dB, *dD;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 4096);
    hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(t1, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
    // hypothesis: A[m][k] = ab[(m + 32*(k/16))*16 + k%16], B[k][n] = bb[(n + 32*(k/16))*16 + k%16],
    // D register r of lane l = C[8*(r/4) + 4*(l/32) + r%4][l%32]
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int m = 8 * (r / 4) + 4 * (l / 32) + r % 4, n = l % 32;
            int s = 0;
            for (int k = 0; k < 32; ++k)
                s += ab[(m + 32 * (k / 16)) * 16 + k % 16] * bb[(n + 32 * (k / 16)) * 16 + k % 16];
            bad += s != D[l * 16 + r];
        }
    printf("T1 layout hypothesis (lane l: row/col l%%32, k = 16*(l/32) + byte): %d of 1024 outputs differ\n", bad);
    printf("T1 raw D lane 0 r 0..3: %d %d %d %d\n", D[0], D[1], D[2], D[3]);
    hipLaunchKernelGGL(t2, dim3(1), dim3(64), 0, 0, dD);
    hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
    bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int n = 3 * (l % 32) + 1, want = -128 * n + 127 - (l % 32);
            if (D[l * 16 + r] != want && bad++ < 8)
                printf("T2 lane %d r %d: got %d want %d\n", l, r, D[l * 16 + r], want);
        }
    printf("T2 extra k-step: %d of 1024 outputs differ\n", bad);
    return 0;
}
