// Microbenchmark: VALU issue rate per SIMD on gfx950 for the instruction mixes the kernels use,
// and MFMA/VALU co-issue.  8 independent chains per thread; cycles per wave-instruction per SIMD
// at nominal 2.4 GHz (= elapsed * 2.4e9 * n_simd / wave_instructions).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef short s2 __attribute__((ext_vector_type(2)));
#define ITERS 2048

__device__ __forceinline__ int med3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

template <int K>
__global__ __launch_bounds__(256) void kern(int* out, int seed) {
    float a[8]; f2 b[8]; int c[8], x[8], y[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 0.001f + i; b[i] = f2{a[i], a[i] + 1}; c[i] = threadIdx.x + i * seed;
        x[i] = __builtin_amdgcn_readfirstlane(seed * (i + 7)); y[i] = threadIdx.x ^ (i * 77);
    }
    v16i acc0 = {0}, acc1 = {0};
    v4i av = {seed, seed + 1, seed + 2, (int)threadIdx.x}, bv = {seed * 3, 5, 7, (int)threadIdx.x};
    const float m = 1.0001f, q = 0.9999f;
    for (int it = 0; it < ITERS; ++it) {
        if constexpr (K == 9 || K == 10) {
            acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc1, 0, 0, 0);
            asm volatile("" : "+v"(av), "+v"(bv));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (K == 0) a[i] = __builtin_fmaf(a[i], m, q);
            if constexpr (K == 1) b[i] = __builtin_elementwise_fma(b[i], f2{m, m}, f2{q, q});
            if constexpr (K == 2) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 3) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 4) asm volatile("v_lshl_add_u32 %0, %0, 9, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 5) asm volatile("v_max_i32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(c[i]));
            if constexpr (K == 6) asm volatile("v_max_i32 %0, %0, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 7) asm volatile("v_add_u32 %0, %0, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 8) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 11) asm volatile("v_max_f32 %0, %0, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 12) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 13) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 14) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 15) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 16) asm volatile("v_mad_i32_i24 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 17) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 18) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 19) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(c[i]));
            if constexpr (K == 20) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i+1)&7]));
            if constexpr (K == 21) asm volatile("v_max_u32 %0, %0, %1" : "+v"(c[i]) : "v"(y[i]));
            if constexpr (K == 22) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 23) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(c[i]), "+v"(y[i]));
            if constexpr (K == 24) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
            if constexpr (K == 10) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x[i]), "v"(y[i]));
        }
    }
    int s = 0;
    for (int i = 0; i < 8; ++i) s += (int)a[i] + (int)b[i].x + (int)b[i].y + c[i];
    for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int* out; (void)hipMalloc(&out, 256 * 1024 * 4 * 8);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_max3_i32", "v_med3_i32", "v_lshl_add_u32",
                           "v_max_i32_dpp", "v_max_i32", "v_add_u32", "v_pk_max_i16",
                           "mfma_i8 x2 only", "mfma_i8 x2 + 8 max3", "v_max_f32", "v_max3_f32", "v_med3_f32", "v_sub_f32", "v_cndmask_b32", "v_mad_i32_i24", "v_add3_u32", "v_xor_b32", "v_cvt_f32_i32", "v_pk_add_f32", "v_max_u32", "v_min3_f32", "v_permlane16_swap_b32", "v_perm_b32"};
    for (int wps : {4}) {
        for (int k = 0; k < 25; ++k) {
            dim3 grid(256 * wps), block(256);
            auto launch = [&]() {
                switch (k) {
#define L(n) case n: kern<n><<<grid, block>>>(out, 3); break;
                    L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18) L(19) L(20) L(21) L(22) L(23) L(24)
                }
            };
            launch(); (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0); for (int r = 0; r < 5; ++r) launch(); (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 5;
            double waves = 256.0 * wps * 4;
            double per_iter = (k >= 9) ? 2.0 : 8.0;     // MFMA rows: cycles per MFMA instruction
            double cyc = ms * 1e-3 * 2.4e9 * 1024 / (waves * ITERS * per_iter);
            printf("waves/SIMD %d  %-22s  %.3f ms  %.2f cycles/instr/SIMD\n", wps, names[k], ms, cyc);
        }
    }
    return 0;
}
