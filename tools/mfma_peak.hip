// Practical ceilings on this MI355X: v_mfma_i32_32x32x32_i8 (K1) and packed f32
// FMA on the VALU (v_pk_fma_f32, K2 §4.2).  MFMA: every CU busy
// with MFMA-only waves (operands in registers, no memory in the loop), on random and on zero
// operands, 1 and 2 waves per SIMD.  Reports TOP/s against the nominal 5033 TOP/s dense-i8 peak
// and the in-kernel clock (s_memtime / s_memrealtime, MI355X_MICROARCH.md "DVFS give-back" 6).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o tools/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(const int* __restrict__ src, int iters,
                                                 int* __restrict__ out,
                                                 unsigned long long* __restrict__ stamps) {
    const int lane = threadIdx.x & 63;
    v4i a[4], b[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        a[s] = *(const v4i*)(src + 4 * ((blockIdx.x * 64 + lane * 8 + s) & 4095));
        b[s] = *(const v4i*)(src + 4 * ((blockIdx.x * 64 + lane * 8 + s + 4) & 4095));
    }
    v16i acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
    const unsigned long long t0c = __builtin_amdgcn_s_memtime(), t0r = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {  // 16 MFMAs per iteration, four accumulation chains
            acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[s], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[(s + 1) & 3], acc1, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[(s + 1) & 3], b[s], acc2, 0, 0, 0);
            acc3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[(s + 2) & 3], b[(s + 3) & 3], acc3, 0, 0, 0);
        }
    }
    const unsigned long long t1c = __builtin_amdgcn_s_memtime(), t1r = __builtin_amdgcn_s_memrealtime();
    int r = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) r += acc0[k] ^ acc1[k] ^ acc2[k] ^ acc3[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) {
        unsigned long long* d = stamps + 4 * blockIdx.x;
        d[0] = t0c; d[1] = t0r; d[2] = t1c; d[3] = t1r;
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));
// 8 independent v_pk_fma_f32 chains per lane (x = x * m + c keeps the values bounded)
__global__ __launch_bounds__(256) void pkfma_loop(const float* __restrict__ src, int iters,
                                                  float* __restrict__ out,
                                                  unsigned long long* __restrict__ stamps) {
    const int lane = threadIdx.x & 63;
    f2v x[8], m, c;
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = f2v{src[(lane * 8 + k) & 4095], src[(lane * 8 + k + 7) & 4095]};
    m = f2v{0.999f, 0.998f};
    c = f2v{src[lane & 4095] * 1e-3f, src[(lane + 1) & 4095] * 1e-3f};
    const unsigned long long t0c = __builtin_amdgcn_s_memtime(), t0r = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = __builtin_elementwise_fma(x[k], m, c);
    }
    const unsigned long long t1c = __builtin_amdgcn_s_memtime(), t1r = __builtin_amdgcn_s_memrealtime();
    float r = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) r += x[k].x + x[k].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) {
        unsigned long long* d = stamps + 4 * blockIdx.x;
        d[0] = t0c; d[1] = t0r; d[2] = t1c; d[3] = t1r;
    }
}

int main(int argc, char** argv) {
    int dev_cu = 0;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    dev_cu = prop.multiProcessorCount;
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    std::vector<int> host(4 * 4096);
    int *src, *out;
    unsigned long long* st;
    (void)hipMalloc(&src, host.size() * 4);
    (void)hipMalloc(&out, 64 * 1024 * 1024);
    (void)hipMalloc(&st, 4 * 8 * 65536);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    printf("[");
    bool first = true;
    for (int data = 0; data < 2; ++data) {  // 0: random, 1: zero
        srand(7);
        for (auto& v : host) v = data ? 0 : (int)(((unsigned)rand() << 16) ^ (unsigned)rand());
        (void)hipMemcpy(src, host.data(), host.size() * 4, hipMemcpyHostToDevice);
        for (int wps = 1; wps <= 2; ++wps) {  // waves per SIMD: blocks of 4 waves, wps per CU
            const int blocks = dev_cu * wps;
            for (int rep = 0; rep < 3; ++rep)  // warm the clock (>= 2 s of back-to-back launches)
                hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, src, iters, out, st);
            (void)hipDeviceSynchronize();
            float ms_sum = 0;
            int n = 0;
            double t_end = 0;
            (void)hipEventRecord(e0, 0);
            do {
                hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, src, iters, out, st);
                ++n;
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms_sum, e0, e1);
                t_end = ms_sum;
            } while (t_end < 2500.0);
            const double ms = t_end / n;
            std::vector<unsigned long long> s(4 * blocks);
            (void)hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
            double clk = 0;
            for (int b = 0; b < blocks; ++b)
                clk += (double)(s[4 * b + 2] - s[4 * b]) / ((double)(s[4 * b + 3] - s[4 * b + 1]) / 100e6);
            clk /= blocks;
            const double ops = 2.0 * 32 * 32 * 32 * 16.0 * iters * 4 * blocks;  // per launch
            const double tops = ops / (ms * 1e-3) / 1e12;
            printf("%s{\"data\": \"%s\", \"waves_per_simd\": %d, \"launch_ms\": %.4f, \"TOPS\": %.1f, "
                   "\"frac_of_5033\": %.4f, \"clock_GHz\": %.3f, \"frac_of_clock_peak\": %.4f}",
                   first ? "" : ", ", data ? "zero" : "random", wps, ms, tops, tops / 5033.1648,
                   clk / 1e9, tops / (2048.0 * 4 * dev_cu * clk / 1e12));
            first = false;
        }
    }
    {   // packed f32 FMA on the VALU, random operands, 2 and 8 waves per SIMD
        std::vector<float> hf(4096);
        srand(9);
        for (auto& v : hf) v = (float)rand() / RAND_MAX;
        float* fsrc;
        (void)hipMalloc(&fsrc, hf.size() * 4);
        (void)hipMemcpy(fsrc, hf.data(), hf.size() * 4, hipMemcpyHostToDevice);
        const int fit = iters * 2;
        for (int wps : {2, 8}) {
            const int blocks = dev_cu * wps;
            for (int rep = 0; rep < 3; ++rep)
                hipLaunchKernelGGL(pkfma_loop, dim3(blocks), dim3(256), 0, 0, fsrc, fit, (float*)out, st);
            (void)hipDeviceSynchronize();
            float ms_sum = 0;
            int n = 0;
            (void)hipEventRecord(e0, 0);
            do {
                hipLaunchKernelGGL(pkfma_loop, dim3(blocks), dim3(256), 0, 0, fsrc, fit, (float*)out, st);
                ++n;
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms_sum, e0, e1);
            } while (ms_sum < 2500.0);
            const double ms = ms_sum / n;
            std::vector<unsigned long long> s(4 * blocks);
            (void)hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
            double clk = 0;
            for (int b = 0; b < blocks; ++b)
                clk += (double)(s[4 * b + 2] - s[4 * b]) / ((double)(s[4 * b + 3] - s[4 * b + 1]) / 100e6);
            clk /= blocks;
            const double flops = 4.0 * 16 * 8 * (double)fit * 256 * blocks;  // 2 fma x 2 flop per pk
            const double tf = flops / (ms * 1e-3) / 1e12;
            printf(", {\"op\": \"v_pk_fma_f32\", \"waves_per_simd\": %d, \"launch_ms\": %.4f, "
                   "\"TFLOPS\": %.1f, \"frac_of_157.3\": %.4f, \"clock_GHz\": %.3f}",
                   wps, ms, tf, tf / 157.3, clk / 1e9);
        }
    }
    printf("]\n");
    return 0;
}
