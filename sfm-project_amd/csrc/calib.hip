// Calibration probe: what this device's i8 matrix pipe sustains right now.
//
// Box-to-box variance is real on this pool (MI355X_MICROARCH.md "DVFS give-back" 5: one binary
// 12 % apart across devices; BENCH_r05's K1 stage ran 11 % slower than the builder's box with no
// code change).  The bench line carries this probe, run in the same process right before the
// timed steps, so a K1 number can be read against the ceiling of the box it ran on rather than a
// constant: every CU runs MFMA-only waves (v_mfma_i32_32x32x32_i8, operands in registers, random
// data, four accumulation chains, no memory in the loop), two waves per SIMD as K1's scans run,
// for about the requested wall time; the in-kernel clock is the median over blocks of
// delta s_memtime / delta s_memrealtime x 100 MHz (MI355X_MICROARCH.md "DVFS give-back" 6).
#include <algorithm>
#include <vector>

#include "sfm_internal.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void calib_mfma_i8_kernel(int iters, unsigned seed,
                                                            int* __restrict__ sink,
                                                            unsigned long long* __restrict__ stamps) {
    const int lane = threadIdx.x & 63;
    v4i a[4], b[4];
    unsigned x = seed ^ (blockIdx.x * 2654435761u) ^ (threadIdx.x * 40503u);
#pragma unroll
    for (int s = 0; s < 4; ++s) {   // random i8 operands (xorshift), different per lane
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            a[s][k] = (int)x;
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            b[s][k] = (int)(x ^ (unsigned)lane);
        }
    }
    v16i acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
    const unsigned long long t0c = __builtin_amdgcn_s_memtime(), t0r = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {  // 16 MFMAs per iteration
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
    sink[blockIdx.x * blockDim.x + threadIdx.x] = r;   // keeps the MFMAs live
    if (threadIdx.x == 0) {
        unsigned long long* d = stamps + 4 * blockIdx.x;
        d[0] = t0c; d[1] = t0r; d[2] = t1c; d[3] = t1r;
    }
}

}  // namespace

// out[0] wall ms of the measured launch, out[1] i8 TOP/s, out[2] median in-kernel clock GHz,
// out[3] fraction of the nominal dense-i8 peak (2048 op/clk/SIMD x 4 x n_cu x 2.4 GHz).
extern "C" int sfm_calib_mfma_i8(sfm_ctx* ctx, float target_ms, double* out) {
    SFM_REQUIRE(ctx && out, "sfm_calib_mfma_i8: ctx/out is NULL");
    SFM_REQUIRE(target_ms > 0.0f && target_ms <= 5000.0f,
                "sfm_calib_mfma_i8: target_ms must be in (0, 5000]");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int blocks = 2 * ctx->n_cu;   // 4 waves per block, two blocks per CU: 2 waves per SIMD
    const size_t sink_b = sfm::align_up(sizeof(int) * (size_t)blocks * 256, 256);
    char* ws = (char*)sfm::workspace(ctx, sink_b + sizeof(unsigned long long) * 4 * (size_t)blocks);
    if (!ws) return SFM_ERR_NOMEM;
    int* sink = (int*)ws;
    unsigned long long* stamps = (unsigned long long*)(ws + sink_b);
    hipEvent_t e0, e1;
    SFM_HIP_CHECK(hipEventCreate(&e0));
    SFM_HIP_CHECK(hipEventCreate(&e1));
    auto timed = [&](int iters, float* ms) -> int {
        SFM_HIP_CHECK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(calib_mfma_i8_kernel, dim3(blocks), dim3(256), 0, st, iters, 0x9E3779B9u,
                           sink, stamps);
        SFM_HIP_CHECK(hipGetLastError());
        SFM_HIP_CHECK(hipEventRecord(e1, st));
        SFM_HIP_CHECK(hipEventSynchronize(e1));
        SFM_HIP_CHECK(hipEventElapsedTime(ms, e0, e1));
        return SFM_OK;
    };
    float ms = 0.0f;
    int iters = 256, rc = SFM_OK;
    // size the loop: short launches until one takes >= 10 ms, then one of about target_ms
    while (rc == SFM_OK && iters < (1 << 26)) {
        rc = timed(iters, &ms);
        if (ms >= 10.0f) break;
        iters *= 4;
    }
    if (rc == SFM_OK) {
        iters = std::max(1, (int)((double)iters * target_ms / std::max(ms, 1e-3f)));
        rc = timed(iters, &ms);
    }
    std::vector<unsigned long long> s(4 * (size_t)blocks);
    if (rc == SFM_OK && hipMemcpy(s.data(), stamps, s.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
        rc = SFM_ERR_HIP;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc != SFM_OK) return rc;
    std::vector<double> clk;
    for (int b = 0; b < blocks; ++b) {
        const double dr = (double)(s[4 * b + 3] - s[4 * b + 1]);
        if (dr > 0) clk.push_back((double)(s[4 * b + 2] - s[4 * b]) / (dr / 100e6) / 1e9);
    }
    std::sort(clk.begin(), clk.end());
    const double ops = (double)blocks * 4.0 * (double)iters * 16.0 * (32.0 * 32.0 * 32.0 * 2.0);
    out[0] = ms;
    out[1] = ops / (ms * 1e-3) / 1e12;
    out[2] = clk.empty() ? 0.0 : clk[clk.size() / 2];
    out[3] = out[1] / (2048.0 * 4.0 * ctx->n_cu * 2.4e9 / 1e12);
    return SFM_OK;
}
