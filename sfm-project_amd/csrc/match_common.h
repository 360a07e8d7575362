// Shared device helpers for the matching kernels: decision rule + ordered compaction.
// Decision rule = DESIGN.md §3.1 (restating code/feature_matching.py:48-58 and SURVEY.md §8a a3').
#pragma once
#include "sfm_internal.h"

namespace sfm {

constexpr long long DIST_INF = 0x7fffffffffffffffLL;

// Ratio test in the distance domain the metric reports: L2 reports d^2, so the test d1 < r*d2 is
// den^2*d1^2 < num^2*d2^2; Hamming reports d, so den*d1 < num*d2.  d2 = INF always passes.
__device__ inline bool ratio_ok(long long d1, long long d2, int num, int den, bool squared) {
    if (den <= 0 || d2 == DIST_INF) return true;
    if (squared) return (long long)den * den * d1 < (long long)num * num * d2;
    return (long long)den * d1 < (long long)num * d2;
}

// Block-wide (256 threads) ordered compaction: threads with keep==true append (i, j, d) in thread
// order after `*base`; returns the new base (uniform).  Uses 8 ints of LDS scratch at `wsum`.
__device__ inline int compact256(bool keep, int i, int j, int d, int base, int* wsum,
                                 int32_t* out_match, int32_t* out_dist) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long bal = __ballot(keep);
    int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; ++w) {
        int s = wsum[w];
        off += (w < wave) ? s : 0;
        tot += s;
    }
    if (keep) {
        int o = base + off + pre;
        out_match[2 * o] = i;
        out_match[2 * o + 1] = j;
        out_dist[o] = d;
    }
    __syncthreads();
    return base + tot;
}

// Block-wide ordered compaction for NT threads (NT/64 waves): as compact256, wsum holds NT/64 ints.
template <int NT>
__device__ inline int compact_n(bool keep, int i, int j, int d, int base, int* wsum,
                                int32_t* out_match, int32_t* out_dist) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long bal = __ballot(keep);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const int s = wsum[w];
        off += (w < wave) ? s : 0;
        tot += s;
    }
    if (keep) {
        const int o = base + off + pre;
        out_match[2 * o] = i;
        out_match[2 * o + 1] = j;
        out_dist[o] = d;
    }
    __syncthreads();
    return base + tot;
}

}  // namespace sfm
