// Verified match graph compaction (the reference's pair_matches list, code/pipeline.py:42-47:
// keep non-empty pairs as Pair(img_inx_1, img_inx_2, matches)), restated for a pair batch on the
// GPU: rows (global pair index, queryIdx, trainIdx) of the RANSAC inliers of every verified pair,
// pair-major and ascending match index within a pair — the order the multi-GPU all-gather keeps.
//
// Two entry points so the caller can size the output between them:
//   sfm_graph_offsets: one block, exclusive scan of the per-pair verified inlier counts -> [P+1]
//   sfm_graph_rows:    one block per pair, ordered ballot compaction of the inlier mask
//                      (packed = 1: 4-byte rows queryIdx << 16 | trainIdx, the exchange format).
// Multi-GPU: every rank writes its rows packed, the ranks all-gather them, and
//   sfm_graph_expand:  one block per pair turns the gathered packed rows back into [n][3] rows,
//                      reading each pair's rows at its source offset in the gathered buffer.
#include "match_common.h"
#include "sfm_internal.h"

namespace {

constexpr int SCAN_T = 1024;

__global__ __launch_bounds__(SCAN_T) void graph_offsets_kernel(int n_pairs,
                                                               const int32_t* __restrict__ inl,
                                                               int min_inl,
                                                               int64_t* __restrict__ offsets) {
    __shared__ int64_t wsum[SCAN_T / 64];
    __shared__ int64_t carry;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n_pairs; base += SCAN_T) {
        const int p = base + tid;
        const int c = (p < n_pairs && inl[p] >= min_inl) ? inl[p] : 0;
        // inclusive wave scan
        int64_t v = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t o = __shfl_up(v, off, 64);
            if (lane >= off) v += o;
        }
        if (lane == 63) wsum[wave] = v;
        __syncthreads();
        int64_t pre = carry;
        for (int w = 0; w < wave; ++w) pre += wsum[w];
        if (p < n_pairs) offsets[p] = pre + v - c;
        __syncthreads();
        if (tid == SCAN_T - 1) carry = pre + v;
        __syncthreads();
    }
    if (tid == 0) offsets[n_pairs] = carry;
}

// (Staging a chunk's [n][3] rows in LDS for consecutive dword stores measured slower here,
// 847 -> 965 us per cfg4 launch: the extra barrier per chunk costs more than the stores;
// profiles/r03/graph_lds_ab_r5f.txt.)
__global__ __launch_bounds__(256) void graph_rows_kernel(
    int k_max, int pair_base, const int32_t* __restrict__ match_count,
    const int32_t* __restrict__ matches, const uint8_t* __restrict__ mask,
    const int32_t* __restrict__ inl, int min_inl, const int64_t* __restrict__ offsets,
    int32_t* __restrict__ rows, int packed) {
    __shared__ int wsum[4];
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (inl[p] < min_inl) return;  // block-uniform
    const int M = match_count[p];
    const uint8_t* mk = mask + (size_t)p * k_max;
    const int32_t* mt = matches + (size_t)p * k_max * 2;
    int64_t base = offsets[p];
    for (int m0 = 0; m0 < M; m0 += 256) {
        const int m = m0 + tid;
        const bool keep = m < M && mk[m] != 0;
        const unsigned long long bal = __ballot(keep);
        const int pre = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = __popcll(bal);
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            off += (w < wave) ? wsum[w] : 0;
            tot += wsum[w];
        }
        if (keep && packed) {
            rows[base + off + pre] = (int32_t)(((uint32_t)mt[2 * m] << 16) | (uint32_t)mt[2 * m + 1]);
        } else if (keep) {
            int32_t* o = rows + (base + off + pre) * 3;
            o[0] = pair_base + p;
            o[1] = mt[2 * m];
            o[2] = mt[2 * m + 1];
        }
        base += tot;
        __syncthreads();
    }
}

// rows[dst[p] + i] = (pair_base + p, v >> 16, v & 0xFFFF), v = packed[src[p] + i], i < count[p];
// 256 rows at a time through LDS, stored as consecutive dwords (0.69 -> 0.58 ms at cfg4 size
// against three 4-B stores at a 12-B lane stride; profiles/r03/graph_lds_ab_r5f.txt)
__global__ __launch_bounds__(256) void graph_expand_kernel(
    int pair_base, const int32_t* __restrict__ count, const int64_t* __restrict__ src,
    const int64_t* __restrict__ dst, const uint32_t* __restrict__ packed,
    int32_t* __restrict__ rows) {
    __shared__ int32_t stage[3 * 256];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n = count[p];
    const uint32_t* in = packed + src[p];
    int32_t* out = rows + dst[p] * 3;
    for (int i0 = 0; i0 < n; i0 += 256) {
        const int i = i0 + tid, c = min(256, n - i0);
        if (i < n) {
            const uint32_t v = in[i];
            stage[3 * tid] = pair_base + p;
            stage[3 * tid + 1] = (int32_t)(v >> 16);
            stage[3 * tid + 2] = (int32_t)(v & 0xFFFFu);
        }
        __syncthreads();
        for (int k = tid; k < 3 * c; k += 256) out[3 * i0 + k] = stage[k];
        __syncthreads();
    }
}

}  // namespace

extern "C" int sfm_graph_offsets(sfm_ctx* ctx, int32_t n_pairs, const int32_t* inl_count,
                                 int32_t min_inliers, int64_t* out_offsets) {
    SFM_REQUIRE(ctx && out_offsets, "sfm_graph_offsets: NULL argument");
    SFM_REQUIRE(n_pairs >= 0, "sfm_graph_offsets: negative size");
    SFM_REQUIRE(n_pairs == 0 || inl_count, "sfm_graph_offsets: NULL inl_count");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(graph_offsets_kernel, dim3(1), dim3(SCAN_T), 0, ctx->stream, n_pairs,
                       inl_count, min_inliers, out_offsets);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

static int graph_rows_launch(const char* fn, sfm_ctx* ctx, int32_t n_pairs, int32_t k_max,
                             int32_t pair_base, const int32_t* match_count,
                             const int32_t* matches, const uint8_t* mask,
                             const int32_t* inl_count, int32_t min_inliers,
                             const int64_t* offsets, int32_t* out, int packed) {
    SFM_REQUIRE(ctx, std::string(fn) + ": ctx is NULL");
    SFM_REQUIRE(n_pairs >= 0 && k_max >= 0 && pair_base >= 0, std::string(fn) + ": negative size");
    SFM_REQUIRE(!packed || k_max <= 65536, std::string(fn) + ": packed rows need k_max <= 65536");
    if (n_pairs == 0 || k_max == 0) return SFM_OK;
    SFM_REQUIRE(match_count && matches && mask && inl_count && offsets && out,
                std::string(fn) + ": NULL array");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(graph_rows_kernel, dim3(n_pairs), dim3(256), 0, ctx->stream, k_max,
                       pair_base, match_count, matches, mask, inl_count, min_inliers, offsets,
                       out, packed);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

extern "C" int sfm_graph_rows(sfm_ctx* ctx, int32_t n_pairs, int32_t k_max, int32_t pair_base,
                              const int32_t* match_count, const int32_t* matches,
                              const uint8_t* mask, const int32_t* inl_count,
                              int32_t min_inliers, const int64_t* offsets, int32_t* out_rows) {
    return graph_rows_launch("sfm_graph_rows", ctx, n_pairs, k_max, pair_base, match_count,
                             matches, mask, inl_count, min_inliers, offsets, out_rows, 0);
}

extern "C" int sfm_graph_rows_packed(sfm_ctx* ctx, int32_t n_pairs, int32_t k_max,
                                     const int32_t* match_count, const int32_t* matches,
                                     const uint8_t* mask, const int32_t* inl_count,
                                     int32_t min_inliers, const int64_t* offsets,
                                     uint32_t* out_packed) {
    return graph_rows_launch("sfm_graph_rows_packed", ctx, n_pairs, k_max, 0, match_count,
                             matches, mask, inl_count, min_inliers, offsets,
                             (int32_t*)out_packed, 1);
}

extern "C" int sfm_graph_expand(sfm_ctx* ctx, int32_t n_pairs, int32_t pair_base,
                                const int32_t* counts, const int64_t* src_offsets,
                                const int64_t* dst_offsets, const uint32_t* packed,
                                int32_t* out_rows) {
    SFM_REQUIRE(ctx, "sfm_graph_expand: ctx is NULL");
    SFM_REQUIRE(n_pairs >= 0 && pair_base >= 0, "sfm_graph_expand: negative size");
    if (n_pairs == 0) return SFM_OK;
    SFM_REQUIRE(counts && src_offsets && dst_offsets && packed && out_rows,
                "sfm_graph_expand: NULL array");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(graph_expand_kernel, dim3(n_pairs), dim3(256), 0, ctx->stream, pair_base,
                       counts, src_offsets, dst_offsets, packed, out_rows);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
