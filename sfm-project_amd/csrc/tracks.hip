// Feature tracks from the verified match graph (the step between the graph
// of code/pipeline.py:36-49 and triangulation / bundle adjustment).
//
// Nodes are (image, keypoint): node = img_base[image] + keypoint.  Every graph row
// (pair, queryIdx, trainIdx) is the edge (node(a, q), node(b, t)) with (a, b) = pairs[pair].
// Connected components by root hooking with compare-and-swap retries (larger root under smaller)
// + pointer jumping: the final label of every node is the smallest node id of its component — the
// unique fixed point, so the result does not depend on thread scheduling (integer atomics only).
// A track is a component with >= min_len nodes and no two nodes in the same image (COLMAP would
// split such a component; the build drops it).
// Tracks are ordered by their smallest node id, their nodes ascending (stable radix sort by
// label), which is exactly what the CPU restatement (tests: union-find) produces.
#include <hipcub/hipcub.hpp>

#include "sfm_internal.h"

namespace {

__global__ __launch_bounds__(256) void tk_init(int n, int32_t* __restrict__ label,
                                               int32_t* __restrict__ iota) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) { label[v] = v; iota[v] = v; }
}

// node -> image (block per image fills its node range)
__global__ __launch_bounds__(256) void tk_node_img(const int32_t* __restrict__ img_base,
                                                   int32_t* __restrict__ node_img) {
    const int img = blockIdx.x;
    for (int v = img_base[img] + threadIdx.x; v < img_base[img + 1]; v += 256) node_img[v] = img;
}

__device__ __forceinline__ int32_t root(const int32_t* label, int32_t x) {
    // labels only decrease and always point to a smaller-or-equal id: the chain terminates
    int32_t l = label[x];
    while (l != x) {
        x = l;
        l = label[x];
    }
    return x;
}

__global__ __launch_bounds__(256) void tk_hook(long long n_rows, const int32_t* __restrict__ rows,
                                               const int32_t* __restrict__ pairs,
                                               const int32_t* __restrict__ img_base,
                                               int32_t* label, int32_t* __restrict__ changed) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_rows) return;
    const int p = rows[3 * e], q = rows[3 * e + 1], t = rows[3 * e + 2];
    const int u = img_base[pairs[2 * p]] + q, v = img_base[pairs[2 * p + 1]] + t;
    int ru = root(label, u), rv = root(label, v);
    if (ru == rv) return;
    *changed = 1;
    // link the larger root under the smaller one; if another edge re-parented it first, follow
    // both roots again and retry (a root's label only ever moves to a smaller id, so this ends):
    // one pass joins every edge, and the root of each component is its smallest node id
    while (ru != rv) {
        const int hi = max(ru, rv), lo = min(ru, rv);
        const int old = atomicCAS(&label[hi], hi, lo);
        if (old == hi) break;
        ru = root(label, old);
        rv = root(label, lo);
    }
}

__global__ __launch_bounds__(256) void tk_compress(int n, int32_t* label) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) label[v] = root(label, v);
}

// After the sort (keys = labels ascending, vals = node ids ascending within a label): per-label
// size and same-image flag.
__global__ __launch_bounds__(256) void tk_stats(int n, const int32_t* __restrict__ key,
                                                const int32_t* __restrict__ val,
                                                const int32_t* __restrict__ node_img,
                                                int32_t* __restrict__ cnt,
                                                int32_t* __restrict__ bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int k = key[i];
    atomicAdd(&cnt[k], 1);
    // node ids are image-major, so two nodes of one image in a track are adjacent after the sort
    if (i > 0 && key[i - 1] == k && node_img[val[i - 1]] == node_img[val[i]]) bad[k] = 1;
}

__global__ __launch_bounds__(256) void tk_flags(int n, const int32_t* __restrict__ key,
                                                const int32_t* __restrict__ cnt,
                                                const int32_t* __restrict__ bad, int min_len,
                                                int32_t* __restrict__ head_keep,
                                                int32_t* __restrict__ node_keep) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int k = key[i];
    const int keep = (cnt[k] >= min_len && !bad[k]) ? 1 : 0;
    node_keep[i] = keep;
    head_keep[i] = (keep && (i == 0 || key[i - 1] != k)) ? 1 : 0;
}

// Scatter kept nodes (positions from the node scan) and track starts (from the head scan).
__global__ __launch_bounds__(256) void tk_emit(int n, const int32_t* __restrict__ key,
                                               const int32_t* __restrict__ val,
                                               const int32_t* __restrict__ node_img,
                                               const int32_t* __restrict__ img_base,
                                               const int32_t* __restrict__ head_keep,
                                               const int32_t* __restrict__ node_keep,
                                               const int32_t* __restrict__ head_pos,
                                               const int32_t* __restrict__ node_pos,
                                               int32_t* __restrict__ track_ptr,
                                               int32_t* __restrict__ track_img,
                                               int32_t* __restrict__ track_kp,
                                               int32_t* __restrict__ n_tracks) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (node_keep[i]) {
        const int o = node_pos[i], v = val[i], img = node_img[v];
        track_img[o] = img;
        track_kp[o] = v - img_base[img];
        if (head_keep[i]) track_ptr[head_pos[i]] = o;
    }
    if (i == n - 1) {
        const int nt = head_pos[i] + head_keep[i];
        *n_tracks = nt;
        track_ptr[nt] = node_pos[i] + node_keep[i];
    }
}

}  // namespace

extern "C" int sfm_tracks(sfm_ctx* ctx, int32_t n_img, const int32_t* img_base, int32_t n_pairs,
                          const int32_t* pairs, int64_t n_rows, const int32_t* rows,
                          int32_t min_len, int32_t* out_n_tracks, int32_t* out_track_ptr,
                          int32_t* out_track_img, int32_t* out_track_kp) {
    SFM_REQUIRE(ctx != nullptr, "sfm_tracks: ctx is NULL");
    SFM_REQUIRE(n_img >= 0 && n_pairs >= 0 && n_rows >= 0 && min_len >= 1,
                "sfm_tracks: bad size or min_len");
    SFM_REQUIRE(img_base && out_n_tracks && out_track_ptr && (n_rows == 0 || (pairs && rows)),
                "sfm_tracks: NULL array");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    int32_t n_nodes = 0;
    if (n_img > 0) {
        SFM_HIP_CHECK(hipMemcpyAsync(&n_nodes, img_base + n_img, sizeof(int32_t),
                                     hipMemcpyDeviceToHost, st));
        SFM_HIP_CHECK(hipStreamSynchronize(st));
    }
    SFM_REQUIRE(n_nodes >= 0, "sfm_tracks: img_base[n_img] < 0");
    if (n_nodes == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(out_n_tracks, 0, sizeof(int32_t), st));
        SFM_HIP_CHECK(hipMemsetAsync(out_track_ptr, 0, sizeof(int32_t), st));
        return SFM_OK;
    }
    SFM_REQUIRE(out_track_img && out_track_kp, "sfm_tracks: NULL output array");
    const size_t n = (size_t)n_nodes;
    // hipCUB temporary storage sizes
    size_t sort_bytes = 0, scan_bytes = 0;
    int end_bit = 1;
    while (end_bit < 31 && (1ll << end_bit) < (long long)n_nodes) ++end_bit;
    SFM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (int32_t*)nullptr,
                                                     (int32_t*)nullptr, (int32_t*)nullptr,
                                                     (int32_t*)nullptr, n_nodes, 0, end_bit, st));
    SFM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (int32_t*)nullptr,
                                                   (int32_t*)nullptr, n_nodes, st));
    const size_t a = sfm::align_up(sizeof(int32_t) * n, 256);
    const size_t tmp = sfm::align_up(std::max(sort_bytes, scan_bytes), 256);
    char* ws = (char*)sfm::workspace(ctx, 12 * a + tmp + 256);
    if (!ws) return SFM_ERR_NOMEM;
    int32_t* label = (int32_t*)ws;
    int32_t* iota = (int32_t*)(ws + a);
    int32_t* key = (int32_t*)(ws + 2 * a);
    int32_t* val = (int32_t*)(ws + 3 * a);
    int32_t* node_img = (int32_t*)(ws + 4 * a);
    int32_t* cnt = (int32_t*)(ws + 5 * a);
    int32_t* bad = (int32_t*)(ws + 6 * a);
    int32_t* head_keep = (int32_t*)(ws + 7 * a);
    int32_t* node_keep = (int32_t*)(ws + 8 * a);
    int32_t* head_pos = (int32_t*)(ws + 9 * a);
    int32_t* node_pos = (int32_t*)(ws + 10 * a);
    int32_t* changed = (int32_t*)(ws + 11 * a);
    void* temp = ws + 12 * a;
    const int nb = (int)((n + 255) / 256);
    hipLaunchKernelGGL(tk_init, dim3(nb), dim3(256), 0, st, n_nodes, label, iota);
    hipLaunchKernelGGL(tk_node_img, dim3(n_img), dim3(256), 0, st, img_base, node_img);
    SFM_HIP_CHECK(hipGetLastError());
    // hook + compress until no edge joins two components: with the CAS retry in tk_hook the first
    // round already joins every edge and the second one only confirms it (the earlier atomicMin
    // hook lost concurrent links and needed several rounds)
    if (n_rows > 0) {
        const unsigned eb = (unsigned)((n_rows + 255) / 256);
        int32_t h_changed = 1;
        int round = 0;
        for (; round < 64 && h_changed; ++round) {
            SFM_HIP_CHECK(hipMemsetAsync(changed, 0, sizeof(int32_t), st));
            hipLaunchKernelGGL(tk_hook, dim3(eb), dim3(256), 0, st, (long long)n_rows, rows, pairs,
                               img_base, label, changed);
            hipLaunchKernelGGL(tk_compress, dim3(nb), dim3(256), 0, st, n_nodes, label);
            SFM_HIP_CHECK(hipGetLastError());
            SFM_HIP_CHECK(hipMemcpyAsync(&h_changed, changed, sizeof(int32_t),
                                         hipMemcpyDeviceToHost, st));
            SFM_HIP_CHECK(hipStreamSynchronize(st));
        }
        SFM_REQUIRE(!h_changed, "sfm_tracks: connected components did not converge in 64 rounds");
    }
    size_t sb = sort_bytes;
    SFM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp, sb, label, key, iota, val, n_nodes, 0,
                                                     end_bit, st));
    SFM_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int32_t) * n, st));
    SFM_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int32_t) * n, st));
    hipLaunchKernelGGL(tk_stats, dim3(nb), dim3(256), 0, st, n_nodes, key, val, node_img, cnt, bad);
    hipLaunchKernelGGL(tk_flags, dim3(nb), dim3(256), 0, st, n_nodes, key, cnt, bad, min_len,
                       head_keep, node_keep);
    SFM_HIP_CHECK(hipGetLastError());
    size_t cb = scan_bytes;
    SFM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp, cb, head_keep, head_pos, n_nodes, st));
    cb = scan_bytes;
    SFM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp, cb, node_keep, node_pos, n_nodes, st));
    hipLaunchKernelGGL(tk_emit, dim3(nb), dim3(256), 0, st, n_nodes, key, val, node_img, img_base,
                       head_keep, node_keep, head_pos, node_pos, out_track_ptr, out_track_img,
                       out_track_kp, out_n_tracks);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
