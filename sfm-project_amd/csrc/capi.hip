// C-ABI entry points of libsfmcore: context management, error reporting, argument validation.
// The per-stage kernels live in match_mfma.hip, match_hamming.hip, ransac.hip and ba.hip.
#include "sfm_internal.h"

static thread_local std::string g_err;

namespace sfm {
void set_error(const std::string& msg) { g_err = msg; }

void* workspace(sfm_ctx* ctx, size_t bytes) {
    // every workspace user may overwrite (or, growing, free) the counted RANSAC batch's wave
    // words: sfm_ransac_wave_stops then fails cleanly instead of reading stale or freed memory
    // (the RANSAC call re-arms it after its own workspace request)
    ctx->rs_last_w = nullptr;
    ctx->rs_last_pairs = ctx->rs_last_hyp = 0;
    if (bytes <= ctx->ws_bytes) return ctx->ws;
    // growing frees and reallocates (a device-wide synchronisation): illegal inside a HIP-graph
    // capture of the context's stream — the caller runs the call once uncaptured to size it
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(ctx->stream, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone) {
        set_error("workspace growth to " + std::to_string(bytes) +
                  " bytes while the context's stream is being captured: run the call once "
                  "uncaptured first so the workspace is sized");
        return nullptr;
    }
    if (ctx->ws) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(ctx->ws);
        ctx->ws = nullptr;
        ctx->ws_bytes = 0;
    }
    size_t want = align_up(bytes + bytes / 4, 1 << 20);
    if (hipMalloc(&ctx->ws, want) != hipSuccess) {
        set_error("workspace allocation of " + std::to_string(want) + " bytes failed");
        return nullptr;
    }
    ctx->ws_bytes = want;
    return ctx->ws;
}
}  // namespace sfm

extern "C" {

const char* sfm_last_error(void) { return g_err.c_str(); }

int32_t sfm_version(void) { return 5; }  // 2: sfm_ba_solve_params.poll 0 = every 8; 3: BA chunk mode; 4: explicit Schur; 5: poll_first

int sfm_ctx_create(int32_t device, sfm_ctx** out) {
    SFM_REQUIRE(out != nullptr, "sfm_ctx_create: out is NULL");
    *out = nullptr;
    int n = 0;
    SFM_HIP_CHECK(hipGetDeviceCount(&n));
    SFM_REQUIRE(device >= 0 && device < n, "sfm_ctx_create: device index out of range");
    SFM_HIP_CHECK(hipSetDevice(device));
    hipDeviceProp_t prop;
    SFM_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0) {
        sfm::set_error(std::string("sfm_ctx_create: libsfmcore is built for gfx950, device is ") +
                       prop.gcnArchName);
        return SFM_ERR_INVALID;
    }
    sfm_ctx* c = new sfm_ctx();
    c->device = device;
    c->n_cu = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        sfm::set_error("sfm_ctx_create: hipStreamCreate failed");
        return SFM_ERR_HIP;
    }
    if (hipEventCreateWithFlags(&c->handoff, hipEventDisableTiming) != hipSuccess) {
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        sfm::set_error("sfm_ctx_create: hipEventCreate failed");
        return SFM_ERR_HIP;
    }
    c->stream = c->own_stream;
    *out = c;
    return SFM_OK;
}

int sfm_ctx_destroy(sfm_ctx* ctx) {
    if (!ctx) return SFM_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->handoff) (void)hipEventDestroy(ctx->handoff);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->poll_ev) (void)hipEventDestroy(ctx->poll_ev);
    if (ctx->rs_acc) (void)hipFree(ctx->rs_acc);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return SFM_OK;
}

int sfm_ctx_set_stream(sfm_ctx* ctx, void* hip_stream) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ctx_set_stream: ctx is NULL");
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the legacy default stream (torch's default)
    if (s == ctx->stream) return SFM_OK;
    // Every call on a context shares one device workspace (match partials, RANSAC planes and
    // G table, BA scratch): work already enqueued on the previous stream must finish with it
    // before the new stream's kernels reuse it.  One event record + one stream wait, no host
    // synchronisation.
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    SFM_HIP_CHECK(hipEventRecord(ctx->handoff, ctx->stream));
    SFM_HIP_CHECK(hipStreamWaitEvent(s, ctx->handoff, 0));
    ctx->stream = s;
    return SFM_OK;
}

int sfm_ctx_sync(sfm_ctx* ctx) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ctx_sync: ctx is NULL");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    SFM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return SFM_OK;
}

int sfm_match_batch(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                    int32_t k_max, int32_t dim, const int32_t* pairs, int32_t n_pairs,
                    const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                    int32_t* out_dist) {
    SFM_REQUIRE(ctx && prm, "sfm_match_batch: ctx/prm is NULL");
    SFM_REQUIRE(n_pairs >= 0 && n_img >= 0 && k_max >= 0, "sfm_match_batch: negative size");
    if (n_pairs == 0) return SFM_OK;
    SFM_REQUIRE(desc && n_kp && pairs && out_count && out_match && out_dist,
                "sfm_match_batch: NULL array");
    SFM_REQUIRE(prm->cross_check >= 0 && prm->cross_check <= 2, "sfm_match_batch: bad cross_check");
    SFM_REQUIRE(!(prm->cross_check == SFM_XC_OPENCV && prm->ratio_den > 0),
                "sfm_match_batch: ratio test is not defined with the OpenCV cross-check rule");
    SFM_REQUIRE(prm->ratio_den >= 0 && prm->ratio_num >= 0 && prm->ratio_num <= 65535 &&
                    prm->ratio_den <= 65535,
                "sfm_match_batch: ratio must be num/den with 0 <= num, den <= 65535");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    if (prm->metric == SFM_METRIC_L2) {
        SFM_REQUIRE(dim == 128, "sfm_match_batch: L2 metric needs dim == 128");
        // cross-check rules: the column-winner kernel, k_max <= 8192 (COLMAP-style 8192 SIFT);
        // ratio-only and no-rule paths: the fused key / forward-reverse kernels, k_max <= 4096
        SFM_REQUIRE(k_max <= 8192, "sfm_match_batch: L2 k_max > 8192 not supported");
        SFM_REQUIRE(k_max <= 4096 || prm->cross_check != SFM_XC_NONE,
                    "sfm_match_batch: L2 k_max > 4096 needs a cross-check rule");
        return sfm_match_l2_launch(ctx, desc, n_kp, n_img, k_max, pairs, n_pairs, prm, out_count,
                                   out_match, out_dist);
    }
    if (prm->metric == SFM_METRIC_HAMMING) {
        SFM_REQUIRE(dim == 32, "sfm_match_batch: Hamming metric needs dim == 32 (256-bit ORB)");
        SFM_REQUIRE(k_max <= 8192, "sfm_match_batch: k_max > 8192 not supported");
        // MFMA path (bits as 0/1 bytes, d = |a| + |b| - 2 a.b) up to 4096 descriptors; the VALU
        // popcount kernel above that (or when SFM_HAMMING_VALU=1, for A/B measurements)
        const char* e = getenv("SFM_HAMMING_VALU");
        if (k_max <= 4096 && !(e && atoi(e) != 0))
            return sfm_match_hamming_mfma_launch(ctx, desc, n_kp, n_img, k_max, pairs, n_pairs,
                                                 prm, out_count, out_match, out_dist);
        return sfm_match_hamming_launch(ctx, desc, n_kp, n_img, k_max, pairs, n_pairs, prm,
                                        out_count, out_match, out_dist);
    }
    sfm::set_error("sfm_match_batch: unknown metric");
    return SFM_ERR_INVALID;
}

int sfm_match_batch_both(sfm_ctx* ctx, const uint8_t* desc, const int32_t* n_kp, int32_t n_img,
                         int32_t k_max, int32_t dim, const int32_t* pairs, int32_t n_pairs,
                         const sfm_match_params* prm, int32_t* out_count, int32_t* out_match,
                         int32_t* out_dist) {
    SFM_REQUIRE(ctx && prm, "sfm_match_batch_both: ctx/prm is NULL");
    SFM_REQUIRE(n_pairs >= 0 && n_img >= 0 && k_max >= 0, "sfm_match_batch_both: negative size");
    if (n_pairs == 0) return SFM_OK;
    SFM_REQUIRE(desc && n_kp && pairs && out_count && out_match && out_dist,
                "sfm_match_batch_both: NULL array");
    SFM_REQUIRE(prm->cross_check >= 0 && prm->cross_check <= 2,
                "sfm_match_batch_both: bad cross_check");
    SFM_REQUIRE(prm->ratio_den == 0,
                "sfm_match_batch_both: no ratio test (it needs the reverse direction's second "
                "nearest neighbour): match both orders with sfm_match_batch");
    SFM_REQUIRE(k_max <= 4096, "sfm_match_batch_both: k_max > 4096 not supported");
    SFM_REQUIRE(prm->metric == SFM_METRIC_L2 || prm->metric == SFM_METRIC_HAMMING,
                "sfm_match_batch_both: unknown metric");
    SFM_REQUIRE(dim == (prm->metric == SFM_METRIC_L2 ? 128 : 32),
                "sfm_match_batch_both: dim must be 128 (L2) or 32 (Hamming)");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    return sfm_match_both_launch(ctx, prm->metric, desc, n_kp, n_img, k_max, pairs, n_pairs, prm,
                                 out_count, out_match, out_dist);
}

}  // extern "C"
