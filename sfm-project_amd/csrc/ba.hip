// Bundle-adjustment linearisation: residuals, Jacobians and the J^TJ blocks (K3, SURVEY.md §8a a7,
// DESIGN.md §4.3).  Fills the empty reference module code/3d_reconstruction.py.
//
// fp64 throughout.  Deterministic (no float atomics): every accumulation has a fixed order.
// Kernels:
//   ba_jtj_kernel      camera waves first (wave per (camera, split), four per block: J_c
//                      recomputed from the camera's rotation — computed once per wave — over a
//                      contiguous share of the camera's observations (cam_ptr/cam_obs CSR), fixed
//                      lane-strided order + recursive-halving wave sum -> U_c, g_c), then
//                      observation blocks
//                      (thread per observation, enough waves to stream HBM: residual, J_c (2x8),
//                      J_p (2x3) -> res, W = w J_c^T J_p staged through LDS for coalesced stores;
//                      V_p, g_p by a segmented scan of the point terms across the wave (points are
//                      point-major contiguous), boundary-cut segments to head/tail records.  The
//                      two halves are independent, so the latency-bound camera reduction runs
//                      underneath the observation stream.
//   ba_finish_kernel   points spanning waves, empty points, the cost; chunk mode
//                      (sfm_ba_set_chunks): also U_c / g_c and the cost from the chunk partials;
//   ba_final_kernel    camera split sums (only with fewer than 256 cameras).
// Algorithmic HBM traffic ~300 B/observation; this is an HBM-bound stage.
#include <algorithm>
#include <cstdlib>

#include "camera_model.h"
#include "sfm_internal.h"

namespace {

struct ObsLin {
    double r[2];
    double Jc[16];  // row-major 2x8
    double Jp[6];   // row-major 2x3
    double w, rho;
};

// Mirrors oracle_ba_obs (oracle/sfm_oracle_ba.c).  R = rotmat(cam[0..2]) (camera_model.h; the
// camera blocks compute it once per camera, the observation blocks once per observation).
__device__ __forceinline__ void linearize(const double (&R)[9], const double* __restrict__ cam,
                                          const double* __restrict__ pp, const double X[3],
                                          double u, double v, double loss_s, bool want_jp,
                                          ObsLin& o) {
    double Y[3], P[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        Y[i] = R[3 * i] * X[0] + R[3 * i + 1] * X[1] + R[3 * i + 2] * X[2];
        P[i] = Y[i] + cam[3 + i];
    }
    const double iz = 1.0 / P[2];
    const double p0 = P[0] * iz, p1 = P[1] * iz;
    const double f = cam[6], k1 = cam[7];
    const double rho2 = p0 * p0 + p1 * p1;
    const double d = 1.0 + k1 * rho2;
    const double e0 = f * d * p0 + pp[0] - u;
    const double e1 = f * d * p1 + pp[1] - v;
    const double e = e0 * e0 + e1 * e1;
    double w = 1.0, rho = e;
    if (loss_s > 0.0) {
        const double s2 = loss_s * loss_s;
        w = 1.0 / (1.0 + e / s2);
        rho = s2 * log1p(e / s2);
    }
    const double m00 = f * (d + 2.0 * k1 * p0 * p0), m01 = f * (2.0 * k1 * p0 * p1);
    const double m11 = f * (d + 2.0 * k1 * p1 * p1);
    const double D[2][3] = {{iz, 0.0, -p0 * iz}, {0.0, iz, -p1 * iz}};
    double A[2][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        A[0][j] = m00 * D[0][j] + m01 * D[1][j];
        A[1][j] = m01 * D[0][j] + m11 * D[1][j];
    }
    const double S[3][3] = {{0.0, Y[2], -Y[1]}, {-Y[2], 0.0, Y[0]}, {Y[1], -Y[0], 0.0}};
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            o.Jc[8 * a + j] = A[a][0] * S[0][j] + A[a][1] * S[1][j] + A[a][2] * S[2][j];
            o.Jc[8 * a + 3 + j] = A[a][j];
            if (want_jp) o.Jp[3 * a + j] = A[a][0] * R[j] + A[a][1] * R[3 + j] + A[a][2] * R[6 + j];
        }
    o.Jc[6] = d * p0;        o.Jc[14] = d * p1;
    o.Jc[7] = f * rho2 * p0; o.Jc[15] = f * rho2 * p1;
    o.r[0] = e0; o.r[1] = e1;
    o.w = w; o.rho = rho;
}

constexpr int NV = 10;      // per-observation point terms: V upper triangle (6), g_p (3), 0.5 rho
constexpr int NU = 36 + 8;  // upper triangle of U_c (8x8) + g_c
#ifndef CAM_MLP
#define CAM_MLP 2  // observations whose gathers a camera-wave lane keeps in flight (2: 196 VGPRs,
                   // 60.3 us vs 61-62 with 4 at 220 VGPRs, profiles/r02/k3_ba_ab.txt)
#endif
#ifndef BA_CAM_HALVES
#define BA_CAM_HALVES 1  // 2: two waves per camera, each accumulating half of the 44 sums
#endif
constexpr int CH = BA_CAM_HALVES, NUH = NU / CH;  // waves per camera, sums per wave
static_assert(NU % CH == 0, "camera halves");
#ifndef BA_SPLIT_TARGET
#define BA_SPLIT_TARGET 256
#endif
constexpr int SPLIT_TARGET = BA_SPLIT_TARGET;  // camera waves wanted (splits per camera = this / n_cam); more only
                                   // add reduction work (block-per-camera version at 500 cameras:
                                   // 2 splits 90 us, 4 splits 113 us vs 1 split 69 us)

__device__ __forceinline__ void write_point(double* __restrict__ V, double* __restrict__ gp, int p,
                                            const double (&a)[NV]) {
    double* Vo = V + 9 * (size_t)p;
    Vo[0] = a[0]; Vo[1] = a[1]; Vo[2] = a[2];
    Vo[3] = a[1]; Vo[4] = a[3]; Vo[5] = a[4];
    Vo[6] = a[2]; Vo[7] = a[4]; Vo[8] = a[5];
    gp[3 * (size_t)p] = a[6]; gp[3 * (size_t)p + 1] = a[7]; gp[3 * (size_t)p + 2] = a[8];
}

// One thread per observation (enough waves to stream HBM): residual, W = w J_c^T J_p, and the
// point terms (w J_p^T J_p upper triangle, w J_p^T r) summed per point by a segmented scan across
// the wave — observations are point-major, so a point's observations are consecutive lanes.
// Points whose observations lie inside one wave are written here; the segments cut by a wave
// boundary go to head/tail records that the finish blocks combine.  The cost (sum of rho/2)
// is reduced per wave.  All orders are fixed: deterministic.
// W (192 B per observation) leaves through LDS in two halves of 12 doubles: each lane writes its
// half row to a padded per-wave image (row stride 13 doubles: conflict-free ds_write_b64), then
// the wave stores the half rows with 16-B lane-contiguous stores (96-B runs) instead of 12 stores
// of 16-B pieces at a 192-B lane stride.  Half images keep the block at 26 KB of LDS (six blocks
// per CU at the kernel's 78 VGPRs).
constexpr int WHALF = 12;           // doubles per staged half row
constexpr int WROW = WHALF + 1;     // + 1 pad
constexpr int OBS_LDS = 64 * WROW;  // doubles per wave

__device__ __forceinline__ void obs_block(
    int ob, int n_obs, const double* __restrict__ cams, const double* __restrict__ pp,
    const double* __restrict__ pts, const int32_t* __restrict__ cam_idx,
    const int32_t* __restrict__ pt_idx, const int32_t* __restrict__ pt_ptr,
    const double* __restrict__ uv, double loss_s, double* __restrict__ W,
    double* __restrict__ res, double* __restrict__ V, double* __restrict__ gp,
    double* __restrict__ seg, int32_t* __restrict__ seg_pt, double* __restrict__ cost_blk,
    double* __restrict__ lds, int nck, const sfm::ChunkOff& cobs, const sfm::ChunkOff& vst) {
    __shared__ double cred[4];
    const int lane = threadIdx.x & 63;
    // Chunk mode (nck > 0): blocks tile a virtual index space in which every chunk starts at a
    // multiple of 256 (vst: the chunks' virtual starts, chunk_layout), so where a point's
    // observations are cut into waves — and with it the association of its V_p / g_p sums — and
    // the blocks' cost shares depend only on the chunk.
    const int vo = ob * 256 + threadIdx.x;
    const int wv = vo >> 6;  // wave index (blocks are whole waves)
    int o = vo, wfirst = wv << 6, wend = n_obs;
    if (nck > 0) {
        // chunks start at block boundaries: the block start decides (a uniform, scalar lookup)
        int c0, c1, v0, v1;
        sfm::chunk_of(ob << 8, nck, vst, cobs, c0, c1);
        sfm::chunk_of(ob << 8, nck, vst, vst, v0, v1);
        o = c0 + (vo - v0);
        wfirst = c0 + ((wv << 6) - v0);
        wend = vo < vst.v[nck] ? c1 : 0;
    }
    const bool valid = o < wend;
    double* wimg = lds + (threadIdx.x >> 6) * OBS_LDS;
    int p = -1;
    double t[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) t[k] = 0.0;
    ObsLin Lw;
    if (valid) {
        const int c = cam_idx[o];
        p = pt_idx[o];
        const double X[3] = {pts[3 * (size_t)p], pts[3 * (size_t)p + 1], pts[3 * (size_t)p + 2]};
        const double2 z = *(const double2*)(uv + 2 * (size_t)o);
        const double* cam = cams + 8 * (size_t)c;
        double R[9];
        rotmat(cam[0], cam[1], cam[2], R);
        ObsLin L;
        linearize(R, cam, pp + 2 * (size_t)c, X, z.x, z.y, loss_s, true, L);
        *(double2*)(res + 2 * (size_t)o) = make_double2(L.r[0], L.r[1]);
        Lw = L;
        int k = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = i; j < 3; ++j) t[k++] = L.w * (L.Jp[i] * L.Jp[j] + L.Jp[3 + i] * L.Jp[3 + j]);
#pragma unroll
        for (int i = 0; i < 3; ++i) t[6 + i] = L.w * (L.Jp[i] * L.r[0] + L.Jp[3 + i] * L.r[1]);
        t[9] = 0.5 * L.rho;
    }
    {   // the wave's W block: 64 rows x 24 doubles, contiguous in W from observation wfirst
        const int nrow = min(64, wend - wfirst);
        double2* Wo = (double2*)(W + 24 * (size_t)max(wfirst, 0));
        double* wr = wimg + lane * WROW;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            if (valid) {
#pragma unroll
                for (int k = 0; k < WHALF; ++k) {
                    const int q = WHALF * hf + k, i = q / 3, j = q % 3;
                    wr[k] = Lw.w * (Lw.Jc[i] * Lw.Jp[j] + Lw.Jc[8 + i] * Lw.Jp[3 + j]);
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const int e = q * 64 + lane;  // double pair e of the half block
                const int row = e / 6, col = 2 * (e - 6 * row);
                if (row < nrow)
                    Wo[12 * row + 6 * hf + col / 2] =
                        make_double2(wimg[row * WROW + col], wimg[row * WROW + col + 1]);
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    // cost: fixed-order wave sums, then the block's four in order: one entry per block
    double cw = t[9];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cw += __shfl_down(cw, off, 64);
    if (lane == 0) cred[threadIdx.x >> 6] = cw;
    __syncthreads();
    if (threadIdx.x == 0) cost_blk[ob] = ((cred[0] + cred[1]) + cred[2]) + cred[3];
    // segmented inclusive scan over runs of equal point id (contiguous by construction)
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int pv = __shfl_up(p, off, 64);
        const bool take = lane >= off && pv == p;
#pragma unroll
        for (int k = 0; k < NV - 1; ++k) {
            const double v = __shfl_up(t[k], off, 64);
            t[k] += take ? v : 0.0;
        }
    }
    const int pn = __shfl_down(p, 1, 64);
    const bool seg_end = valid && (lane == 63 || pn != p);
    int o_first = 0, o_last = 0;
    if (seg_end) { o_first = pt_ptr[p]; o_last = pt_ptr[p + 1] - 1; }
    const bool starts_here = o_first >= wfirst, ends_here = o_last == o;
    // the wave's tail record id (read by the fix-up) is always written: no memset needed
    if (lane == 63) seg_pt[wv * 2 + 1] = (seg_end && starts_here && !ends_here) ? p : -1;
    if (!seg_end) return;
    if (starts_here && ends_here) {
        write_point(V, gp, p, t);
    } else {
        const int side = starts_here ? 1 : 0;  // 1: tail (continues into later waves), 0: head
        double* r = seg + ((size_t)wv * 2 + side) * NV;
#pragma unroll
        for (int k = 0; k < NV - 1; ++k) r[k] = t[k];
    }
}

// Wave (camera c, split s): fixed-order partial U_c / g_c over a contiguous share of the camera's
// observations (J_c recomputed from the camera's rotation, computed once per wave: cheaper than
// storing J_c, HBM is the bound), lane-strided order + shuffle tree — written directly when
// splits == 1, else as partials for ba_final_kernel.  One camera per WAVE (four per block): the
// camera work holds a quarter of the block slots it held as block-per-camera, so the observation
// blocks of the same launch stream underneath it from the start.
// Sums t in [H*NUH, H*NUH + NUH) of one observation into acc[t - H*NUH] (compile-time indices).
template <int H>
__device__ __forceinline__ void cam_accum_half(double (&acc)[NU], const ObsLin& L) {
    int t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = i; j < 8; ++j) {
            if (t >= H * NUH && t < H * NUH + NUH)
                acc[t - H * NUH] += L.w * (L.Jc[i] * L.Jc[j] + L.Jc[8 + i] * L.Jc[8 + j]);
            ++t;
        }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (t >= H * NUH && t < H * NUH + NUH)
            acc[t - H * NUH] += L.w * (L.Jc[i] * L.r[0] + L.Jc[8 + i] * L.r[1]);
        ++t;
    }
}

// Sum t of the 44 (upper-triangle U_c entry in row-major order, then g_c) into U_c (both
// triangles) or g_c.
__device__ __forceinline__ void cam_store_one(int t, double v, double* __restrict__ Uc,
                                              double* __restrict__ g) {
    if (t >= 36) {
        g[t - 36] = v;
        return;
    }
    int i = 0;
    while (t >= 8 - i) { t -= 8 - i; ++i; }
    const int j = i + t;
    Uc[8 * i + j] = v;
    Uc[8 * j + i] = v;
}

// Chunk mode (cb != nullptr): `splits` = G waves per camera; wave g of camera c takes chunks
// g, g + G, ... of the camera's observations (cb: the camera's list cut at the chunk starts), one
// fixed-order partial per chunk into part[c][chunk], rotation computed once per wave.
__device__ __forceinline__ void camera_wave(
    int cw, const double* __restrict__ cams, const double* __restrict__ pp,
    const double* __restrict__ pts, const int32_t* __restrict__ pt_idx,
    const double* __restrict__ uv, const int32_t* __restrict__ cam_ptr,
    const int32_t* __restrict__ cam_obs, double loss_s, int splits, double* __restrict__ part,
    double* __restrict__ U, double* __restrict__ gc, const int32_t* __restrict__ cb, int nck) {
    const int lane = threadIdx.x & 63;
    const int hw = cw % CH;  // which NUH of the 44 sums this wave accumulates (wave-uniform)
    cw /= CH;
    const int c = cw / splits, s = cw - c * splits;
    double acc[NU];  // entries outside [hw*NUH, hw*NUH + NUH) are dead when CH > 1
    const double* cam = cams + 8 * (size_t)c;
    double R[9];
    auto rotation = [&]() {
#ifdef BA_ABL_NOROT  // ablation (timing only)
        for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
#else
        rotmat(cam[0], cam[1], cam[2], R);
#endif
    };
    // CAM_MLP observations per step: the dependent gathers (cam_obs -> pt_idx -> point, uv) of
    // all of them are issued before any is used (memory-level parallelism; latency-bound waves)
    auto accumulate = [&](int e0, int e1) {
#pragma unroll
        for (int i = 0; i < NU; ++i) acc[i] = 0.0;
        for (int e = e0 + lane; e < e1; e += CAM_MLP * 64) {
            int o[CAM_MLP], pi[CAM_MLP];
            double X[CAM_MLP][3], u[CAM_MLP], v[CAM_MLP];
#pragma unroll
            for (int q = 0; q < CAM_MLP; ++q) o[q] = (e + q * 64 < e1) ? cam_obs[e + q * 64] : -1;
#pragma unroll
            for (int q = 0; q < CAM_MLP; ++q) pi[q] = o[q] >= 0 ? pt_idx[o[q]] : 0;
#pragma unroll
            for (int q = 0; q < CAM_MLP; ++q) {
                const int oo = o[q] >= 0 ? o[q] : 0;
                X[q][0] = pts[3 * (size_t)pi[q]];
                X[q][1] = pts[3 * (size_t)pi[q] + 1];
                X[q][2] = pts[3 * (size_t)pi[q] + 2];
                u[q] = uv[2 * (size_t)oo];
                v[q] = uv[2 * (size_t)oo + 1];
            }
#pragma unroll
            for (int q = 0; q < CAM_MLP; ++q) {
                if (o[q] < 0) break;
                ObsLin L;
                linearize(R, cam, pp + 2 * (size_t)c, X[q], u[q], v[q], loss_s, false, L);
                if (CH == 1) {
                    int t = 0;
#pragma unroll
                    for (int i = 0; i < 8; ++i)
#pragma unroll
                        for (int j = i; j < 8; ++j)
                            acc[t++] += L.w * (L.Jc[i] * L.Jc[j] + L.Jc[8 + i] * L.Jc[8 + j]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) acc[36 + i] += L.w * (L.Jc[i] * L.r[0] + L.Jc[8 + i] * L.r[1]);
                } else {
                    // the same expressions, sum t of this wave's half into acc[t - hw*NUH]
                    if (hw == 0) cam_accum_half<0>(acc, L);
                    else cam_accum_half<1>(acc, L);
                }
            }
        }
    };
    // the wave's NR sums by recursive halving (~NR exchanges, not 6 NR): lane l ends holding sum
    // t0 + idx and stores it, so the partial / U_c row is written by one store per lane
    constexpr int NR = CH == 1 ? NU : NUH;  // live sums of this wave
    const int t0 = CH == 1 ? 0 : hw * NUH;
    if (cb) {   // chunk mode: chunks s, s + G, ... (sfm_ba_set_chunks)
        // A camera without observations in a chunk stores its zero partial directly, and the
        // rotation is formed only by a wave with work: with local visibility (cfg5: a camera's
        // observations in 1.06 of 8 chunks) 7 of 8 waves are such, and their rotation, empty
        // sweep and 44-sum tree made chunk mode's camera half 34 % slower than the plain one
        // (profiles/r06/ba_study/s15_jtj_local.jsonl).  The same bits: an empty sweep's sum is +0.
        bool rot = false;
        for (int k = s; k < nck; k += splits) {
            const int e0 = cb[(size_t)c * (nck + 1) + k], e1 = cb[(size_t)c * (nck + 1) + k + 1];
            double* dst = part + ((size_t)c * nck + k) * NU + t0;
            if (e0 == e1) {   // wave-uniform
                if (lane < NR) dst[lane] = 0.0;
                continue;
            }
            if (!rot) {
                rotation();
                rot = true;
            }
            accumulate(e0, e1);
            int idx;
            if (sfm::wave_halving_sum<NR>(acc, lane, idx)) dst[idx] = acc[0];
        }
        return;
    }
    rotation();
    const int c0 = cam_ptr[c], c1 = cam_ptr[c + 1];
    const int len = (c1 - c0 + splits - 1) / splits;
    const int e0 = c0 + s * len;
    accumulate(e0, min(c1, e0 + len));
    int idx;
    if (!sfm::wave_halving_sum<NR>(acc, lane, idx)) return;
    if (splits > 1) {
        part[((size_t)c * splits + s) * NU + t0 + idx] = acc[0];
        return;
    }
    cam_store_one(t0 + idx, acc[0], U + 64 * (size_t)c, gc + 8 * (size_t)c);
}

// One launch for both independent halves of the linearisation: blocks [0, n_camb) are the
// latency-bound camera waves (four cameras per block, dispatched first), the rest the
// HBM-streaming observation blocks, so the camera reduction runs underneath the observation
// stream instead of after it.  The finish blocks (which read the observation blocks' segment
// records) are a second launch.  (Measured alternative: the camera kernel on a forked
// high-priority stream — the cross-queue join left ~18 us idle per call)
#ifdef BA_MINW  // build knob: minimum waves per SIMD for the merged kernel (caps its VGPRs)
#define BA_JTJ_ATTR __attribute__((amdgpu_waves_per_eu(BA_MINW, 8)))
#else
#define BA_JTJ_ATTR
#endif
__global__ __launch_bounds__(256) BA_JTJ_ATTR void ba_jtj_kernel(
    int n_camb, int n_camw, int n_obs, const double* __restrict__ cams,
    const double* __restrict__ pp, const double* __restrict__ pts,
    const int32_t* __restrict__ cam_idx, const int32_t* __restrict__ pt_idx,
    const int32_t* __restrict__ pt_ptr, const double* __restrict__ uv,
    const int32_t* __restrict__ cam_ptr, const int32_t* __restrict__ cam_obs, double loss_s,
    int splits, double* __restrict__ part, double* __restrict__ U, double* __restrict__ gc,
    double* __restrict__ W, double* __restrict__ res, double* __restrict__ V,
    double* __restrict__ gp, double* __restrict__ seg, int32_t* __restrict__ seg_pt,
    double* __restrict__ cost_blk, const int32_t* __restrict__ cb, int nck, sfm::ChunkOff cobs,
    sfm::ChunkOff vst) {
    __shared__ double lds[4 * OBS_LDS];
    const int b = blockIdx.x;
    if (b < n_camb) {
        const int cw = b * 4 + (threadIdx.x >> 6);
        if (cw < n_camw)
            camera_wave(cw, cams, pp, pts, pt_idx, uv, cam_ptr, cam_obs, loss_s, splits, part, U,
                        gc, cb, nck);
    } else {
        obs_block(b - n_camb, n_obs, cams, pp, pts, cam_idx, pt_idx, pt_ptr, uv, loss_s, W, res,
                  V, gp, seg, seg_pt, cost_blk, lds, nck, cobs, vst);
    }
}

#ifdef BA_SEQ  // A/B variant: the two halves as two launches, each at its own register budget
__global__ __launch_bounds__(256) void ba_cam_kernel(
    int n_camw, const double* __restrict__ cams, const double* __restrict__ pp,
    const double* __restrict__ pts, const int32_t* __restrict__ pt_idx,
    const double* __restrict__ uv, const int32_t* __restrict__ cam_ptr,
    const int32_t* __restrict__ cam_obs, double loss_s, int splits, double* __restrict__ part,
    double* __restrict__ U, double* __restrict__ gc) {
    const int cw = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (cw < n_camw)
        camera_wave(cw, cams, pp, pts, pt_idx, uv, cam_ptr, cam_obs, loss_s, splits, part, U, gc,
                    nullptr, 0);
}
__global__ __launch_bounds__(256) void ba_obs_kernel(
    int n_obs, const double* __restrict__ cams, const double* __restrict__ pp,
    const double* __restrict__ pts, const int32_t* __restrict__ cam_idx,
    const int32_t* __restrict__ pt_idx, const int32_t* __restrict__ pt_ptr,
    const double* __restrict__ uv, double loss_s, double* __restrict__ W, double* __restrict__ res,
    double* __restrict__ V, double* __restrict__ gp, double* __restrict__ seg,
    int32_t* __restrict__ seg_pt, double* __restrict__ cost_blk) {
    __shared__ double lds[4 * OBS_LDS];
    sfm::ChunkOff none{};
    obs_block(blockIdx.x, n_obs, cams, pp, pts, cam_idx, pt_idx, pt_ptr, uv, loss_s, W, res, V, gp,
              seg, seg_pt, cost_blk, lds, 0, none, none);
}
#endif

__device__ __forceinline__ void chunk_final_one(int g, int n_cam, int nck, int exp,
                                                const double* __restrict__ part,
                                                double* __restrict__ U, double* __restrict__ gc);

// Chunk mode: chunk k's cost = the fixed-order sum of its 256-observation blocks' shares
// blk[vst_k / 256, vst_{k+1} / 256) (chunks start at block boundaries of the virtual index space,
// so the blocks and this order depend only on the chunk): lane-strided, then an xor tree; one wave
// per chunk (waves w, w + nwave, ... of the calling block).  exp = 0: cost[0] = the canonical tree
// over the chunks; exp = 1: cost[k] per chunk.  Called by every thread of the block.
__device__ __forceinline__ void chunk_cost_finish(int nck, int exp, const sfm::ChunkOff& vst,
                                                  const double* __restrict__ blk,
                                                  double* __restrict__ cost, int nwave) {
    __shared__ double kc[SFM_BA_MAX_CHUNKS];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int k = tid >> 6; k < nck; k += nwave) {
        const int b0 = vst.v[k] >> 8, b1 = vst.v[k + 1] >> 8;
        double s = 0.0;
#pragma unroll 4
        for (int b = b0 + lane; b < b1; b += 64) s += blk[b];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) kc[k] = s;
    }
    __syncthreads();
    if (tid != 0) return;
    if (exp) {
        for (int k = 0; k < nck; ++k) cost[k] = kc[k];
        return;
    }
    double a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = k < nck ? kc[k] : 0.0;
    cost[0] = sfm::chunk_tree16(a);
}

// Finish work (256-thread block fb): points spanning waves (the point whose tail record wave g
// wrote owns tail + the head records of the following waves up to its last observation, fixed
// order), zero V_p / g_p for points without observations, and (block 0) the cost as a
// fixed-order sum of the per-block shares.  Chunk mode: block 0 forms the chunk costs
// (chunk_cost_finish) and thread g < n_cam * 44 the camera sum g from the chunk partials.
__global__ __launch_bounds__(256) void ba_finish_kernel(
    int n_wave, int n_blk, int n_pt, const int32_t* __restrict__ pt_ptr,
    const double* __restrict__ seg, const int32_t* __restrict__ seg_pt, double* __restrict__ V,
    double* __restrict__ gp, const double* __restrict__ cost_blk, double* __restrict__ cost,
    int nck, sfm::ChunkOff cobs, sfm::ChunkOff vst, int n_cam, int exp,
    const double* __restrict__ part, double* __restrict__ U, double* __restrict__ gc) {
    const int fb = blockIdx.x;
    const int tid = threadIdx.x;
    const int g = fb * 256 + tid;
    if (nck > 0) {
        if (fb == 0) chunk_cost_finish(nck, exp, vst, cost_blk, cost, 4);
        if (g < n_cam * NU) chunk_final_one(g, n_cam, nck, exp, part, U, gc);
    } else if (fb == 0) {
        __shared__ double red[4];
        double s = 0.0;  // fixed order (w = tid, tid + 256, ...); unrolled so the loads overlap
#pragma unroll 8
        for (int w = tid; w < n_blk; w += 256) s += cost_blk[w];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_down(s, off, 64);
        if ((tid & 63) == 0) red[tid >> 6] = s;
        __syncthreads();
        if (tid == 0) cost[0] = ((red[0] + red[1]) + red[2]) + red[3];
    }
    if (g < n_pt && pt_ptr[g] == pt_ptr[g + 1]) {
        double z[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) z[k] = 0.0;
        write_point(V, gp, g, z);
    }
    if (g < n_wave) {
        const int p = seg_pt[g * 2 + 1];
        if (p >= 0) {
            double a[NV];
#pragma unroll
            for (int k = 0; k < NV - 1; ++k) a[k] = seg[((size_t)g * 2 + 1) * NV + k];
            a[NV - 1] = 0.0;
            int vl = pt_ptr[p + 1] - 1;   // the point's last observation, as a virtual index
            if (nck > 0) {
                int c0, c1, v0, v1;
                sfm::chunk_of(vl, nck, cobs, cobs, c0, c1);
                sfm::chunk_of(vl, nck, cobs, vst, v0, v1);
                vl = v0 + (vl - c0);
            }
            const int w_last = vl >> 6;
            for (int w = g + 1; w <= w_last; ++w) {
#pragma unroll
                for (int k = 0; k < NV - 1; ++k) a[k] += seg[((size_t)w * 2) * NV + k];
            }
            write_point(V, gp, p, a);
        }
    }
}

// Few cameras (splits > 1): U_c / g_c component = the camera's split partials summed in order.
__global__ __launch_bounds__(256) void ba_final_kernel(int n_cam, int splits,
                                                       const double* __restrict__ part,
                                                       double* __restrict__ U,
                                                       double* __restrict__ gc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_cam * NU) return;
    const int c = g / NU, k = g - c * NU;
    double v = 0.0;
    for (int sp = 0; sp < splits; ++sp) v += part[((size_t)c * splits + sp) * NU + k];
    if (k >= 36) {
        gc[8 * (size_t)c + k - 36] = v;
    } else {
        int i = 0, t = k;
        while (t >= 8 - i) { t -= 8 - i; ++i; }
        const int j = i + t;
        U[64 * (size_t)c + 8 * i + j] = v;
        U[64 * (size_t)c + 8 * j + i] = v;
    }
}

// Chunk mode, thread g = (camera, sum t) (run by ba_finish_kernel).  exp = 0: U_c / g_c = the
// canonical tree over the chunk partials; exp = 1 (a shard): the chunk partials themselves,
// U [nck][n_cam][64], gc [nck][n_cam][8].
__device__ __forceinline__ void chunk_final_one(int g, int n_cam, int nck, int exp,
                                                const double* __restrict__ part,
                                                double* __restrict__ U, double* __restrict__ gc) {
    const int c = g / NU, k = g - c * NU;
    int i = 0, j = 0;
    if (k < 36) {
        int t = k;
        while (t >= 8 - i) { t -= 8 - i; ++i; }
        j = i + t;
    }
    auto put = [&](int slot, double v) {
        if (k >= 36) {
            gc[8 * ((size_t)slot * n_cam + c) + k - 36] = v;
        } else {
            double* u = U + 64 * ((size_t)slot * n_cam + c);
            u[8 * i + j] = v;
            u[8 * j + i] = v;
        }
    };
    if (exp) {
        for (int ch = 0; ch < nck; ++ch) put(ch, part[((size_t)c * nck + ch) * NU + k]);
        return;
    }
    double a[16];
#pragma unroll
    for (int ch = 0; ch < 16; ++ch) a[ch] = ch < nck ? part[((size_t)c * nck + ch) * NU + k] : 0.0;
    put(0, sfm::chunk_tree16(a));
}

// ---- LM support: cost at trial parameters, parameter update -----------------

// Thread per observation: 0.5 rho, summed per block in a fixed order; blocks summed by the
// ba_cost_final kernel in a fixed order.
__global__ __launch_bounds__(256) void ba_cost_kernel(
    int n_obs, const double* __restrict__ cams, const double* __restrict__ pp,
    const double* __restrict__ pts, const int32_t* __restrict__ cam_idx,
    const int32_t* __restrict__ pt_idx, const double* __restrict__ uv, double loss_s,
    double* __restrict__ part) {
    __shared__ double red[4];
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    double h = 0.0;
    if (o < n_obs) {
        const int c = cam_idx[o], p = pt_idx[o];
        const double* cam = cams + 8 * (size_t)c;
        double R[9];
        rotmat(cam[0], cam[1], cam[2], R);
        const double X0 = pts[3 * (size_t)p], X1 = pts[3 * (size_t)p + 1], X2 = pts[3 * (size_t)p + 2];
        double P[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) P[i] = (R[3 * i] * X0 + R[3 * i + 1] * X1 + R[3 * i + 2] * X2) + cam[3 + i];
        const double iz = 1.0 / P[2];
        const double p0 = P[0] * iz, p1 = P[1] * iz;
        const double f = cam[6], k1 = cam[7];
        const double d = 1.0 + k1 * (p0 * p0 + p1 * p1);
        const double e0 = f * d * p0 + pp[2 * (size_t)c] - uv[2 * (size_t)o];
        const double e1 = f * d * p1 + pp[2 * (size_t)c + 1] - uv[2 * (size_t)o + 1];
        const double e = e0 * e0 + e1 * e1;
        double rho = e;
        if (loss_s > 0.0) {
            const double s2 = loss_s * loss_s;
            rho = s2 * log1p(e / s2);
        }
        h = 0.5 * rho;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) h += __shfl_down(h, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// Chunk mode: 0.5 rho at trial parameters over the virtual index space of sfm_ba_jtj (every chunk
// starts at a 256-observation block boundary, chunk_layout): block b -> the fixed-order share of
// its (at most 256) observations of one chunk, part[b]; ba_cost_chunk_final then forms the chunk
// costs exactly as ba_finish_kernel forms the linearisation's (chunk_cost_finish).
__device__ __forceinline__ double half_rho(const double* __restrict__ cams, const double* __restrict__ pp,
                                           const double* __restrict__ pts, int c, int p, double u,
                                           double v, double loss_s) {
    const double* cam = cams + 8 * (size_t)c;
    double R[9];
    rotmat(cam[0], cam[1], cam[2], R);
    const double X0 = pts[3 * (size_t)p], X1 = pts[3 * (size_t)p + 1], X2 = pts[3 * (size_t)p + 2];
    double P[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) P[i] = (R[3 * i] * X0 + R[3 * i + 1] * X1 + R[3 * i + 2] * X2) + cam[3 + i];
    const double iz = 1.0 / P[2];
    const double p0 = P[0] * iz, p1 = P[1] * iz;
    const double f = cam[6], k1 = cam[7];
    const double d = 1.0 + k1 * (p0 * p0 + p1 * p1);
    const double e0 = f * d * p0 + pp[2 * (size_t)c] - u;
    const double e1 = f * d * p1 + pp[2 * (size_t)c + 1] - v;
    const double e = e0 * e0 + e1 * e1;
    double rho = e;
    if (loss_s > 0.0) {
        const double s2 = loss_s * loss_s;
        rho = s2 * log1p(e / s2);
    }
    return 0.5 * rho;
}

__global__ __launch_bounds__(256) void ba_cost_chunk_kernel(
    int nck, sfm::ChunkOff cobs, sfm::ChunkOff vst, const double* __restrict__ cams,
    const double* __restrict__ pp, const double* __restrict__ pts,
    const int32_t* __restrict__ cam_idx, const int32_t* __restrict__ pt_idx,
    const double* __restrict__ uv, double loss_s, double* __restrict__ part) {
    __shared__ double red[4];
    const int vo = blockIdx.x * 256 + threadIdx.x;
    int c0, c1, v0, v1;   // chunks start at block boundaries: the block decides (scalar lookup)
    sfm::chunk_of((int)blockIdx.x << 8, nck, vst, cobs, c0, c1);
    sfm::chunk_of((int)blockIdx.x << 8, nck, vst, vst, v0, v1);
    const int o = c0 + (vo - v0);
    double h = 0.0;
    if (o < c1)
        h = half_rho(cams, pp, pts, cam_idx[o], pt_idx[o], uv[2 * (size_t)o], uv[2 * (size_t)o + 1],
                     loss_s);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) h += __shfl_down(h, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// One block of 16 waves: wave k forms chunk k's cost (chunk_cost_finish).
__global__ __launch_bounds__(1024) void ba_cost_chunk_final(int nck, int exp, sfm::ChunkOff vst,
                                                            const double* __restrict__ part,
                                                            double* __restrict__ cost) {
    chunk_cost_finish(nck, exp, vst, part, cost, 16);
}

__global__ __launch_bounds__(256) void ba_chunk_tree_kernel(int nck, long long n,
                                                            const double* __restrict__ parts,
                                                            double* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = k < nck ? parts[(size_t)k * n + i] : 0.0;
    out[i] = sfm::chunk_tree16(a);
}

__global__ __launch_bounds__(1024) void ba_cost_final(int n_blk, const double* __restrict__ part,
                                                      double* __restrict__ cost) {
    __shared__ double red[16];
    const int tid = threadIdx.x;
    double a = 0.0;
    for (int k = tid; k < n_blk; k += 1024) a += part[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) a += __shfl_down(a, off, 64);
    if ((tid & 63) == 0) red[tid >> 6] = a;
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int w = 0; w < 16; ++w) s += red[w];
        *cost = s;
    }
}

// cams ⊕ dc: R <- exp([δr]x) R (the left increment the Jacobians are taken in), t, f, k1
// additive; points additive; δr = 0 exactly keeps r.  Thread per camera / point.  Mirrors oracle/ba_lm.py update().
__global__ __launch_bounds__(256) void ba_update_kernel(int n_cam, const double* __restrict__ cams,
                                                        const double* __restrict__ dc, int n_pt,
                                                        const double* __restrict__ pts,
                                                        const double* __restrict__ dp,
                                                        double* __restrict__ cams_out,
                                                        double* __restrict__ pts_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_cam) {
        const double* c = cams + 8 * (size_t)i;
        const double* d = dc + 8 * (size_t)i;
        double A[9], B[9], R[9];
        rotmat(d[0], d[1], d[2], A);
        rotmat(c[0], c[1], c[2], B);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                R[3 * r + k] = A[3 * r] * B[k] + A[3 * r + 1] * B[3 + k] + A[3 * r + 2] * B[6 + k];
        // log map, stable near 0 and pi
        const double cs = fmin(fmax(0.5 * ((R[0] + R[4] + R[8]) - 1.0), -1.0), 1.0);
        const double w0 = R[7] - R[5], w1 = R[2] - R[6], w2 = R[3] - R[1];
        const double sn = 0.5 * sqrt(w0 * w0 + w1 * w1 + w2 * w2);
        const double th = atan2(sn, cs);
        double o0, o1, o2;
        if (sn > 1e-7) {
            const double k = th / (2.0 * sn);
            o0 = w0 * k; o1 = w1 * k; o2 = w2 * k;
        } else if (cs > 0.0) {
            o0 = 0.5 * w0; o1 = 0.5 * w1; o2 = 0.5 * w2;
        } else {  // th ~ pi: axis from the largest diagonal column of (R + I) / 2
            const double B0 = 0.5 * (R[0] + 1.0), B4 = 0.5 * (R[4] + 1.0), B8 = 0.5 * (R[8] + 1.0);
            const int j = (B0 >= B4 && B0 >= B8) ? 0 : (B4 >= B8 ? 1 : 2);
            const double bjj = j == 0 ? B0 : (j == 1 ? B4 : B8);
            const double sq = sqrt(bjj);
            double a0 = (j == 0 ? B0 : 0.5 * R[j]) / sq;          // column j of B = (R+I)/2
            double a1 = (j == 1 ? B4 : 0.5 * R[3 + j]) / sq;
            double a2 = (j == 2 ? B8 : 0.5 * R[6 + j]) / sq;
            if (a0 * w0 + a1 * w1 + a2 * w2 < 0.0) { a0 = -a0; a1 = -a1; a2 = -a2; }
            const double n = sqrt(a0 * a0 + a1 * a1 + a2 * a2);
            o0 = th * a0 / n; o1 = th * a1 / n; o2 = th * a2 / n;
        }
        double* out = cams_out + 8 * (size_t)i;
        // δr = 0 exactly (a held rotation): exp(0) = I, keep r bit for bit instead of the
        // rounding of the log map of R(r)
        const bool keep = d[0] == 0.0 && d[1] == 0.0 && d[2] == 0.0;
        out[0] = keep ? c[0] : o0; out[1] = keep ? c[1] : o1; out[2] = keep ? c[2] : o2;
#pragma unroll
        for (int k = 3; k < 8; ++k) out[k] = c[k] + d[k];
    }
    if (i < n_pt) {
#pragma unroll
        for (int k = 0; k < 3; ++k) pts_out[3 * (size_t)i + k] = pts[3 * (size_t)i + k] + dp[3 * (size_t)i + k];
    }
}

// Chunk mode: cobs = the chunks' observation offsets, vst = their starts in the virtual index
// space in which every chunk begins at a 256-observation block boundary (so an observation wave /
// block, and every order built on them, depends only on its chunk); returns the virtual count.
// Chunk mode: camera waves per camera (each takes chunks g, g + G, ...): enough for
// CHUNK_WAVE_TARGET waves in all, as the plain form's SPLIT_TARGET (so G = 1 from 256 cameras on).
// Round 6: with cfg5's local visibility (a camera's observations in 1.06 of 8 chunks) G = 8 kept
// 8 waves per camera, 7 of them idle, occupying the CU slots the observation stream needs: the
// final model's K3 0.120-0.125 ms at G = 8, 0.117-0.118 at G = 2, 0.107-0.108 at G = 1
// (plain 0.101-0.107); random visibility, where every camera touches every chunk, 0.117 / 0.110 /
// 0.118 (profiles/r06/ba_study/s17_*).  (Round 5's 4096 target measured 119 vs 126 us on the
// random-visibility problem.)  SFM_BA_CKW overrides (A/B).  Any G gives the same bits (a chunk's
// partial does not depend on which wave forms it).
constexpr int CHUNK_WAVE_TARGET = 256;
int chunk_waves(int nck, int n_cam) {
    static const int env = [] {
        const char* e = getenv("SFM_BA_CKW");
        return e ? atoi(e) : 0;
    }();
    const int g = env > 0 ? env : (CHUNK_WAVE_TARGET + n_cam - 1) / std::max(n_cam, 1);
    return std::max(1, std::min(nck, g));
}

int chunk_layout(const sfm_ctx* ctx, sfm::ChunkOff& cobs, sfm::ChunkOff& vst) {
    const int nck = ctx->ba_nchunk;
    vst.v[0] = 0;
    for (int k = 0; k < nck; ++k) {
        cobs.v[k] = ctx->ba_chunk_obs[k];
        vst.v[k + 1] = vst.v[k] + ((ctx->ba_chunk_obs[k + 1] - ctx->ba_chunk_obs[k] + 255) & ~255);
    }
    cobs.v[nck] = ctx->ba_chunk_obs[nck];
    return vst.v[nck];
}

}  // namespace

extern "C" int sfm_ba_jtj(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* pp,
                          int32_t n_pt, const double* pts, int32_t n_obs, const int32_t* cam_idx,
                          const int32_t* pt_idx, const double* uv, const int32_t* pt_ptr,
                          const int32_t* cam_ptr, const int32_t* cam_obs, double loss_s,
                          double* U, double* V, double* W, double* gc, double* gp, double* res,
                          double* cost) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ba_jtj: ctx is NULL");
    SFM_REQUIRE(n_cam >= 0 && n_pt >= 0 && n_obs >= 0, "sfm_ba_jtj: negative size");
    SFM_REQUIRE(cost != nullptr, "sfm_ba_jtj: cost is NULL");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // chunk mode, export form: U / gc / cost hold one slot per local chunk
    const size_t nslot = (ctx->ba_nchunk > 0 && ctx->ba_ntotal > 0) ? ctx->ba_nchunk : 1;
    if (ctx->ba_nchunk > 0)
        SFM_REQUIRE(ctx->ba_chunk_pt[ctx->ba_nchunk] == n_pt && ctx->ba_chunk_obs[ctx->ba_nchunk] == n_obs,
                    "sfm_ba_jtj: chunk offsets do not match n_pt / n_obs");
    if (n_pt == 0 || n_cam == 0) {
        SFM_HIP_CHECK(hipMemsetAsync(cost, 0, sizeof(double) * nslot, st));
        if (n_cam > 0) {
            SFM_HIP_CHECK(hipMemsetAsync(U, 0, sizeof(double) * 64 * n_cam * nslot, st));
            SFM_HIP_CHECK(hipMemsetAsync(gc, 0, sizeof(double) * 8 * n_cam * nslot, st));
        }
        if (n_pt > 0) {
            SFM_HIP_CHECK(hipMemsetAsync(V, 0, sizeof(double) * 9 * n_pt, st));
            SFM_HIP_CHECK(hipMemsetAsync(gp, 0, sizeof(double) * 3 * n_pt, st));
        }
        return SFM_OK;
    }
    SFM_REQUIRE(cams && pp && pts && cam_idx && pt_idx && uv && pt_ptr && cam_ptr && cam_obs && U &&
                    V && W && gc && gp && res,
                "sfm_ba_jtj: NULL array");
    // chunk mode: the observation blocks tile a virtual index space in which every chunk starts at
    // a multiple of 256 (obs_block); cobs / vst = the chunks' real / virtual starts
    sfm::ChunkOff cobs{}, vst{};
    const int n_vobs = ctx->ba_nchunk > 0 ? chunk_layout(ctx, cobs, vst) : n_obs;
    // workspace: segment records (2 per wave) | their point ids | cost per block | camera partials
    const int n_wave = (n_vobs + 63) / 64;
    const int n_obsb = (n_vobs + 255) / 256;
    // few cameras: split each camera's observations so the camera waves still fill the chip;
    // chunk mode: G waves per camera, each a share of the chunks (camera_wave), at least
    // SPLIT_TARGET camera waves in all
    const bool ck = ctx->ba_nchunk > 0;
    const int splits = ck ? chunk_waves(ctx->ba_nchunk, n_cam)
                          : std::max(1, std::min(16, (SPLIT_TARGET + n_cam - 1) / n_cam));
    SFM_REQUIRE(!ck || ctx->ba_cam_bounds, "sfm_ba_jtj: chunk mode without cam_bounds");
    const size_t sb = sfm::align_up(sizeof(double) * NV * 2 * (size_t)std::max(n_wave, 1), 256);
    const size_t ib = sfm::align_up(sizeof(int32_t) * 2 * (size_t)std::max(n_wave, 1), 256);
    const size_t cb = sfm::align_up(sizeof(double) * (size_t)std::max(n_obsb, 1), 256);
    const size_t pb = sfm::align_up(sizeof(double) * NU * (size_t)n_cam * (ck ? ctx->ba_nchunk : splits), 256);
    char* ws = (char*)sfm::workspace(ctx, sb + ib + cb + pb + 1024);
    if (!ws) return SFM_ERR_NOMEM;
    double* seg = (double*)ws;
    int32_t* seg_pt = (int32_t*)(ws + sb);
    double* cost_blk = (double*)(ws + sb + ib);
    double* part = (double*)(ws + sb + ib + cb);
    // camera waves (four per block) + observation blocks in one launch, then the finish blocks
#ifdef BA_ABL_OBSONLY  // ablation (timing only): observation blocks alone
    const int n_camw = 0;
#else
    const int n_camw = n_cam * splits * CH;
#endif
    const int n_camb = (n_camw + 3) / 4;
#ifdef BA_ABL_CAMONLY  // ablation (timing only): camera waves alone
    const int n_ob_launch = 0;
#else
    const int n_ob_launch = n_obsb;
#endif
#ifdef BA_SEQ
    hipLaunchKernelGGL(ba_cam_kernel, dim3(n_camb), dim3(256), 0, st, n_camw, cams, pp, pts, pt_idx,
                       uv, cam_ptr, cam_obs, loss_s, splits, part, U, gc);
    if (n_ob_launch > 0)
        hipLaunchKernelGGL(ba_obs_kernel, dim3(n_ob_launch), dim3(256), 0, st, n_obs, cams, pp, pts,
                           cam_idx, pt_idx, pt_ptr, uv, loss_s, W, res, V, gp, seg, seg_pt,
                           cost_blk);
#else
    hipLaunchKernelGGL(ba_jtj_kernel, dim3(n_camb + n_ob_launch), dim3(256), 0, st, n_camb, n_camw,
                       n_obs, cams, pp, pts, cam_idx, pt_idx, pt_ptr, uv, cam_ptr, cam_obs, loss_s,
                       splits, part, U, gc, W, res, V, gp, seg, seg_pt, cost_blk,
                       ck ? ctx->ba_cam_bounds : nullptr, ctx->ba_nchunk, cobs, vst);
#endif
    SFM_HIP_CHECK(hipGetLastError());
    const int nw = n_obs > 0 ? n_wave : 0;
    // chunk mode: the finish blocks also form U / g_c and the cost from the chunk partials (the
    // canonical tree, or exported per chunk for the caller's exchange)
    const int n_fin = std::max({(nw + 255) / 256, (n_pt + 255) / 256, ck ? (n_cam * NU + 255) / 256 : 0, 1});
    hipLaunchKernelGGL(ba_finish_kernel, dim3(n_fin), dim3(256), 0, st, nw, n_obs > 0 ? n_obsb : 0,
                       n_pt, pt_ptr, seg, seg_pt, V, gp, cost_blk, cost, ctx->ba_nchunk, cobs, vst,
                       n_cam, ctx->ba_ntotal > 0 ? 1 : 0, part, U, gc);
    SFM_HIP_CHECK(hipGetLastError());
    if (ck) return SFM_OK;
    if (splits > 1) {
        hipLaunchKernelGGL(ba_final_kernel, dim3((n_cam * NU + 255) / 256), dim3(256), 0, st,
                           n_cam, splits, part, U, gc);
        SFM_HIP_CHECK(hipGetLastError());
    }
    return SFM_OK;
}

extern "C" int sfm_ba_cost(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* pp,
                           int32_t n_pt, const double* pts, int32_t n_obs, const int32_t* cam_idx,
                           const int32_t* pt_idx, const double* uv, double loss_s, double* cost) {
    SFM_REQUIRE(ctx != nullptr && cost != nullptr, "sfm_ba_cost: ctx/cost is NULL");
    SFM_REQUIRE(n_cam >= 0 && n_pt >= 0 && n_obs >= 0, "sfm_ba_cost: negative size");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (n_obs == 0) {
        const size_t nslot = (ctx->ba_nchunk > 0 && ctx->ba_ntotal > 0) ? ctx->ba_nchunk : 1;
        SFM_HIP_CHECK(hipMemsetAsync(cost, 0, sizeof(double) * nslot, st));
        return SFM_OK;
    }
    SFM_REQUIRE(cams && pp && pts && cam_idx && pt_idx && uv, "sfm_ba_cost: NULL array");
    if (ctx->ba_nchunk > 0) {   // chunk mode (sfm_ba_set_chunks): chunk partials, tree or export
        const int nck = ctx->ba_nchunk;
        SFM_REQUIRE(ctx->ba_chunk_obs[nck] == n_obs, "sfm_ba_cost: chunk offsets do not match n_obs");
        sfm::ChunkOff cobs{}, vst{};
        const int nvb = chunk_layout(ctx, cobs, vst) / 256;
        double* kpart = (double*)sfm::workspace(ctx, sizeof(double) * (size_t)nvb + 256);
        if (!kpart) return SFM_ERR_NOMEM;
        hipLaunchKernelGGL(ba_cost_chunk_kernel, dim3(nvb), dim3(256), 0, st, nck, cobs, vst, cams,
                           pp, pts, cam_idx, pt_idx, uv, loss_s, kpart);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(ba_cost_chunk_final, dim3(1), dim3(1024), 0, st, nck,
                           ctx->ba_ntotal > 0 ? 1 : 0, vst, kpart, cost);
        SFM_HIP_CHECK(hipGetLastError());
        return SFM_OK;
    }
    const int nb = (n_obs + 255) / 256;
    double* part = (double*)sfm::workspace(ctx, sizeof(double) * (size_t)nb + 256);
    if (!part) return SFM_ERR_NOMEM;
    hipLaunchKernelGGL(ba_cost_kernel, dim3(nb), dim3(256), 0, st, n_obs, cams, pp, pts, cam_idx,
                       pt_idx, uv, loss_s, part);
    SFM_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ba_cost_final, dim3(1), dim3(1024), 0, st, nb, part, cost);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

extern "C" int sfm_ba_update(sfm_ctx* ctx, int32_t n_cam, const double* cams, const double* dc,
                             int32_t n_pt, const double* pts, const double* dp, double* cams_out,
                             double* pts_out) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ba_update: ctx is NULL");
    SFM_REQUIRE(n_cam >= 0 && n_pt >= 0, "sfm_ba_update: negative size");
    const int n = std::max(n_cam, n_pt);
    if (n == 0) return SFM_OK;
    SFM_REQUIRE((n_cam == 0 || (cams && dc && cams_out)) && (n_pt == 0 || (pts && dp && pts_out)),
                "sfm_ba_update: NULL array");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(ba_update_kernel, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, n_cam,
                       cams, dc, n_pt, pts, dp, cams_out, pts_out);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

extern "C" int sfm_ba_set_chunks(sfm_ctx* ctx, int32_t n_chunk, const int32_t* chunk_pt,
                                 const int32_t* chunk_obs, int32_t n_total,
                                 const int32_t* cam_bounds) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ba_set_chunks: ctx is NULL");
    SFM_REQUIRE(n_chunk >= 0 && n_chunk <= SFM_BA_MAX_CHUNKS,
                "sfm_ba_set_chunks: n_chunk must be in [0, 16]");
    if (n_chunk == 0) {
        ctx->ba_nchunk = ctx->ba_ntotal = 0;
        ctx->ba_cam_bounds = nullptr;
        return SFM_OK;
    }
    SFM_REQUIRE(chunk_pt && chunk_obs && cam_bounds, "sfm_ba_set_chunks: NULL array");
    SFM_REQUIRE(n_total == 0 || (n_total >= n_chunk && n_total <= SFM_BA_MAX_CHUNKS),
                "sfm_ba_set_chunks: n_total must be 0 or in [n_chunk, 16]");
    SFM_REQUIRE(chunk_pt[0] == 0 && chunk_obs[0] == 0, "sfm_ba_set_chunks: offsets must start at 0");
    for (int k = 0; k < n_chunk; ++k)
        SFM_REQUIRE(chunk_pt[k + 1] >= chunk_pt[k] && chunk_obs[k + 1] >= chunk_obs[k],
                    "sfm_ba_set_chunks: offsets must be non-decreasing");
    ctx->ba_nchunk = n_chunk;
    ctx->ba_ntotal = n_total;
    for (int k = 0; k <= n_chunk; ++k) {
        ctx->ba_chunk_pt[k] = chunk_pt[k];
        ctx->ba_chunk_obs[k] = chunk_obs[k];
    }
    ctx->ba_cam_bounds = cam_bounds;
    return SFM_OK;
}

extern "C" int sfm_ba_chunk_tree(sfm_ctx* ctx, int32_t n_total, int64_t n, const double* parts,
                                 double* out) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ba_chunk_tree: ctx is NULL");
    SFM_REQUIRE(n_total >= 1 && n_total <= SFM_BA_MAX_CHUNKS && n >= 0,
                "sfm_ba_chunk_tree: bad size");
    if (n == 0) return SFM_OK;
    SFM_REQUIRE(parts && out, "sfm_ba_chunk_tree: NULL array");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(ba_chunk_tree_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, n_total, (long long)n, parts, out);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
