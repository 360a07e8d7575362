// Bundle-adjustment step solve (K4): the damped normal
// equations of the J^TJ blocks that sfm_ba_jtj builds, reduced to the cameras by the Schur
// complement and solved by block-Jacobi preconditioned CG without forming S (Ceres'
// ITERATIVE_SCHUR + SCHUR_JACOBI):
//     [U_d  W ; Wᵀ  V_d] [δc; δp] = -[g_c; g_p],   A_d = A + λ·clamp(diag A, 1e-6, 1e32)
//     S δc = b,  S = U_d - Σ_o W_o V_d⁻¹ W_oᵀ,  b = -g_c + Σ_o W_o V_d⁻¹ g_p
//     δp = V_d⁻¹ (-g_p - Σ_o W_oᵀ δc)
// Restated on the CPU by oracle/ba_lm.py (schur_pcg), which the GPU tests compare against.
//
// fp64, deterministic (every sum has a fixed order; no float atomics).  Kernels:
//   bas_point_setup     thread per point: V_d⁻¹ (3x3, adjugate), v_g = V_d⁻¹ g_p
//   bas_camera_setup    block per camera: diagonal block of S (36 sums over the camera's
//                       observations), its inverse (8x8 Cholesky) = the preconditioner, b, and
//                       the CG start x = 0, r = b, z = M r, p = z
//   CG iteration (3 launches, no host synchronisation; converged iterations exit at once):
//     bas_pcg_point     8 lanes per point: t_p = V_d⁻¹ Σ_o W_oᵀ p_c (SoA W), u_o = W_o t_p
//     bas_pcg_camera    block per camera: q_c = U_d p_c - Σ_o u_o       (64 B per observation)
//     bas_pcg_vec       thread per camera component: α, x, r, z = M r, partial r·z, r·r
//   sharded (sfm_ba_solve_stage): bas_pcg_point, bas_pcg_camera phase 1 (-> comm), the caller's
//     all-reduce, then bas_pcg_finish_vec (q from comm, p·q, α and the vector update in one launch)
//   bas_backsub        8 lanes per point: δp, and the point terms of gᵀδ and δᵀ(JᵀJ)δ
//   bas_model           one block: gᵀδ, δᵀ(JᵀJ)δ (LM predicted decrease), iterations, |r|/|b|
// HBM: a CG iteration reads W once (192 B per observation), writes and reads u (2 x 64 B) plus
// the camera/point vectors; this stage is HBM-bound.
#include <algorithm>

#include "sfm_internal.h"

namespace {

constexpr double DIAG_MIN = 1e-6, DIAG_MAX = 1e32;
constexpr int CT = 256;  // threads per camera block
// Chunk mode (sfm_ba_set_chunks) camera passes: the camera's chunks one after the other, each over
// the whole block (block-strided from the chunk's start, then block_sum) — a camera's observations
// sit in one or two chunks (points are chunked by id and a camera sees a local set), so spreading
// the chunks over lane groups would leave most groups idle.  The association of a chunk's sum
// depends only on that chunk (never on how many chunks the calling rank holds); empty chunks
// are zero without a reduction.

struct PcgState {
    double beta;    // β_k of the current iteration (published by the previous iteration's vector
                    // kernel, or bas_pcg_init for k = 0)
    double rz;      // r·z of the current iterate
    double bb;      // |b|^2
    double rr;      // |r|^2 after the last step
    int32_t iter;   // iterations done
    int32_t done;   // converged (or max_iter reached)
    uint32_t cnt;   // blocks of the current vector kernel that finished (last-block publish)
};

__device__ __forceinline__ double dclamp(double d) { return fmin(fmax(d, DIAG_MIN), DIAG_MAX); }

// Fixed-order block sum over CT threads of n <= 64 values per thread (each wave's recursive-halving
// sum, then the 4 wave partials in order).  Result in out[i] for i < n after the call.
template <int N>
__device__ __forceinline__ void block_sum(double (&a)[N], double (*red)[N], double* out) {
    static_assert(CT == 256, "block_sum: four waves");
    const int tid = threadIdx.x;
    int idx;
    if (sfm::wave_halving_sum<N>(a, tid & 63, idx)) red[tid >> 6][idx] = a[0];
    __syncthreads();
    if (tid < N) out[tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    __syncthreads();
}

// ---- setup -------------------------------------------------------------------------------------

// Points with more observations than this are handled by a wave each in the CG point pass
// (long tracks: with 8 lanes per point a wave would wait for its longest point).
constexpr int LONG_OBS = 64;
constexpr int LONG_BLOCKS = 64;  // extra point-pass blocks (4 waves each) that take the long points

__device__ __forceinline__ void soa_one(int e, int n_obs, const int32_t* __restrict__ cam_obs,
                                        const int32_t* __restrict__ pt_idx,
                                        const double* __restrict__ W, double* __restrict__ Wp,
                                        int32_t* __restrict__ ptc);

// Blocks [0, pblk): a point each thread (V_d⁻¹, V_d⁻¹ g_p, the long-track list); blocks from pblk
// on: bas_soa's work for observation e (one launch for both, they are independent).
__global__ __launch_bounds__(256) void bas_point_setup(int n_pt, const int32_t* __restrict__ pt_ptr,
                                                       const double* __restrict__ V,
                                                       const double* __restrict__ gp, double lam,
                                                       double* __restrict__ Vinv,
                                                       double* __restrict__ vg,
                                                       int32_t* __restrict__ long_list,
                                                       int32_t* __restrict__ long_cnt, int pblk,
                                                       int n_obs, const int32_t* __restrict__ cam_obs,
                                                       const int32_t* __restrict__ pt_idx,
                                                       const double* __restrict__ W,
                                                       double* __restrict__ Wp,
                                                       int32_t* __restrict__ ptc) {
    if ((int)blockIdx.x >= pblk) {
        const int e = ((int)blockIdx.x - pblk) * blockDim.x + threadIdx.x;
        if (e < n_obs) soa_one(e, n_obs, cam_obs, pt_idx, W, Wp, ptc);
        return;
    }
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pt) return;
    if (pt_ptr[p + 1] - pt_ptr[p] > LONG_OBS)  // order of the list is irrelevant (points independent)
        long_list[atomicAdd(long_cnt, 1)] = p;
    double* Vi = Vinv + 9 * (size_t)p;
    double* g = vg + 3 * (size_t)p;
    if (pt_ptr[p + 1] == pt_ptr[p]) {  // unobserved point: δp = 0
#pragma unroll
        for (int k = 0; k < 9; ++k) Vi[k] = 0.0;
        g[0] = g[1] = g[2] = 0.0;
        return;
    }
    const double* Vp = V + 9 * (size_t)p;
    const double a = Vp[0] + lam * dclamp(Vp[0]), b = Vp[1], c = Vp[2];
    const double d = Vp[4] + lam * dclamp(Vp[4]), e = Vp[5];
    const double f = Vp[8] + lam * dclamp(Vp[8]);
    // symmetric [[a b c][b d e][c e f]]: adjugate / determinant
    const double A0 = d * f - e * e, A1 = c * e - b * f, A2 = b * e - c * d;
    const double A4 = a * f - c * c, A5 = b * c - a * e, A8 = a * d - b * b;
    const double inv = 1.0 / (a * A0 + b * A1 + c * A2);
    const double m[9] = {A0 * inv, A1 * inv, A2 * inv, A1 * inv, A4 * inv,
                         A5 * inv, A2 * inv, A5 * inv, A8 * inv};
#pragma unroll
    for (int k = 0; k < 9; ++k) Vi[k] = m[k];
    const double* gg = gp + 3 * (size_t)p;
#pragma unroll
    for (int i = 0; i < 3; ++i) g[i] = m[3 * i] * gg[0] + m[3 * i + 1] * gg[1] + m[3 * i + 2] * gg[2];
}

// Component-major (SoA) copy of W for the point-major passes: Wp[24][n_obs] in observation
// (point-major) order, so bas_pcg_point and bas_backsub read W with lane-contiguous 8-B loads
// instead of 192-B rows per lane; ptc = pt_idx in camera-major order (cam_obs) for the camera
// setup.  The camera side never needs W again after the setup: the point pass hands it
// u_o = W_o t_p (bas_pcg_point).
__device__ __forceinline__ void soa_one(int e, int n_obs, const int32_t* __restrict__ cam_obs,
                                        const int32_t* __restrict__ pt_idx,
                                        const double* __restrict__ W, double* __restrict__ Wp,
                                        int32_t* __restrict__ ptc) {
    const size_t n = (size_t)n_obs;
    if (Wp) {   // nullptr: the explicit Schur solve (no CG point pass; backsub reads W row-major)
        const double2* a = (const double2*)(W + 24 * (size_t)e);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const double2 v = a[k];
            Wp[(2 * k) * n + e] = v.x;
            Wp[(2 * k + 1) * n + e] = v.y;
        }
    }
    ptc[e] = pt_idx[cam_obs[e]];
}

// Block per camera: S_cc = U_d - Σ_o W_o V_d⁻¹ W_oᵀ (upper triangle, 36 sums) and
// b_c = -g_c + Σ_o W_o v_g (8 sums) over the camera's observations (cam_obs order, lane-strided,
// fixed tree); then the preconditioner block M_c = S_cc⁻¹ and the CG start.
// Sharded solve (points split over ranks): phase 1 writes the 44 local sums to comm[44c..] and
// stops; after the all-reduce of comm, phase 2 takes the sums from comm (phase 0: unsharded).
__global__ __launch_bounds__(CT) void bas_camera_setup(
    int n_cam, int n_obs, const int32_t* __restrict__ cam_ptr, const int32_t* __restrict__ ptc,
    const int32_t* __restrict__ cam_obs, const double* __restrict__ U,
    const double* __restrict__ W, const double* __restrict__ Vinv,
    const double* __restrict__ vg, const double* __restrict__ gc, double lam,
    double* __restrict__ Ud, double* __restrict__ Mc, double* __restrict__ x,
    double* __restrict__ r, double* __restrict__ z, double* __restrict__ pv,
    double* __restrict__ rz_c, double* __restrict__ bb_c, int32_t* __restrict__ bad, int phase,
    double* __restrict__ comm, const int32_t* __restrict__ cb, int nck, int ntot,
    double* __restrict__ Scc, double* __restrict__ pv2) {
    constexpr int N = 44;
    __shared__ double red[4][N];
    __shared__ double tot[N];
    __shared__ double cpart[SFM_BA_MAX_CHUNKS][N];
    const int c = blockIdx.x, tid = threadIdx.x;
    // the 44 sums of one observation e (camera-major position) into acc
    auto accum = [&](int e, double (&acc)[N]) {
        const int p = ptc[e];
        const double* Vi = Vinv + 9 * (size_t)p;
        const double* g = vg + 3 * (size_t)p;
        double w[24], vi[9];
        const double2* Wo = (const double2*)(W + 24 * (size_t)cam_obs[e]);  // the row, once per solve
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const double2 v = Wo[k];
            w[2 * k] = v.x;
            w[2 * k + 1] = v.y;
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) vi[k] = Vi[k];
        double wv[24];  // W_o V_d⁻¹ (8x3)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                wv[3 * i + j] = w[3 * i] * vi[j] + w[3 * i + 1] * vi[3 + j] + w[3 * i + 2] * vi[6 + j];
        int t = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = i; j < 8; ++j)
                acc[t++] += wv[3 * i] * w[3 * j] + wv[3 * i + 1] * w[3 * j + 1] + wv[3 * i + 2] * w[3 * j + 2];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[36 + i] += w[3 * i] * g[0] + w[3 * i + 1] * g[1] + w[3 * i + 2] * g[2];
    };
    if (cb) {   // chunk mode (sfm_ba_set_chunks): wave w sums chunks w, w + 4, ... of the camera
        if (phase == 2) {   // the gathered partials of all ntot chunks: the canonical tree
            if (tid < N) {
                double a[16];
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    a[k] = k < ntot ? comm[((size_t)k * n_cam + c) * N + tid] : 0.0;
                tot[tid] = sfm::chunk_tree16(a);
            }
            __syncthreads();
        } else {   // the camera's chunks in turn, each block-wide (see CT above)
            for (int k = 0; k < nck; ++k) {
                const int e0 = cb[(size_t)c * (nck + 1) + k], e1 = cb[(size_t)c * (nck + 1) + k + 1];
                if (e0 == e1) {   // block-uniform
                    if (tid < N) cpart[k][tid] = 0.0;
                    continue;
                }
                double acc[N];
#pragma unroll
                for (int i = 0; i < N; ++i) acc[i] = 0.0;
                for (int e = e0 + tid; e < e1; e += CT) accum(e, acc);
                block_sum<N>(acc, red, cpart[k]);
            }
            __syncthreads();
            if (phase == 1) {   // export: this rank's chunk partials, [chunk][camera][44]
                for (int t = tid; t < nck * N; t += CT)
                    comm[((size_t)(t / N) * n_cam + c) * N + t % N] = cpart[t / N][t % N];
                return;
            }
            if (tid < N) {
                double a[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) a[k] = k < nck ? cpart[k][tid] : 0.0;
                tot[tid] = sfm::chunk_tree16(a);
            }
            __syncthreads();
        }
    } else if (phase == 2) {
        if (tid < N) tot[tid] = comm[N * (size_t)c + tid];
        __syncthreads();
    } else {
    double acc[N];
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = 0.0;
    for (int e = cam_ptr[c] + tid; e < cam_ptr[c + 1]; e += CT) accum(e, acc);
    if (phase == 1) {
        block_sum<N>(acc, red, comm + N * (size_t)c);
        return;
    }
    block_sum<N>(acc, red, tot);
    }
    // The block's tail, spread over the first wave (it was one thread: the 8x8 Cholesky and the
    // inverse's 128 fp64 divisions in series, ~13 us per block, twice over at 500 cameras on 256
    // CUs).  Every value is the serial code's expression in its order: lane (i, j) forms S_ij
    // from the upper triangle, lane 0 each diagonal of L, lanes below it the column, lane c
    // column c of M = L^-T L^-1, so the bits are the single thread's.
    __shared__ double Ssh[64], Lsh[64], Msh[64], bsh[8], zsh[8];
    __shared__ int spd;
    const double* Uc = U + 64 * (size_t)c;
    if (tid < 64) {
        const int i = tid >> 3, j = tid & 7, a = min(i, j), b2 = max(i, j);
        double u = Uc[tid];
        if (i == j) u += lam * dclamp(Uc[tid]);
        Ud[64 * (size_t)c + tid] = u;
        double uab = Uc[8 * a + b2];
        if (a == b2) uab += lam * dclamp(Uc[8 * a + b2]);
        const double sv = uab - tot[8 * a - a * (a - 1) / 2 + (b2 - a)];
        Ssh[tid] = sv;
        if (Scc) Scc[64 * (size_t)c + tid] = sv;   // the explicit system's diagonal block
        Lsh[tid] = 0.0;
        if (tid == 0) spd = 1;
    }
    __syncthreads();
    for (int j = 0; j < 8; ++j) {   // Cholesky, column j (inv8_spd's order)
        if (tid == 0) {
            double sv = Ssh[8 * j + j];
            for (int k = 0; k < j; ++k) sv -= Lsh[8 * j + k] * Lsh[8 * j + k];
            if (!(sv > 0.0)) spd = 0;
            Lsh[8 * j + j] = sqrt(sv);
        }
        __syncthreads();
        if (tid > j && tid < 8) {
            double t = Ssh[8 * tid + j];
            for (int k = 0; k < j; ++k) t -= Lsh[8 * tid + k] * Lsh[8 * j + k];
            Lsh[8 * tid + j] = t / Lsh[8 * j + j];
        }
        __syncthreads();
    }
    const bool ok = spd != 0;
    if (tid < 8) {   // column tid of M: solve L y = e_c, then L^T m = y
        const int cc = tid;
        double m[8];
        if (ok) {
            double y[8];
            for (int i = 0; i < 8; ++i) {
                double t = (i == cc) ? 1.0 : 0.0;
                for (int k = 0; k < i; ++k) t -= Lsh[8 * i + k] * y[k];
                y[i] = t / Lsh[8 * i + i];
            }
            for (int i = 7; i >= 0; --i) {
                double t = y[i];
                for (int k = i + 1; k < 8; ++k) t -= Lsh[8 * k + i] * m[k];
                m[i] = t / Lsh[8 * i + i];
            }
        } else {   // not SPD: the diagonal preconditioner
            for (int i = 0; i < 8; ++i) m[i] = i == cc ? 1.0 / fmax(Ssh[9 * cc], DIAG_MIN) : 0.0;
            if (cc == 0) atomicOr(bad, 1);
        }
        for (int i = 0; i < 8; ++i) Msh[8 * i + cc] = m[i];
        bsh[cc] = tot[36 + cc] - gc[8 * (size_t)c + cc];
    }
    __syncthreads();
    if (tid < 64) Mc[64 * (size_t)c + tid] = Msh[tid];
    if (tid < 8) {
        double sz = 0.0;
        for (int j = 0; j < 8; ++j) sz += Msh[8 * tid + j] * bsh[j];
        zsh[tid] = sz;
        x[8 * (size_t)c + tid] = 0.0;
        r[8 * (size_t)c + tid] = bsh[tid];
        z[8 * (size_t)c + tid] = sz;
        pv[8 * (size_t)c + tid] = 0.0;  // p_{-1}: p_0 = z_0 + 0 * p_{-1}
    }
    // the explicit system's p in its two parity slots, zeroed (p_{-1} = 0; was a memset per solve)
    if (pv2 && tid < 16) pv2[(size_t)(tid >> 3) * 8 * n_cam + 8 * (size_t)c + (tid & 7)] = 0.0;
    __syncthreads();
    if (tid == 0) {
        double rz = 0.0, bb = 0.0;
        for (int i = 0; i < 8; ++i) {
            rz += bsh[i] * zsh[i];
            bb += bsh[i] * bsh[i];
        }
        rz_c[c] = rz;   // parity slot 0: rz_0
        bb_c[c] = bb;   // |b|^2 share, also rr_0 (parity slot 0 of the rr partials)
    }
}

// ---- CG iteration ------------------------------------------------------------------------------
//
// Three launches per iteration k and no communication between the blocks of a launch (kernel
// boundaries are the only grid-wide synchronisation, so no fences or flags):
//   bas_pcg_point(k)   t = V_d⁻¹ Wᵀ p_k (p_k = z_k + β_k p_{k-1} formed on the fly), u_o = W_o t_p
//   bas_pcg_camera(k)  p_k stored; q = U_d p_k - Σ_o u_o; per-camera p·q
//   bas_pcg_vec(k)     α = rz_k / Σ p·q; x += α p; r -= α q; z = M r; per-camera r·z, r·r
// The CG scalars are fixed-order sums of the per-camera partials that every block recomputes with
// the same code (canon_sum), so every block of every kernel sees bit-identical α, β and the same
// convergence decision.  Partials that a launch both reads and writes are double-buffered by the
// parity of k; once converged, bas_pcg_vec carries the partials into the next slot, so the
// decision sticks for the remaining (empty) launches.

// Canonical fixed-order sum of a[0..n) by threads 0..255 of the block (any block size >= 256):
// thread t sums a[t], a[t+256], ... in order; then a shuffle tree per wave and the 4 wave sums in
// order.  Every caller gets the same bits for the same data.
__device__ double canon_sum(const double* __restrict__ a, int n, double* red4) {
    const int tid = threadIdx.x;
    double v = 0.0;
    if (tid < 256)
        for (int i = tid; i < n; i += 256) v += a[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_down(v, off, 64);
    __syncthreads();
    if (tid < 256 && (tid & 63) == 0) red4[tid >> 6] = v;
    __syncthreads();
    const double s = ((red4[0] + red4[1]) + red4[2]) + red4[3];
    __syncthreads();
    return s;
}

struct Scalars {
    double beta;  // β_k (0 at k = 0)
    double rz;    // rz_k
    bool done;    // converged before iteration k
};

// The CG scalars of iteration k from the per-camera partials, one pass over the three arrays
// (rz partials: rzc[2][n_cam], slot k&1 = rz_k; rr partials rrc[2][n_cam] likewise): each sum has
// canon_sum's association, so every block of every kernel gets the same bits.
__device__ Scalars pcg_scalars(int k, int n_cam, const double* __restrict__ rzc,
                               const double* __restrict__ rrc, double bb, double tol,
                               double* red4x3) {
    const int tid = threadIdx.x;
    const double* a0 = rzc + (size_t)(k & 1) * n_cam;
    const double* a1 = rrc + (size_t)(k & 1) * n_cam;
    const double* a2 = rzc + (size_t)((k + 1) & 1) * n_cam;
    const bool nb = k > 0;
    double v0 = 0.0, v1 = 0.0, v2 = 0.0;
    if (tid < 256)
        for (int i = tid; i < n_cam; i += 256) {
            v0 += a0[i];
            v1 += a1[i];
            if (nb) v2 += a2[i];
        }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        v0 += __shfl_down(v0, off, 64);
        v1 += __shfl_down(v1, off, 64);
        v2 += __shfl_down(v2, off, 64);
    }
    __syncthreads();
    if (tid < 256 && (tid & 63) == 0) {
        red4x3[tid >> 6] = v0;
        red4x3[4 + (tid >> 6)] = v1;
        red4x3[8 + (tid >> 6)] = v2;
    }
    __syncthreads();
    const double* r = red4x3;
    Scalars sc;
    sc.rz = ((r[0] + r[1]) + r[2]) + r[3];
    const double rr = ((r[4] + r[5]) + r[6]) + r[7];
    sc.beta = nb ? sc.rz / (((r[8] + r[9]) + r[10]) + r[11]) : 0.0;
    sc.done = !(bb > 0.0) || rr <= tol * tol * bb;
    __syncthreads();
    return sc;
}

// The CG scalars of iteration k + 1, computed ONCE by the last block of iteration k's vector kernel
// (after every block wrote its per-camera partials of slot (k+1)&1: store, fence, counter) and
// published in st for the next iteration's kernels — instead of every block of the point pass
// re-reducing the three n_cam-long partial arrays (round 4: 12 KB of L2 reads and two block
// barriers per point-pass block).  The same canon_sum association: the same bits.
__device__ void publish_next(int k, int n_cam, const double* __restrict__ rzc,
                             const double* __restrict__ rrc, double tol, PcgState* __restrict__ st,
                             unsigned nblk, double* red4x3) {
    __shared__ bool last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&st->cnt, 1u) == nblk - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    const Scalars sc = pcg_scalars(k + 1, n_cam, rzc, rrc, st->bb, tol, red4x3);
    if (threadIdx.x == 0) {
        st->beta = sc.beta;
        st->rz = sc.rz;
        st->done = sc.done ? 1 : 0;
        st->cnt = 0u;
    }
}

__device__ __forceinline__ Scalars read_scalars(const PcgState* __restrict__ st) {
    Scalars sc;
    sc.beta = st->beta;
    sc.rz = st->rz;
    sc.done = st->done != 0;
    return sc;
}

#ifndef SFM_BA_PG
#define SFM_BA_PG 8
#endif
#ifndef SFM_BA_CC
#define SFM_BA_CC 256
#endif
constexpr int PG = SFM_BA_PG;  // lanes per point in the point-major passes

// u_o (8 doubles) of one observation.  BA_U_NT: non-temporal stores — u (64 B per observation,
// 66 MB at 1 M observations) is read once, by the next kernel, and never fits the L2; plain
// stores leave it dirty in L2 at the kernel boundary.
#ifndef BA_U_NT
#define BA_U_NT 1
#endif
__device__ __forceinline__ void store_u(double* __restrict__ dst, const double (&uo)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#if BA_U_NT
        __builtin_nontemporal_store(uo[i], dst + i);
#else
        dst[i] = uo[i];
#endif
    }
}

// Wave per long-track point (more than LONG_OBS observations; listed by bas_point_setup): lane j
// takes observations j, j+64, ... in order, a 64-lane xor butterfly combines them, then the lanes
// write u_o = W_o t_p for their observations.  The waves of the lb long-track blocks stride over
// the list; every wave reaches the end of it.
__device__ __forceinline__ void pcg_point_long(int b, int lb, int n_obs,
                                               const int32_t* __restrict__ pt_ptr,
                                               const int32_t* __restrict__ cam_idx,
                                               const double* __restrict__ Wp,
                                               const double* __restrict__ Vinv,
                                               const double* __restrict__ z,
                                               const double* __restrict__ pold, double beta,
                                               const int32_t* __restrict__ long_list,
                                               const int32_t* __restrict__ long_cnt,
                                               double* __restrict__ u) {
    const int lane = threadIdx.x & 63;
    const int nl = *long_cnt;
    const size_t n = (size_t)n_obs;
    for (int wv = b * 4 + (threadIdx.x >> 6); wv < nl; wv += lb * 4) {
        const int g = long_list[wv];
        const int o0 = pt_ptr[g], o1 = pt_ptr[g + 1];
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        for (int o = o0 + lane; o < o1; o += 64) {
            const double* Wo = Wp + o;
            const int c = cam_idx[o];
            const double* zp = z + 8 * (size_t)c;
            const double* pp = pold + 8 * (size_t)c;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const double xi = zp[i] + beta * pp[i];  // p_k, as in bas_pcg_point
                s0 += Wo[(3 * i) * n] * xi;
                s1 += Wo[(3 * i + 1) * n] * xi;
                s2 += Wo[(3 * i + 2) * n] * xi;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            s0 += __shfl_xor(s0, off, 64);
            s1 += __shfl_xor(s1, off, 64);
            s2 += __shfl_xor(s2, off, 64);
        }
        const double* Vi = Vinv + 9 * (size_t)g;
        const double t0 = Vi[0] * s0 + Vi[1] * s1 + Vi[2] * s2;
        const double t1 = Vi[3] * s0 + Vi[4] * s1 + Vi[5] * s2;
        const double t2 = Vi[6] * s0 + Vi[7] * s1 + Vi[8] * s2;
        for (int o = o0 + lane; o < o1; o += 64) {
            const double* Wo = Wp + o;
            double uo[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                uo[i] = Wo[(3 * i) * n] * t0 + Wo[(3 * i + 1) * n] * t1 + Wo[(3 * i + 2) * n] * t2;
            store_u(u + 8 * (size_t)o, uo);
        }
    }
}

// PG lanes per point: t_p = V_d⁻¹ Σ_o W_oᵀ p_c.  Lane j of a point takes its observations
// j, j+PG, ... in order; the PG partial sums are combined by a fixed butterfly (every lane gets
// the same bits), and each lane then writes u_o = W_o t_p (8 doubles) for its observations: the
// camera pass sums u_o instead of reading W a second time (64 B instead of 192 + 24 B per
// observation and CG iteration).  Points with more than LONG_OBS observations are left to the
// grid's first n_long_blk blocks, a wave per point (pcg_point_long).
__global__ __launch_bounds__(256) void bas_pcg_point(
    int k, int n_pt, int n_cam, int n_obs, const int32_t* __restrict__ pt_ptr,
    const int32_t* __restrict__ cam_idx, const double* __restrict__ Wp,
    const double* __restrict__ Vinv, const double* __restrict__ z, const double* __restrict__ pold,
    const double* __restrict__ rzc, const double* __restrict__ rrc, double tol,
    PcgState* __restrict__ st, double* __restrict__ u, int n_long_blk,
    const int32_t* __restrict__ long_list, const int32_t* __restrict__ long_cnt) {
    // the CG scalars of iteration k were published by the previous vector kernel (publish_next)
    if ((int)blockIdx.x < n_long_blk) {  // block-uniform: the long-track blocks, dispatched first
        const Scalars sc = read_scalars(st);
        if (!sc.done)
            pcg_point_long(blockIdx.x, n_long_blk, n_obs, pt_ptr, cam_idx, Wp, Vinv, z, pold,
                           sc.beta, long_list, long_cnt, u);
        return;
    }
    const int g = (blockIdx.x - n_long_blk) * (blockDim.x / PG) + threadIdx.x / PG;
    const int j = threadIdx.x % PG;
    const bool valid = g < n_pt;
    const int o0 = (valid ? pt_ptr[g] : 0) + j;
    const int o1 = valid ? pt_ptr[g + 1] : 0;
    const size_t n = (size_t)n_obs;
    // the lane's first observation is loaded before the CG scalars are reduced, so the two
    // latencies overlap (the whole grid is resident at once: this pass is latency-bound)
    double w[24], zc[8], pc[8];
    const bool has = o0 < o1;
    {
        const int oo = has ? o0 : 0;
        const int c = has ? cam_idx[oo] : 0;
#pragma unroll
        for (int m = 0; m < 24; ++m) w[m] = has ? Wp[m * n + oo] : 0.0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            zc[i] = z[8 * (size_t)c + i];
            pc[i] = pold[8 * (size_t)c + i];
        }
    }
    const Scalars sc = read_scalars(st);
    if (sc.done) return;
    if (valid && o1 - (o0 - j) > LONG_OBS) return;  // group-uniform: a long-track block's point
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    if (has) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double xi = zc[i] + sc.beta * pc[i];  // p_k, the same expression as bas_pcg_camera
            s0 += w[3 * i] * xi;
            s1 += w[3 * i + 1] * xi;
            s2 += w[3 * i + 2] * xi;
        }
    }
    for (int o = o0 + PG; o < o1; o += PG) {
        const double* Wo = Wp + o;
        const int c = cam_idx[o];
        const double* zp = z + 8 * (size_t)c;
        const double* pp = pold + 8 * (size_t)c;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double xi = zp[i] + sc.beta * pp[i];
            s0 += Wo[(3 * i) * n] * xi;
            s1 += Wo[(3 * i + 1) * n] * xi;
            s2 += Wo[(3 * i + 2) * n] * xi;
        }
    }
#pragma unroll
    for (int off = PG / 2; off >= 1; off >>= 1) {
        s0 += __shfl_xor(s0, off, PG);
        s1 += __shfl_xor(s1, off, PG);
        s2 += __shfl_xor(s2, off, PG);
    }
    if (!has) return;
    const double* Vi = Vinv + 9 * (size_t)g;
    const double t0 = Vi[0] * s0 + Vi[1] * s1 + Vi[2] * s2;
    const double t1 = Vi[3] * s0 + Vi[4] * s1 + Vi[5] * s2;
    const double t2 = Vi[6] * s0 + Vi[7] * s1 + Vi[8] * s2;
    auto put = [&](int o, const double (&wo)[24]) {
        double uo[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) uo[i] = wo[3 * i] * t0 + wo[3 * i + 1] * t1 + wo[3 * i + 2] * t2;
        store_u(u + 8 * (size_t)o, uo);
    };
    put(o0, w);
    for (int o = o0 + PG; o < o1; o += PG) {  // points with more than PG observations
#pragma unroll
        for (int m = 0; m < 24; ++m) w[m] = Wp[m * n + o];
        put(o, w);
    }
}

constexpr int CC = SFM_BA_CC;  // threads per camera block in the CG camera pass
#ifndef CAM_PCG_MLP
#define CAM_PCG_MLP 4  // observations per lane whose loads the CG camera pass keeps in flight
#endif

// Block per camera: p_k stored; q_c = U_d p_c - Σ_o u_o (u_o = W_o t_p, bas_pcg_point); p_c·q_c.
// Sharded solve: phase 1 writes the local Σ_o u_o to comm[8c..] and stops; after the
// all-reduce of comm, phase 2 finishes the camera from it (phase 0: unsharded).  Phase 3 (the
// one-launch finish, bas_pcg_finish_vec): phase 1 plus U_d p_k into q and p_k into pv.
__global__ __launch_bounds__(CC) void bas_pcg_camera(
    int k, int n_cam, const int32_t* __restrict__ cam_ptr, const int32_t* __restrict__ cam_obs,
    const double* __restrict__ u, const double* __restrict__ Ud, const double* __restrict__ z, double* __restrict__ pv,
    const PcgState* __restrict__ st, double* __restrict__ q, double* __restrict__ pq, int phase,
    double* __restrict__ comm, const int32_t* __restrict__ cb, int nck, int ntot) {
    __shared__ double red[CC / 64][8];
    __shared__ double pc_s[8];
    __shared__ double cpart[SFM_BA_MAX_CHUNKS][8];
    if (st->done) return;
    const double beta = st->beta;
    const int c = blockIdx.x, tid = threadIdx.x;
    double ur[8];  // U_d row tid (tid < 8), in flight during the observation loop
    if (tid < 8 && phase != 1) {
        const double* u = Ud + 64 * (size_t)c + 8 * tid;
#pragma unroll
        for (int j = 0; j < 8; ++j) ur[j] = u[j];
    }
    double acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.0;
    auto add_obs = [&](int e) {
        const double2* uo = (const double2*)(u + 8 * (size_t)cam_obs[e]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double2 v = uo[i];
            acc[2 * i] += v.x;
            acc[2 * i + 1] += v.y;
        }
    };
    // the lane's observations e, e + CC, ... < e1 in order; CAM_PCG_MLP of them per step have their
    // cam_obs and u loads in flight together (500 camera blocks leave ~2 waves per SIMD: the pass
    // is latency-bound), the sums still taken one observation after the other
    auto sum_range = [&](int e, int e1) {
        for (; e + (CAM_PCG_MLP - 1) * CC < e1; e += CAM_PCG_MLP * CC) {
            int o[CAM_PCG_MLP];
#pragma unroll
            for (int m = 0; m < CAM_PCG_MLP; ++m) o[m] = cam_obs[e + m * CC];
            double2 v[CAM_PCG_MLP][4];
#pragma unroll
            for (int m = 0; m < CAM_PCG_MLP; ++m)
#pragma unroll
                for (int i = 0; i < 4; ++i) v[m][i] = ((const double2*)(u + 8 * (size_t)o[m]))[i];
#pragma unroll
            for (int m = 0; m < CAM_PCG_MLP; ++m)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[2 * i] += v[m][i].x;
                    acc[2 * i + 1] += v[m][i].y;
                }
        }
        for (; e < e1; e += CC) add_obs(e);
    };
    if (cb) {   // chunk mode: the camera's chunks in turn, each block-wide (see CT above)
        static_assert(CC == CT, "bas_pcg_camera chunk mode: block_sum's four waves");
        if (phase != 2) {
            for (int k = 0; k < nck; ++k) {
                const int e0 = cb[(size_t)c * (nck + 1) + k], e1 = cb[(size_t)c * (nck + 1) + k + 1];
                if (e0 == e1) {   // block-uniform
                    if (tid < 8) cpart[k][tid] = 0.0;
                    continue;
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i] = 0.0;
                sum_range(e0 + tid, e1);
                block_sum<8>(acc, red, cpart[k]);
            }
        }
    } else {
    if (phase != 2) sum_range(cam_ptr[c] + tid, cam_ptr[c + 1]);
    int idx;   // the wave's 8 sums by recursive halving; the waves' partials summed in order below
    if (sfm::wave_halving_sum<8>(acc, tid & 63, idx)) red[tid >> 6][idx] = acc[0];
    }
    if (tid < 8) {
        const size_t kk = 8 * (size_t)c + tid;
        const double pk = z[kk] + beta * pv[kk];  // p_k, the same expression as bas_pcg_point
        pc_s[tid] = pk;
    }
    __syncthreads();
    if (tid < 8) {
        const size_t kk = 8 * (size_t)c + tid;
        double wt = 0.0;
        if (cb) {
            if (phase == 1 || phase == 3)   // export: [chunk][camera][8]
                for (int k = 0; k < nck; ++k) comm[((size_t)k * n_cam + c) * 8 + tid] = cpart[k][tid];
            if (phase == 1) return;
            double a[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                a[k] = phase == 2 ? (k < ntot ? comm[((size_t)k * n_cam + c) * 8 + tid] : 0.0)
                                  : (k < nck ? cpart[k][tid] : 0.0);
            wt = sfm::chunk_tree16(a);
        } else {
#pragma unroll
        for (int w = 0; w < CC / 64; ++w) wt += red[w][tid];
        if (phase == 1 || phase == 3) comm[kk] = wt;
        if (phase == 1) return;
        if (phase == 2) wt = comm[kk];
        }
        double sU = 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j) sU += ur[j] * pc_s[j];
        pv[kk] = pc_s[tid];
        if (phase == 3) {
            q[kk] = sU;
            return;
        }
        const double qi = sU - wt;
        q[kk] = qi;
        double v = pc_s[tid] * qi;
        v += __shfl_down(v, 4, 8);
        v += __shfl_down(v, 2, 8);
        v += __shfl_down(v, 1, 8);
        if (tid == 0) pq[c] = v;
    }
}

// Thread per (camera, component) gi = 8 c + i (a camera's 8 components are 8 consecutive lanes):
// α = rz_k / Σ p·q; x += α p; r -= α q; z = M r; per-camera r·z and r·r into slot (k+1)&1 (rr = 0
// on a breakdown).  A breakdown (p·q <= 0) stops the iteration.  The component's x, p, r, q and
// its row of M are loaded before canon_sum's barriers (they do not depend on α), so their latency
// overlaps the reduction's (round 6: the kernel is a chain of dependent global round trips).
__global__ __launch_bounds__(256) void bas_pcg_vec(
    int k, int n_cam, const double* __restrict__ Mc, double* __restrict__ x,
    double* __restrict__ r, double* __restrict__ z, const double* __restrict__ pv,
    const double* __restrict__ q, const double* __restrict__ pq, double* __restrict__ rzc,
    double* __restrict__ rrc, PcgState* __restrict__ st, double tol) {
    __shared__ double red4[12];
    const bool done = st->done != 0;
    const double rz_k = st->rz;
    const int gi = blockIdx.x * blockDim.x + threadIdx.x;
    const int c = gi >> 3, i = gi & 7;
    const bool valid = c < n_cam;
    const int s0 = k & 1, s1 = (k + 1) & 1;
    if (done) {
        // converged earlier: carry the partials forward so iteration k+1 sees the same sums
        if (valid && i == 0) {
            rzc[(size_t)s1 * n_cam + c] = rzc[(size_t)s0 * n_cam + c];
            rrc[(size_t)s1 * n_cam + c] = rrc[(size_t)s0 * n_cam + c];
        }
        return;
    }
    const size_t kk = 8 * (size_t)(valid ? c : 0) + i;
    double xv = 0.0, pvv = 0.0, rv = 0.0, qv = 0.0, m[8];
    if (valid) {
        xv = x[kk];
        pvv = pv[kk];
        rv = r[kk];
        qv = q[kk];
    }
    const double* M = Mc + 64 * (size_t)(valid ? c : 0) + 8 * i;
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = M[j];
    const double pqs = canon_sum(pq, n_cam, red4);
    const bool breakdown = !(pqs > 0.0);
    const double alpha = breakdown ? 0.0 : rz_k / pqs;
    double ri = 0.0;
    if (valid) {
        x[kk] = xv + alpha * pvv;
        ri = rv - alpha * qv;
        r[kk] = ri;
    }
    double zi = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) zi += m[j] * __shfl(ri, (threadIdx.x & ~7) + j, 64);
    double rz = ri * zi, rr = ri * ri;
    rz += __shfl_down(rz, 4, 8); rr += __shfl_down(rr, 4, 8);
    rz += __shfl_down(rz, 2, 8); rr += __shfl_down(rr, 2, 8);
    rz += __shfl_down(rz, 1, 8); rr += __shfl_down(rr, 1, 8);
    if (valid) {
        z[kk] = zi;
        if (i == 0) {
            rzc[(size_t)s1 * n_cam + c] = rz;
            rrc[(size_t)s1 * n_cam + c] = breakdown ? 0.0 : rr;
        }
    }
    if (gi == 0) st->iter = k + 1;
    publish_next(k, n_cam, rzc, rrc, tol, st, gridDim.x, red4);
}

// ---- explicit reduced camera system (sfm_ba_set_schur) -------------------------------------------
//
// T_slot = Σ over the slot's camera-pair instances (a, b) of Y_a W_bᵀ, Y_a = W_a V_d⁻¹ (the point of
// a), so the off-diagonal Schur blocks are S_ij = -T_ij; the diagonal blocks S_cc come from
// bas_camera_setup.  One wave (one workgroup) per (chunk, slot) group, a lane PAIR per instance:
// lane 2j + h takes rows 4h .. 4h + 3 of the 8x8 block for instances j, j + 32, ... of the group (an
// order that depends only on the group).  The wave's 32 instances' W_a, W_b (16-byte pieces, 12 per
// record: whole cache lines per load instruction) and V_d⁻¹ (dwords, 18 per record) are staged
// into LDS by global_load_lds, double-buffered: batch t + 1's records arrive while batch t is
// multiplied from LDS (no staging VGPRs); the index chain inst -> pt_idx runs ahead (a, b two
// batches, p one).  32 accumulators per lane, then the recursive-halving sum over the lanes of the
// same h: lane 2j + h ends holding element 32 h + j and stores it.  At cfg5's final model
// 0.175 - 0.181 ms per solve against 0.19 for direct loads by each lane pair (16 B of 32 different
// records per instruction); 1 / 2 / 4 / 8 waves per group with direct loads 0.25 / 0.22 / 0.31 /
// 0.57, the chain pipelined without staging 0.27 - 0.29, LDS staging through VGPRs 0.31 (its load
// latency exposed), W_b and V_d⁻¹ staged with W_a in registers (half the LDS, 8 waves per CU
// instead of 5) 0.183 — profiles/r06/ba_study/t6_t7_schur_build_variants.txt, t9_*, t10_*.  Same
// bits in every form.
typedef __attribute__((address_space(3))) void tb_lds_void;
typedef const __attribute__((address_space(1))) void tb_gbl_void;
__global__ __launch_bounds__(64) void bas_schur_build(
    int n_seg, int n_inst, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ inst, const int32_t* __restrict__ pt_idx,
    const double* __restrict__ W, const double* __restrict__ Vinv, double* __restrict__ Tpart) {
    constexpr int WB = 32 * 12 * 16, VB = 32 * 18 * 4, BUF = 2 * WB + VB;   // bytes per buffer
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * BUF];
    const int s = blockIdx.x, lane = threadIdx.x;
    const int h = lane & 1, j = lane >> 1;
    const int i0 = seg[2 * n_seg + s], i1 = seg[3 * n_seg + s];
    const unsigned char* Wb8 = (const unsigned char*)W;
    const unsigned char* Vb8 = (const unsigned char*)Vinv;
    // every lane issues every piece (lanes past the batch read record 0: valid memory, never
    // used), so no load sits in a branch and the compiler's vmcnt counts stay exact
    auto stage = [&](int a, int b, int p, unsigned char* buf) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int q = lane + 64 * k, rec = q / 12, off = q - 12 * rec;
            const int ar = __shfl(a, rec), br = __shfl(b, rec);
            __builtin_amdgcn_global_load_lds((tb_gbl_void*)(Wb8 + 192 * (size_t)ar + 16 * off),
                                             (tb_lds_void*)(buf + 1024 * k), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((tb_gbl_void*)(Wb8 + 192 * (size_t)br + 16 * off),
                                             (tb_lds_void*)(buf + WB + 1024 * k), 16, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int d = lane + 64 * k, rec = d / 18, off = d - 18 * rec;
            const int pr = __shfl(p, rec);
            __builtin_amdgcn_global_load_lds((tb_gbl_void*)(Vb8 + 72 * (size_t)pr + 4 * off),
                                             (tb_lds_void*)(buf + 2 * WB + 256 * k), 4, 0, 0);
        }
    };
    auto ab = [&](int base, int& a, int& b) {   // batch `base`'s instance of this lane (< 32)
        a = 0; b = 0;
        if (lane < 32 && base + lane < i1) { a = inst[base + lane]; b = inst[n_inst + base + lane]; }
    };
    double acc[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) acc[t] = 0.0;
    if (i0 < i1) {
        int a0, b0, a1, b1, a2, b2;
        ab(i0, a0, b0);
        const int p0 = pt_idx[a0];
        stage(a0, b0, p0, lds);
        ab(i0 + 32, a1, b1);
        int p1 = pt_idx[a1];
        ab(i0 + 64, a2, b2);
        __syncthreads();
        int t = 0;
        for (int base = i0; base < i1; base += 32, ++t) {
            const unsigned char* cur = lds + (t & 1) * BUF;
            unsigned char* nxt = lds + ((t + 1) & 1) * BUF;
            const int nb = min(32, i1 - base);
            const int jj = min(j, 31);
            double wa[12], wb[24], vi[9];
            {
                const double2* sWa = (const double2*)cur;
                const double2* sWb = (const double2*)(cur + WB);
                const double* sV = (const double*)(cur + 2 * WB);
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const double2 x = sWa[12 * jj + 6 * h + u];
                    wa[2 * u] = x.x; wa[2 * u + 1] = x.y;
                }
#pragma unroll
                for (int u = 0; u < 12; ++u) {
                    const double2 x = sWb[12 * jj + u];
                    wb[2 * u] = x.x; wb[2 * u + 1] = x.y;
                }
#pragma unroll
                for (int u = 0; u < 9; ++u) vi[u] = sV[9 * jj + u];
            }
            // the next batch's records into the other buffer (its readers passed the last
            // barrier), the index chain one step on: they arrive while this batch is multiplied
            int p2 = 0, a3 = 0, b3 = 0;
            if (base + 32 < i1) {
                stage(a1, b1, p1, nxt);
                p2 = pt_idx[a2];
                ab(base + 96, a3, b3);
            }
            if (j < nb) {
                double y[12];
#pragma unroll
                for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        y[3 * i2 + c] = wa[3 * i2] * vi[c] + wa[3 * i2 + 1] * vi[3 + c] + wa[3 * i2 + 2] * vi[6 + c];
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 8; ++c)
                        acc[8 * r + c] += y[3 * r] * wb[3 * c] + y[3 * r + 1] * wb[3 * c + 1] + y[3 * r + 2] * wb[3 * c + 2];
            }
            __syncthreads();   // the next batch has landed; this buffer may be refilled
            a1 = a2; b1 = b2; p1 = p2; a2 = a3; b2 = b3;
        }
    }
    int idx;
    if (sfm::wave_halving_sum_strided<32, 2>(acc, lane, idx))
        Tpart[(size_t)s * 64 + 32 * h + idx] = acc[0];   // the group's row
}

// T = per slot, the canonical chunk tree over its group partials (parts [n_group][64]; chunks
// without a group are 0 leaves — the dense [n_total][n_slot] tree's bits).  Thread per element.
// The CG's iteration-0 scalars from the camera set-up's partials (one block of 256).
__device__ void pcg_init_body(int n_cam, const double* __restrict__ rzc,
                              const double* __restrict__ bb_c, double tol,
                              PcgState* __restrict__ st) {
    __shared__ double red4[12];
    const double bb = canon_sum(bb_c, n_cam, red4);
    const Scalars sc = pcg_scalars(0, n_cam, rzc, bb_c, bb, tol, red4);
    if (threadIdx.x == 0) {
        st->bb = bb;
        st->rz = sc.rz;
        st->beta = sc.beta;
        st->rr = bb;
        st->iter = 0;
        st->done = sc.done ? 1 : 0;
        st->cnt = 0u;
    }
}

// Block tblk (one past the tree's blocks) runs bas_pcg_init's work: the camera set-up that wrote
// its partials finished before this launch, so the explicit solve needs no launch of its own for it.
__global__ __launch_bounds__(256) void bas_schur_tree(int n_slot, const int32_t* __restrict__ sg_ptr,
                                                      const int32_t* __restrict__ sg,
                                                      const int32_t* __restrict__ gk,
                                                      const double* __restrict__ parts,
                                                      double* __restrict__ out, int tblk, int n_cam,
                                                      const double* __restrict__ rzc,
                                                      const double* __restrict__ bb_c, double tol,
                                                      PcgState* __restrict__ st) {
    if ((int)blockIdx.x == tblk) {
        pcg_init_body(n_cam, rzc, bb_c, tol, st);
        return;
    }
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)n_slot * 64) return;
    const int s = (int)(i >> 6), e = (int)(i & 63);
    double a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = 0.0;
    for (int j = sg_ptr[s]; j < sg_ptr[s + 1]; ++j) {
        const int g = sg[j];
        const double v = parts[(size_t)g * 64 + e];
        const int k = gk[g];
#pragma unroll
        for (int q = 0; q < 16; ++q) a[q] = (q == k) ? v : a[q];
    }
    out[i] = sfm::chunk_tree16(a);
}

// One block row c of the explicit CG product (one wave; bas_point + bas_pcg_camera's role once S
// is formed): p_k = z_k + β_k p_{k-1} (p_{k-1} from the other parity slot of pv2), the row's blocks in
// row_ent order, 8 lanes per block (lane r: row r of the block, or column r for a transposed
// slot), blocks g, g + 8, ... per lane group, then a fixed xor tree over the 8 groups;
// q_c = S_cc p_c - Σ T p_j, p_k stored, p·q of the camera.
__device__ __forceinline__ void schur_spmv_row(int c, int lane, int k, int n_cam, double beta,
                                               const int32_t* __restrict__ row_ptr,
                                               const int32_t* __restrict__ row_ent,
                                               const int32_t* __restrict__ slot_cam,
                                               const double* __restrict__ T,
                                               const double* __restrict__ Scc,
                                               const double* __restrict__ z, double* __restrict__ pv2,
                                               double* __restrict__ q, double* __restrict__ pq) {
    const double* pold = pv2 + (size_t)((k + 1) & 1) * 8 * n_cam;
    double* pnew = pv2 + (size_t)(k & 1) * 8 * n_cam;
    const int g = lane >> 3, r = lane & 7;
    const int e0 = row_ptr[c], e1 = row_ptr[c + 1];
    double s = 0.0;
    // the lane group's entries two at a time: both entries' index loads, then both blocks' and
    // neighbours' loads, are in flight together (a row's entry chain is row_ent -> slot_cam ->
    // T / z / p: three dependent global round trips per entry otherwise)
    int e = e0 + g;
    for (; e + 8 < e1; e += 16) {
        const int ent0 = row_ent[e], ent1 = row_ent[e + 8];
        const int slot0 = ent0 >> 1, tr0 = ent0 & 1, slot1 = ent1 >> 1, tr1 = ent1 & 1;
        const int j0 = slot_cam[2 * slot0 + (tr0 ? 0 : 1)];   // the other camera of the block
        const int j1 = slot_cam[2 * slot1 + (tr1 ? 0 : 1)];
        const double* Tb0 = T + 64 * (size_t)slot0;
        const double* Tb1 = T + 64 * (size_t)slot1;
        double t0[8], t1[8], z0[8], z1[8], o0[8], o1[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            t0[m] = tr0 ? Tb0[8 * m + r] : Tb0[8 * r + m];
            t1[m] = tr1 ? Tb1[8 * m + r] : Tb1[8 * r + m];
            z0[m] = z[8 * (size_t)j0 + m];
            o0[m] = pold[8 * (size_t)j0 + m];
            z1[m] = z[8 * (size_t)j1 + m];
            o1[m] = pold[8 * (size_t)j1 + m];
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) s += t0[m] * (z0[m] + beta * o0[m]);
#pragma unroll
        for (int m = 0; m < 8; ++m) s += t1[m] * (z1[m] + beta * o1[m]);
    }
    if (e < e1) {
        const int ent = row_ent[e];
        const int slot = ent >> 1, tr = ent & 1;
        const int j = slot_cam[2 * slot + (tr ? 0 : 1)];
        const double* Tb = T + 64 * (size_t)slot;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const double pj = z[8 * (size_t)j + m] + beta * pold[8 * (size_t)j + m];
            s += (tr ? Tb[8 * m + r] : Tb[8 * r + m]) * pj;
        }
    }
    s += __shfl_xor(s, 8, 64);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    double pc[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) pc[m] = z[8 * (size_t)c + m] + beta * pold[8 * (size_t)c + m];
    double sp = 0.0;
#pragma unroll
    for (int m = 0; m < 8; ++m) sp += Scc[64 * (size_t)c + 8 * r + m] * pc[m];
    const double qi = sp - s;
    double pr = 0.0;
#pragma unroll
    for (int m = 0; m < 8; ++m) pr = (m == r) ? pc[m] : pr;
    if (lane < 8) {
        pnew[8 * (size_t)c + r] = pr;
        q[8 * (size_t)c + r] = qi;
    }
    double v = pr * qi;
    v += __shfl_down(v, 4, 8);
    v += __shfl_down(v, 2, 8);
    v += __shfl_down(v, 1, 8);
    if (lane == 0) pq[c] = v;
}

// Explicit CG product (bas_point + bas_pcg_camera's role once S is formed): wave per block row.
__global__ __launch_bounds__(256) void bas_pcg_spmv(
    int k, int n_cam, const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ row_ent,
    const int32_t* __restrict__ slot_cam, const double* __restrict__ T,
    const double* __restrict__ Scc, const double* __restrict__ z, double* __restrict__ pv2,
    const PcgState* __restrict__ st, double* __restrict__ q, double* __restrict__ pq) {
    const Scalars sc = read_scalars(st);
    if (sc.done) return;   // the same for every block (published before the launch)
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (c < n_cam)
        schur_spmv_row(c, lane, k, n_cam, sc.beta, row_ptr, row_ent, slot_cam, T, Scc, z, pv2, q, pq);
}

// Largest camera count for which the sharded solve finishes an iteration in one launch
// (bas_pcg_finish_vec keeps every camera's p·q in LDS and recomputes them in every block:
// n_cam² · 11 B of L2 reads).  Mirrored by sfmcore.BA_FINISH_VEC_MAX_CAM.
constexpr int FINISH_VEC_MAX_CAM = 1024;
constexpr int FV = 512;   // threads per bas_pcg_finish_vec block: 64 cameras per pass
constexpr int FVR = 8;    // passes per round: 512 cameras' loads in flight at once

// Sharded solve, after the all-reduce of comm = Σ_o W_o t_p over all ranks: bas_pcg_camera's
// phase 2 and bas_pcg_vec in one launch (thread per camera component).  Phase 3 of the camera
// pass left p_k (pv) and U_d p_k (su) per camera, so q = su - comm.  Every block forms p·q for
// ALL cameras (8 lanes each, bas_pcg_camera's shuffle tree, into LDS; 512 cameras' loads per
// round in flight together), and canon_sum over LDS gives every block the unsharded solve's
// Σ p·q bit for bit without a second launch.  No block reads z or writes p, so both stay in
// place.
__global__ __launch_bounds__(FV) void bas_pcg_finish_vec(
    int k, int n_cam, const double* __restrict__ su, const double* __restrict__ comm,
    const double* __restrict__ pv, const double* __restrict__ Mc, double* __restrict__ x,
    double* __restrict__ r, double* __restrict__ z, double* __restrict__ rzc,
    double* __restrict__ rrc, PcgState* __restrict__ st, int ntot, double tol) {
    __shared__ double pq_s[FINISH_VEC_MAX_CAM];
    __shared__ double red4[12];
    const int tid = threadIdx.x;
    const int c = blockIdx.x * (FV / 8) + (tid >> 3), i = tid & 7;
    const bool valid = c < n_cam;
    const int s0 = k & 1, s1 = (k + 1) & 1;
    const size_t kk = 8 * (size_t)(valid ? c : 0) + i;
    // rounds of FVR passes x FV/8 cameras, straight-line (clamped loads, every lane shuffles) so
    // a round's loads are in flight together; the first round's loads, this thread's x, r and
    // preconditioner row are issued before the CG state is read (the latencies overlap)
    double pj[FVR], sj[FVR], cm[FVR];
    auto load_round = [&](int c0) {
#pragma unroll
        for (int m = 0; m < FVR; ++m) {
            const int cc = min(c0 + m * (FV / 8) + (tid >> 3), n_cam - 1);
            const size_t b = 8 * (size_t)cc + i;
            pj[m] = pv[b];
            sj[m] = su[b];
            if (ntot > 0) {   // chunk mode: the gathered chunk partials [chunk][camera][8], tree
                double a[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) a[k] = k < ntot ? comm[(size_t)k * 8 * n_cam + b] : 0.0;
                cm[m] = sfm::chunk_tree16(a);
            } else {
                cm[m] = comm[b];
            }
        }
    };
    load_round(0);
    const double xk = x[kk], rk = r[kk];
    double Mr[8];
    {
        const double* M = Mc + 64 * (size_t)(valid ? c : 0) + 8 * i;
#pragma unroll
        for (int j = 0; j < 8; ++j) Mr[j] = M[j];
    }
    const bool done = st->done != 0;
    if (done) {
        if (valid && i == 0) {
            rzc[(size_t)s1 * n_cam + c] = rzc[(size_t)s0 * n_cam + c];
            rrc[(size_t)s1 * n_cam + c] = rrc[(size_t)s0 * n_cam + c];
        }
        return;
    }
    const double rz_k = st->rz;
    double pk = 0.0, qi = 0.0;
    for (int c0 = 0; c0 < n_cam; c0 += FVR * (FV / 8)) {
        if (c0 > 0) load_round(c0);
#pragma unroll
        for (int m = 0; m < FVR; ++m) {
            const int cc = c0 + m * (FV / 8) + (tid >> 3);
            const double q = sj[m] - cm[m];
            double v = pj[m] * q;
            v += __shfl_down(v, 4, 8);
            v += __shfl_down(v, 2, 8);
            v += __shfl_down(v, 1, 8);
            if (i == 0 && cc < n_cam) pq_s[cc] = v;
            if (cc == c) {
                pk = pj[m];
                qi = q;
            }
        }
    }
    __syncthreads();
    const double pqs = canon_sum(pq_s, n_cam, red4);
    const bool breakdown = !(pqs > 0.0);
    const double alpha = breakdown ? 0.0 : rz_k / pqs;
    double ri = 0.0;
    if (valid) {
        x[kk] = xk + alpha * pk;
        ri = rk - alpha * qi;
        r[kk] = ri;
    }
    double zi = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) zi += Mr[j] * __shfl(ri, (tid & 63 & ~7) + j, 64);
    double rz = ri * zi, rr = ri * ri;
    rz += __shfl_down(rz, 4, 8); rr += __shfl_down(rr, 4, 8);
    rz += __shfl_down(rz, 2, 8); rr += __shfl_down(rr, 2, 8);
    rz += __shfl_down(rz, 1, 8); rr += __shfl_down(rr, 1, 8);
    if (valid) {
        z[kk] = zi;
        if (i == 0) {
            rzc[(size_t)s1 * n_cam + c] = rz;
            rrc[(size_t)s1 * n_cam + c] = breakdown ? 0.0 : rr;
        }
    }
    if (blockIdx.x == 0 && tid == 0) st->iter += 1;  // k-free: a captured window replays at any k
    publish_next(k, n_cam, rzc, rrc, tol, st, gridDim.x, red4);
}

// One block: |b|^2 (canonical sum of the setup's per-camera shares) and the iteration count.
// ... and the CG scalars of iteration 0 (β = 0, rz_0, the convergence test), published as every
// later iteration's are by publish_next.
__global__ __launch_bounds__(256) void bas_pcg_init(int n_cam, const double* __restrict__ rzc,
                                                    const double* __restrict__ bb_c, double tol,
                                                    PcgState* __restrict__ st) {
    pcg_init_body(n_cam, rzc, bb_c, tol, st);
}

// Fixed-order sum over a 1024-thread block (16 waves); returns the total to every thread.
__device__ __forceinline__ double block_sum1024(double v, double* red) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_down(v, off, 64);
    const int tid = threadIdx.x;
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) s += red[w];
    __syncthreads();
    return s;
}

// ---- back-substitution and the LM model terms -------------------------------------------------

// Thread per point: δp = -v_g - V_d⁻¹ Σ_o W_oᵀ δc; per-point share of gᵀδ + ... :
//   mterm[p] = (g_p·δp,  δpᵀ V δp + 2 Σ_o δc_cᵀ W_o δp)   (the undamped JᵀJ)
__global__ __launch_bounds__(256) void bas_backsub(int n_pt, int n_obs,
                                                   const int32_t* __restrict__ pt_ptr,
                                                   const int32_t* __restrict__ cam_idx,
                                                   const double* __restrict__ Wp,
                                                   const double* __restrict__ V,
                                                   const double* __restrict__ Vinv,
                                                   const double* __restrict__ vg,
                                                   const double* __restrict__ gp,
                                                   const double* __restrict__ dc,
                                                   double* __restrict__ dp,
                                                   double* __restrict__ mpart) {
    // PG lanes per point (as bas_pcg_point): lane j sums observations j, j+PG, ...
    __shared__ double red[2][4];
    const int g = blockIdx.x * (blockDim.x / PG) + threadIdx.x / PG;
    const int j = threadIdx.x % PG;
    const bool valid = g < n_pt;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    const size_t n = (size_t)n_obs;
    const int o1 = valid ? pt_ptr[g + 1] : 0;
    for (int o = (valid ? pt_ptr[g] : 0) + j; o < o1; o += PG) {
        const double* Wo = Wp + o;
        const double* x = dc + 8 * (size_t)cam_idx[o];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double xi = x[i];
            s0 += Wo[(3 * i) * n] * xi;
            s1 += Wo[(3 * i + 1) * n] * xi;
            s2 += Wo[(3 * i + 2) * n] * xi;
        }
    }
#pragma unroll
    for (int off = PG / 2; off >= 1; off >>= 1) {
        s0 += __shfl_down(s0, off, PG);
        s1 += __shfl_down(s1, off, PG);
        s2 += __shfl_down(s2, off, PG);
    }
    double m0 = 0.0, m1 = 0.0;
    if (valid && j == 0) {
        const double* Vi = Vinv + 9 * (size_t)g;
        const double* gv = vg + 3 * (size_t)g;
        const double d0 = -gv[0] - (Vi[0] * s0 + Vi[1] * s1 + Vi[2] * s2);
        const double d1 = -gv[1] - (Vi[3] * s0 + Vi[4] * s1 + Vi[5] * s2);
        const double d2 = -gv[2] - (Vi[6] * s0 + Vi[7] * s1 + Vi[8] * s2);
        dp[3 * (size_t)g] = d0;
        dp[3 * (size_t)g + 1] = d1;
        dp[3 * (size_t)g + 2] = d2;
        const double* gg = gp + 3 * (size_t)g;
        const double* Vp = V + 9 * (size_t)g;
        m0 = gg[0] * d0 + gg[1] * d1 + gg[2] * d2;
        const double v0 = Vp[0] * d0 + Vp[1] * d1 + Vp[2] * d2;
        const double v1 = Vp[3] * d0 + Vp[4] * d1 + Vp[5] * d2;
        const double v2 = Vp[6] * d0 + Vp[7] * d1 + Vp[8] * d2;
        // Σ_o δcᵀ W_o δp = (Σ_o W_oᵀ δc)·δp = s·δp
        m1 = d0 * v0 + d1 * v1 + d2 * v2 + 2.0 * (s0 * d0 + s1 * d1 + s2 * d2);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        m0 += __shfl_down(m0, off, 64);
        m1 += __shfl_down(m1, off, 64);
    }
    const int tid = threadIdx.x;
    if ((tid & 63) == 0) { red[0][tid >> 6] = m0; red[1][tid >> 6] = m1; }
    __syncthreads();
    if (tid == 0) {
        mpart[2 * (size_t)blockIdx.x] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        mpart[2 * (size_t)blockIdx.x + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}

// Chunk mode: bas_backsub over chunk-aligned point groups.  Block (k, b) of the nck x BPB grid
// takes chunk k's point groups b, b + BPB, ... (32 points each, PG lanes per point, bas_backsub's
// per-point code) and accumulates each lane's model terms in that order; then the wave trees and
// the 4 waves in order -> mpart[(k BPB + b)][2].  The order depends only on the chunk.
constexpr int BPB = 64;
// W element m of observation o at Wp[o * so + m * sm]: the SoA planes (so 1, sm n_obs) or K3's
// row-major W (so 24, sm 1; the explicit Schur solve skips the SoA copy) — the same values, the same
// sums.
__global__ __launch_bounds__(256) void bas_backsub_ck(sfm::ChunkOff cpt, int n_obs,
                                                      long long so, long long sm,
                                                      const int32_t* __restrict__ pt_ptr,
                                                      const int32_t* __restrict__ cam_idx,
                                                      const double* __restrict__ Wp,
                                                      const double* __restrict__ V,
                                                      const double* __restrict__ Vinv,
                                                      const double* __restrict__ vg,
                                                      const double* __restrict__ gp,
                                                      const double* __restrict__ dc,
                                                      double* __restrict__ dp,
                                                      double* __restrict__ mpart) {
    __shared__ double red[2][4];
    const int k = blockIdx.x / BPB, b = blockIdx.x - k * BPB;
    const int p0 = cpt.v[k], p1 = cpt.v[k + 1];
    const int j = threadIdx.x % PG;
    double m0 = 0.0, m1 = 0.0;
    for (int gb = p0 + b * (256 / PG); gb < p1; gb += BPB * (256 / PG)) {
        const int g = gb + threadIdx.x / PG;
        const bool valid = g < p1;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        const int o1 = valid ? pt_ptr[g + 1] : 0;
        for (int o = (valid ? pt_ptr[g] : 0) + j; o < o1; o += PG) {
            const double* Wo = Wp + o * so;
            const double* x = dc + 8 * (size_t)cam_idx[o];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const double xi = x[i];
                s0 += Wo[(3 * i) * sm] * xi;
                s1 += Wo[(3 * i + 1) * sm] * xi;
                s2 += Wo[(3 * i + 2) * sm] * xi;
            }
        }
#pragma unroll
        for (int off = PG / 2; off >= 1; off >>= 1) {
            s0 += __shfl_down(s0, off, PG);
            s1 += __shfl_down(s1, off, PG);
            s2 += __shfl_down(s2, off, PG);
        }
        if (valid && j == 0) {
            const double* Vi = Vinv + 9 * (size_t)g;
            const double* gv = vg + 3 * (size_t)g;
            const double d0 = -gv[0] - (Vi[0] * s0 + Vi[1] * s1 + Vi[2] * s2);
            const double d1 = -gv[1] - (Vi[3] * s0 + Vi[4] * s1 + Vi[5] * s2);
            const double d2 = -gv[2] - (Vi[6] * s0 + Vi[7] * s1 + Vi[8] * s2);
            dp[3 * (size_t)g] = d0;
            dp[3 * (size_t)g + 1] = d1;
            dp[3 * (size_t)g + 2] = d2;
            const double* gg = gp + 3 * (size_t)g;
            const double* Vp = V + 9 * (size_t)g;
            m0 += gg[0] * d0 + gg[1] * d1 + gg[2] * d2;
            const double v0 = Vp[0] * d0 + Vp[1] * d1 + Vp[2] * d2;
            const double v1 = Vp[3] * d0 + Vp[4] * d1 + Vp[5] * d2;
            const double v2 = Vp[6] * d0 + Vp[7] * d1 + Vp[8] * d2;
            m1 += d0 * v0 + d1 * v1 + d2 * v2 + 2.0 * (s0 * d0 + s1 * d1 + s2 * d2);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        m0 += __shfl_down(m0, off, 64);
        m1 += __shfl_down(m1, off, 64);
    }
    const int tid = threadIdx.x;
    if ((tid & 63) == 0) { red[0][tid >> 6] = m0; red[1][tid >> 6] = m1; }
    __syncthreads();
    if (tid == 0) {
        mpart[2 * (size_t)blockIdx.x] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        mpart[2 * (size_t)blockIdx.x + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}

// Chunk mode, one wave: chunk k's model terms = its BPB block partials (one per lane, xor tree);
// exp: this rank's chunks to out[k][2] (the exchange form); else the canonical tree -> out[0..2).
// gathered (ntot > 0, in = the gathered [ntot][2]): out[0..2) = the tree of in.
__device__ __forceinline__ void mchunk_terms(int lane, int nck, int ntot,
                                             const double* __restrict__ mpart,
                                             const double* __restrict__ in, double (&a)[16],
                                             double (&b)[16]) {
    if (ntot > 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            a[k] = k < ntot ? in[2 * k] : 0.0;
            b[k] = k < ntot ? in[2 * k + 1] : 0.0;
        }
    } else {
        static_assert(BPB == 64, "one block partial per lane");
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            double u = 0.0, v = 0.0;
            if (k < nck) {
                u = mpart[2 * ((size_t)k * BPB + lane)];
                v = mpart[2 * ((size_t)k * BPB + lane) + 1];
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    u += __shfl_xor(u, off, 64);
                    v += __shfl_xor(v, off, 64);
                }
            }
            a[k] = u;
            b[k] = v;
        }
    }
}

// The non-export form's tree by one wave (lane < 64): out[0..2) from lane 0.
__device__ __forceinline__ void mchunk_tree(int lane, int nck, int ntot,
                                            const double* __restrict__ mpart,
                                            const double* __restrict__ in, double* out) {
    double a[16], b[16];
    mchunk_terms(lane, nck, ntot, mpart, in, a, b);
    if (lane != 0) return;
    out[0] = sfm::chunk_tree16(a);
    out[1] = sfm::chunk_tree16(b);
}

__global__ __launch_bounds__(64) void bas_mchunk(int nck, int exp, int ntot,
                                                 const double* __restrict__ mpart,
                                                 const double* __restrict__ in,
                                                 double* __restrict__ out) {
    const int lane = threadIdx.x;
    if (!exp) {
        mchunk_tree(lane, nck, ntot, mpart, in, out);
        return;
    }
    double a[16], b[16];
    mchunk_terms(lane, nck, ntot, mpart, in, a, b);
    if (lane != 0) return;
    for (int k = 0; k < nck; ++k) { out[2 * k] = a[k]; out[2 * k + 1] = b[k]; }
}

// Sharded solve, one block: this rank's point-block partials of bas_backsub summed into
// comm[0..2) (fixed order), the operand of the all-reduce that precedes bas_model.
__global__ __launch_bounds__(1024) void bas_mpart_total(int n_pblk, const double* __restrict__ mpart,
                                                        double* __restrict__ comm) {
    __shared__ double red[16];
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < n_pblk; k += 1024) { a += mpart[2 * (size_t)k]; b += mpart[2 * (size_t)k + 1]; }
    const double sa = block_sum1024(a, red);
    const double sb = block_sum1024(b, red);
    if (threadIdx.x == 0) { comm[0] = sa; comm[1] = sb; }
}

// One block: camera terms (g_c·δc, δcᵀ U δc) + the point-block partials -> info.
//   info = {iterations, |r|/|b|, gᵀδ, δᵀ JᵀJ δ, preconditioner fallback (0/1)}
// Chunk mode (nck > 0 or ntot > 0): the back-substitution's model partials are the chunk tree of
// bas_mchunk's non-export form — formed here by wave 0 (the same code, the same bits) and taken by
// thread 0 where it took the separate kernel's total, one launch fewer per solve.
__global__ __launch_bounds__(1024) void bas_model(int n_cam, int n_pblk, const double* __restrict__ U,
                                                  const double* __restrict__ gc,
                                                  const double* __restrict__ dc,
                                                  const double* __restrict__ mpart,
                                                  const double* __restrict__ rrc,
                                                  const PcgState* __restrict__ st,
                                                  const int32_t* __restrict__ bad,
                                                  double* __restrict__ info, int nck, int ntot,
                                                  const double* __restrict__ min) {
    __shared__ double red[16];
    __shared__ double mt[2];
    const int tid = threadIdx.x;
    if ((nck > 0 || ntot > 0) && tid < 64) mchunk_tree(tid, nck, ntot, mpart, min, mt);
    double a = 0.0, b = 0.0;
    for (int c = tid; c < n_cam; c += 1024) {
        const double* Uc = U + 64 * (size_t)c;
        const double* d = dc + 8 * (size_t)c;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < 8; ++j) s += Uc[8 * i + j] * d[j];
            b += d[i] * s;
            a += gc[8 * (size_t)c + i] * d[i];
        }
    }
    if (nck > 0 || ntot > 0) {
        __syncthreads();
        if (tid == 0) { a += mt[0]; b += mt[1]; }
    } else {
        for (int k = tid; k < n_pblk; k += 1024) { a += mpart[2 * (size_t)k]; b += mpart[2 * (size_t)k + 1]; }
    }
    const double ga = block_sum1024(a, red);
    const double qb = block_sum1024(b, red);
    const int it = st->iter;
    const double rr = canon_sum(rrc + (size_t)(it & 1) * n_cam, n_cam, red);
    if (tid == 0) {
        info[0] = (double)it;
        info[1] = st->bb > 0.0 ? sqrt(rr / st->bb) : 0.0;
        info[2] = ga;
        info[3] = qb;
        info[4] = (double)*bad;
    }
}

}  // namespace

// Device workspace of a solve (one carve for the unsharded solve and every stage of the sharded
// one: the same sizes give the same pointers, so state persists across the stage calls).
// Chunk mode of a call (sfm_ba_set_chunks), read from the context.
struct ChunkArgs {
    const int32_t* cb = nullptr;   // [n_cam][nck + 1] positions in cam_obs (nullptr: off)
    int nck = 0, ntot = 0;
    sfm::ChunkOff cpt;             // local chunk point offsets
};
static ChunkArgs chunk_args(const sfm_ctx* ctx) {
    ChunkArgs a;
    if (ctx->ba_nchunk > 0) {
        a.cb = ctx->ba_cam_bounds;
        a.nck = ctx->ba_nchunk;
        a.ntot = ctx->ba_ntotal;
        for (int k = 0; k <= a.nck; ++k) a.cpt.v[k] = ctx->ba_chunk_pt[k];
    }
    return a;
}

struct SolveWs {
    double *Vinv, *vg, *Ud, *Mc, *r, *z, *pv, *q, *rzc, *rrc, *pq, *mpart, *mtot, *Wp, *u;
    double *Scc = nullptr, *T = nullptr, *Tpart = nullptr, *pv2 = nullptr;   // explicit S only
    PcgState* state;
    int32_t* bad;
    int32_t* long_cnt;   // long-track points (bas_point_setup)
    int32_t* long_list;
    int lblk;            // long-track blocks ahead of the point pass's point blocks
    int32_t* ptc;
    int pblk, gblk, vblk;
};

static int solve_ws(sfm_ctx* ctx, int32_t n_cam, int32_t n_pt, int32_t n_obs, SolveWs& w) {
    // workspace: Vinv 9 | vg 3 per point; Ud 64 | M 64 | r z p q 8 each | rz, rr partials
    // (2 parity slots each) | p·q per camera; backsub partials; state; bad flag; per observation
    // Wp 24 | u 8 doubles | ptc
    w.pblk = std::max(1, (n_pt + 255) / 256);
    const size_t np = (size_t)std::max(n_pt, 1), nc = (size_t)n_cam;
    const size_t b_pt = sfm::align_up(sizeof(double) * 12 * np + sizeof(int32_t) * np, 256);
    const size_t b_cam = sfm::align_up(sizeof(double) * (128 + 32 + 5) * nc, 256);
    w.gblk = std::max(1, (n_pt + 256 / PG - 1) / (256 / PG));  // PG lanes per point
    // backsub partials: per point block, or (chunk mode) BPB per chunk + the combined 2 terms
    const size_t n_part = std::max((size_t)2 * w.gblk, (size_t)2 * SFM_BA_MAX_CHUNKS * BPB + 2);
    const size_t b_part = sfm::align_up(sizeof(double) * n_part, 256);
    const size_t no = (size_t)std::max(n_obs, 1);
    const size_t b_soa = sfm::align_up(sizeof(double) * 32 * no + sizeof(int32_t) * no, 256);
    // explicit reduced camera system: S_cc, T, its chunk partials, p in two parity slots
    const size_t ns = (size_t)ctx->ba_nslot, ngr = (size_t)std::max(ctx->ba_ngroup, 1);
    const size_t b_ex = ns > 0 ? sfm::align_up(sizeof(double) * (64 * nc + 64 * ns + 64 * ngr + 16 * nc), 256) : 0;
    char* ws = (char*)sfm::workspace(ctx, b_pt + b_cam + b_part + 512 + b_soa + b_ex);
    if (!ws) return SFM_ERR_NOMEM;
    if (ns > 0) {
        w.Scc = (double*)(ws + b_pt + b_cam + b_part + 512 + b_soa);
        w.T = w.Scc + 64 * nc;
        w.Tpart = w.T + 64 * ns;
        w.pv2 = w.Tpart + 64 * ngr;
    }
    w.Vinv = (double*)ws;
    w.vg = w.Vinv + 9 * np;
    w.long_list = (int32_t*)(w.vg + 3 * np);
    w.Ud = (double*)(ws + b_pt);
    w.Mc = w.Ud + 64 * nc;
    w.r = w.Mc + 64 * nc;
    w.z = w.r + 8 * nc;
    w.pv = w.z + 8 * nc;
    w.q = w.pv + 8 * nc;
    w.rzc = w.q + 8 * nc;    // [2][n_cam]
    w.rrc = w.rzc + 2 * nc;  // [2][n_cam]
    w.pq = w.rrc + 2 * nc;
    w.mpart = (double*)(ws + b_pt + b_cam);
    w.mtot = w.mpart + n_part - 2;   // chunk mode: the combined model terms
    w.state = (PcgState*)(ws + b_pt + b_cam + b_part);
    w.bad = (int32_t*)(ws + b_pt + b_cam + b_part + 256);
    w.long_cnt = w.bad + 1;
    w.lblk = n_obs > LONG_OBS ? LONG_BLOCKS : 0;
    w.Wp = (double*)(ws + b_pt + b_cam + b_part + 512);
    w.u = w.Wp + 24 * no;
    w.ptc = (int32_t*)(w.u + 8 * no);
    w.vblk = (8 * n_cam + 255) / 256;
    return SFM_OK;
}

// Point setup, SoA W and the camera setup (phase 0: whole; 1: partial sums -> comm).
static int solve_setup(hipStream_t st, const SolveWs& w, const ChunkArgs& ck, int32_t n_cam,
                       int32_t n_pt, int32_t n_obs,
                       const int32_t* pt_idx, const int32_t* pt_ptr, const int32_t* cam_ptr,
                       const int32_t* cam_obs, const double* U, const double* V, const double* W,
                       const double* gc, const double* gp, double lam, double* dc, int phase,
                       double* comm, bool soa = true) {
    SFM_HIP_CHECK(hipMemsetAsync(w.bad, 0, 2 * sizeof(int32_t), st));  // bad flag, long count
    // the point set-up and the SoA copy / camera-major point ids (bas_soa's work) in one launch
    const int pb = n_pt > 0 ? w.pblk : 0, ob = n_obs > 0 ? (n_obs + 255) / 256 : 0;
    if (pb + ob > 0) {
        hipLaunchKernelGGL(bas_point_setup, dim3(pb + ob), dim3(256), 0, st, n_pt, pt_ptr, V, gp,
                           lam, w.Vinv, w.vg, w.long_list, w.long_cnt, pb, n_obs, cam_obs, pt_idx,
                           W, soa ? w.Wp : nullptr, w.ptc);
        SFM_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(bas_camera_setup, dim3(n_cam), dim3(CT), 0, st, n_cam, n_obs, cam_ptr,
                       w.ptc, cam_obs, U, W, w.Vinv, w.vg, gc, lam, w.Ud, w.Mc, dc, w.r, w.z, w.pv,
                       w.rzc, w.rrc, w.bad, phase, comm, ck.cb, ck.nck, ck.ntot, w.Scc, w.pv2);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

// Back-substitution + the model terms (chunk mode: chunk-aligned blocks, combined by bas_model's
// chunk tree, or exported to comm[k][2] when exp).  Returns the (n_pblk, mpart) pair bas_model reads.
static int solve_backsub(hipStream_t st, const SolveWs& w, const ChunkArgs& ck, int32_t n_pt,
                         int32_t n_obs, const int32_t* pt_ptr, const int32_t* cam_idx,
                         const double* V, const double* gp, const double* dc, double* dp, bool exp,
                         double* comm, const double* W = nullptr) {
    if (!ck.cb) {
        hipLaunchKernelGGL(bas_backsub, dim3(w.gblk), dim3(256), 0, st, n_pt, n_obs, pt_ptr,
                           cam_idx, w.Wp, V, w.Vinv, w.vg, gp, dc, dp, w.mpart);
        SFM_HIP_CHECK(hipGetLastError());
        return SFM_OK;
    }
    // W given: row-major (the explicit Schur solve made no SoA copy)
    hipLaunchKernelGGL(bas_backsub_ck, dim3(ck.nck * BPB), dim3(256), 0, st, ck.cpt, n_obs,
                       W ? 24LL : 1LL, W ? 1LL : (long long)n_obs, pt_ptr, cam_idx, W ? W : w.Wp,
                       V, w.Vinv, w.vg, gp, dc, dp, w.mpart);
    SFM_HIP_CHECK(hipGetLastError());
    if (exp) {   // the non-export tree is formed by bas_model
        hipLaunchKernelGGL(bas_mchunk, dim3(1), dim3(64), 0, st, ck.nck, 1, 0, w.mpart,
                           (const double*)nullptr, comm);
        SFM_HIP_CHECK(hipGetLastError());
    }
    return SFM_OK;
}

// Explicit S: this problem's group partials of T ([n_seg][64], one wave per group) into out.
static int schur_build(const sfm_ctx* ctx, hipStream_t st, const SolveWs& w, const int32_t* pt_idx,
                       const double* W, double* out) {
    if (ctx->ba_nseg > 0) {
        hipLaunchKernelGGL(bas_schur_build, dim3(ctx->ba_nseg), dim3(64), 0, st, ctx->ba_nseg,
                           ctx->ba_ninst, ctx->ba_seg, ctx->ba_inst, pt_idx, W, w.Vinv, out);
        SFM_HIP_CHECK(hipGetLastError());
    }
    return SFM_OK;
}

// Explicit S: T from the whole problem's group partials (slot trees; p's parity slots are zeroed by
// bas_camera_setup).
static int schur_finish(const sfm_ctx* ctx, hipStream_t st, const SolveWs& w, int32_t n_cam,
                        const double* parts, double tol) {
    const long long n = (long long)ctx->ba_nslot * 64;
    const int tblk = (int)((n + 255) / 256);
    hipLaunchKernelGGL(bas_schur_tree, dim3((unsigned)tblk + 1), dim3(256), 0, st, ctx->ba_nslot,
                       ctx->ba_sg_ptr, ctx->ba_sg, ctx->ba_gk, parts, w.T, tblk, n_cam, w.rzc, w.rrc,
                       tol, w.state);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;   // p's parity slots: zeroed by bas_camera_setup
}

// One explicit CG iteration: the S product, then the vector update (p_k in parity slot k & 1).
static void schur_iter(const sfm_ctx* ctx, hipStream_t st, const SolveWs& w, int k, int32_t n_cam,
                       double* dc, double tol) {
    hipLaunchKernelGGL(bas_pcg_spmv, dim3((n_cam + 3) / 4), dim3(256), 0, st, k, n_cam,
                       ctx->ba_row_ptr, ctx->ba_row_ent, ctx->ba_slot_cam, w.T, w.Scc, w.z, w.pv2,
                       w.state, w.q, w.pq);
    hipLaunchKernelGGL(bas_pcg_vec, dim3(w.vblk), dim3(256), 0, st, k, n_cam, w.Mc, dc, w.r, w.z,
                       w.pv2 + (size_t)(k & 1) * 8 * n_cam, w.q, w.pq, w.rzc, w.rrc, w.state, tol);
}

// Iterations enqueued after a poll's flag copy before the host waits for it (sfm_ba_solve).
constexpr int POLL_AHEAD = 2;

// The flag copy of a look-ahead poll: state->done -> pinned[0], then ctx->poll_ev.
static int solve_poll_issue(sfm_ctx* ctx, hipStream_t st, const SolveWs& w) {
    if (!ctx->pinned)
        SFM_HIP_CHECK(hipHostMalloc((void**)&ctx->pinned, 64, hipHostMallocDefault));
    if (!ctx->poll_ev) SFM_HIP_CHECK(hipEventCreateWithFlags(&ctx->poll_ev, hipEventDisableTiming));
    SFM_HIP_CHECK(hipMemcpyAsync(ctx->pinned, &w.state->done, sizeof(int32_t),
                                 hipMemcpyDeviceToHost, st));
    SFM_HIP_CHECK(hipEventRecord(ctx->poll_ev, st));
    return SFM_OK;
}

static int solve_poll(sfm_ctx* ctx, hipStream_t st, const SolveWs& w, int32_t* done) {
    if (!ctx->pinned)
        SFM_HIP_CHECK(hipHostMalloc((void**)&ctx->pinned, 64, hipHostMallocDefault));
    SFM_HIP_CHECK(hipMemcpyAsync(ctx->pinned, &w.state->done, sizeof(int32_t),
                                 hipMemcpyDeviceToHost, st));
    SFM_HIP_CHECK(hipStreamSynchronize(st));
    *done = ctx->pinned[0];
    return SFM_OK;
}

#define SFM_SOLVE_ARGS_CHECK(NAME)                                                                \
    SFM_REQUIRE(ctx != nullptr && prm != nullptr, NAME ": ctx/prm is NULL");                     \
    SFM_REQUIRE(n_cam > 0 && n_pt >= 0 && n_obs >= 0, NAME ": bad size");                        \
    SFM_REQUIRE(prm->max_iter >= 0 && prm->lambda >= 0.0 && prm->tol >= 0.0,                      \
                NAME ": max_iter, lambda and tol must be >= 0");                                  \
    /* per-observation arrays may be NULL without observations, per-point ones without points */ \
    SFM_REQUIRE(cam_ptr && U && gc && dc && info &&                                               \
                    (n_obs == 0 || (cam_idx && pt_idx && cam_obs && W)) &&                        \
                    (n_pt == 0 || (pt_ptr && V && gp && dp)),                                     \
                NAME ": NULL array")

extern "C" int sfm_ba_solve(sfm_ctx* ctx, int32_t n_cam, int32_t n_pt, int32_t n_obs,
                            const int32_t* cam_idx, const int32_t* pt_idx, const int32_t* pt_ptr,
                            const int32_t* cam_ptr, const int32_t* cam_obs, const double* U,
                            const double* V, const double* W, const double* gc, const double* gp,
                            const sfm_ba_solve_params* prm, double* dc, double* dp,
                            double* info) {
    SFM_SOLVE_ARGS_CHECK("sfm_ba_solve");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    SolveWs w;
    if (solve_ws(ctx, n_cam, n_pt, n_obs, w) != SFM_OK) return SFM_ERR_NOMEM;
    const double lam = prm->lambda, tol = prm->tol;
    const ChunkArgs ck = chunk_args(ctx);
    SFM_REQUIRE(ck.ntot == 0, "sfm_ba_solve: chunk mode of a shard (n_total > 0) needs the stages");
    if (ck.cb)
        SFM_REQUIRE(ck.cpt.v[ck.nck] == n_pt, "sfm_ba_solve: chunk offsets do not match n_pt");
    const bool ex = ctx->ba_nslot > 0;   // explicit reduced camera system (sfm_ba_set_schur)
    SFM_REQUIRE(!ex || ck.cb, "sfm_ba_solve: the explicit Schur system needs chunk mode");
    const int rc = solve_setup(st, w, ck, n_cam, n_pt, n_obs, pt_idx, pt_ptr, cam_ptr, cam_obs, U,
                               V, W, gc, gp, lam, dc, 0, nullptr, !ex);
    if (rc != SFM_OK) return rc;
    if (ex) {
        if (schur_build(ctx, st, w, pt_idx, W, w.Tpart) != SFM_OK) return SFM_ERR_HIP;
        if (schur_finish(ctx, st, w, n_cam, w.Tpart, tol) != SFM_OK) return SFM_ERR_HIP;   // + init
    } else {
        hipLaunchKernelGGL(bas_pcg_init, dim3(1), dim3(256), 0, st, n_cam, w.rzc, w.rrc, tol, w.state);
    }
    SFM_HIP_CHECK(hipGetLastError());
    // 0 (the zero-initialised struct) = every 8 iterations, the library default; < 0 = never
    // (no host synchronisation: fully asynchronous, capturable in a hip graph).  A stream under
    // capture never polls, whatever prm->poll says: a sfm_version-1 caller that captures with a
    // zero-initialised struct (then "never") keeps working, with the same results.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    SFM_HIP_CHECK(hipStreamIsCapturing(st, &cap));
    const int poll = cap != hipStreamCaptureStatusNone ? -1
                   : prm->poll == 0 ? SFM_BA_POLL_DEFAULT : prm->poll;
    const int first = prm->poll_first > 0 ? prm->poll_first : std::max(poll, 1);
    // Look-ahead poll: at a poll point the flag is copied to pinned memory behind an event and
    // POLL_AHEAD more iterations are enqueued before the host waits on that event, so the GPU
    // runs them while the host wakes up instead of idling through the round trip (a converged
    // flag makes them empty launches; bas_model reads the last real iteration's slot).
    static const int ahead = [] {
        const char* e = getenv("SFM_BA_POLL_AHEAD");
        return e ? std::max(0, atoi(e)) : POLL_AHEAD;
    }();
    int check_at = -1;   // iteration at which the pending flag copy is read
    for (int k = 0; k < prm->max_iter; ++k) {
        // state->done is set by bas_pcg_point of the first iteration after convergence: once it
        // reads 1, every later iteration would exit at once, so stop enqueueing them
        if (poll > 0 && k >= first && (k - first) % poll == 0 && check_at < 0) {
            if (ahead == 0) {
                int32_t done = 0;
                const int prc = solve_poll(ctx, st, w, &done);
                if (prc != SFM_OK) return prc;
                if (done) break;
            } else {
                if (solve_poll_issue(ctx, st, w) != SFM_OK) return SFM_ERR_HIP;
                check_at = k + ahead;
            }
        }
        if (k == check_at) {
            SFM_HIP_CHECK(hipEventSynchronize(ctx->poll_ev));
            check_at = -1;
            if (ctx->pinned[0]) break;
        }
        if (ex) {
            schur_iter(ctx, st, w, k, n_cam, dc, tol);
            continue;
        }
        hipLaunchKernelGGL(bas_pcg_point, dim3(w.gblk + w.lblk), dim3(256), 0, st, k, n_pt, n_cam,
                           n_obs, pt_ptr, cam_idx, w.Wp, w.Vinv, w.z, w.pv, w.rzc, w.rrc, tol,
                           w.state, w.u, w.lblk, w.long_list, w.long_cnt);
        hipLaunchKernelGGL(bas_pcg_camera, dim3(n_cam), dim3(CC), 0, st, k, n_cam, cam_ptr,
                           cam_obs, w.u, w.Ud, w.z, w.pv, w.state, w.q, w.pq, 0, nullptr, ck.cb,
                           ck.nck, 0);
        hipLaunchKernelGGL(bas_pcg_vec, dim3(w.vblk), dim3(256), 0, st, k, n_cam, w.Mc, dc, w.r,
                           w.z, w.pv, w.q, w.pq, w.rzc, w.rrc, w.state, tol);
    }
    SFM_HIP_CHECK(hipGetLastError());
    if (solve_backsub(st, w, ck, n_pt, n_obs, pt_ptr, cam_idx, V, gp, dc, dp, false, nullptr,
                      ex ? W : nullptr) != SFM_OK)
        return SFM_ERR_HIP;
    hipLaunchKernelGGL(bas_model, dim3(1), dim3(1024), 0, st, n_cam, ck.cb ? 1 : w.gblk, U, gc, dc,
                       (const double*)w.mpart, w.rrc, w.state, w.bad, info, ck.cb ? ck.nck : 0, 0,
                       (const double*)nullptr);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

// The sharded solve as caller-driven stages (no callbacks across the ABI): the caller all-reduces
// comm between the stages that produce partial sums and the ones that consume them.  Every stage
// after an all-reduce works on replicated camera-space values, so all ranks take the same CG
// decisions and issue the same collectives.
extern "C" int sfm_ba_solve_stage(sfm_ctx* ctx, int32_t stage, int32_t k, int32_t n_cam,
                                  int32_t n_pt, int32_t n_obs, const int32_t* cam_idx,
                                  const int32_t* pt_idx, const int32_t* pt_ptr,
                                  const int32_t* cam_ptr, const int32_t* cam_obs, const double* U,
                                  const double* V, const double* W, const double* gc,
                                  const double* gp, const sfm_ba_solve_params* prm, double* comm,
                                  double* dc, double* dp, double* info, int32_t* done) {
    SFM_SOLVE_ARGS_CHECK("sfm_ba_solve_stage");
    SFM_REQUIRE(comm != nullptr, "sfm_ba_solve_stage: comm is NULL");
    SFM_REQUIRE(stage >= SFM_BA_STAGE_SETUP && stage <= SFM_BA_STAGE_SCHUR,
                "sfm_ba_solve_stage: unknown stage");
    SFM_REQUIRE(stage != SFM_BA_STAGE_POLL || done != nullptr, "sfm_ba_solve_stage: done is NULL");
    SFM_REQUIRE(k >= 0, "sfm_ba_solve_stage: k must be >= 0");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    SolveWs w;
    if (solve_ws(ctx, n_cam, n_pt, n_obs, w) != SFM_OK) return SFM_ERR_NOMEM;
    const double lam = prm->lambda, tol = prm->tol;
    // up to FINISH_VEC_MAX_CAM cameras an iteration ends in one launch after the all-reduce
    const bool fused = n_cam <= FINISH_VEC_MAX_CAM;
    // chunk mode: the exchange is an all-gather of chunk partials (sfm_ba_set_chunks, n_total > 0)
    const ChunkArgs ck = chunk_args(ctx);
    SFM_REQUIRE(!ck.cb || ck.ntot > 0, "sfm_ba_solve_stage: chunk mode needs n_total > 0");
    if (ck.cb)
        SFM_REQUIRE(ck.cpt.v[ck.nck] == n_pt, "sfm_ba_solve_stage: chunk offsets do not match n_pt");
    const bool ex = ctx->ba_nslot > 0;   // explicit reduced camera system (sfm_ba_set_schur)
    SFM_REQUIRE(!ex || ck.cb, "sfm_ba_solve_stage: the explicit Schur system needs chunk mode");
    SFM_REQUIRE(stage != SFM_BA_STAGE_SCHUR || ex, "sfm_ba_solve_stage: SCHUR without sfm_ba_set_schur");
    switch (stage) {
    case SFM_BA_STAGE_SETUP:  // -> comm[0, 44 n_cam) (chunk mode: [n_chunk][n_cam][44])
        return solve_setup(st, w, ck, n_cam, n_pt, n_obs, pt_idx, pt_ptr, cam_ptr, cam_obs, U, V,
                           W, gc, gp, lam, dc, 1, comm, !ex);
    case SFM_BA_STAGE_SCHUR:  // explicit S: this shard's group partials of T -> comm [n_seg][64]
        return schur_build(ctx, st, w, pt_idx, W, comm);
    case SFM_BA_STAGE_SETUP_FINISH:
        hipLaunchKernelGGL(bas_camera_setup, dim3(n_cam), dim3(CT), 0, st, n_cam, n_obs, cam_ptr,
                           w.ptc, cam_obs, U, W, w.Vinv, w.vg, gc, lam, w.Ud, w.Mc, dc, w.r, w.z,
                           w.pv, w.rzc, w.rrc, w.bad, 2, comm, ck.cb, ck.nck, ck.ntot, w.Scc, w.pv2);
        SFM_HIP_CHECK(hipGetLastError());
        if (ex) {   // the tree launch also forms the CG's iteration-0 scalars
            if (schur_finish(ctx, st, w, n_cam, comm + (size_t)ck.ntot * 44 * n_cam, tol) != SFM_OK)
                return SFM_ERR_HIP;
        } else {
            hipLaunchKernelGGL(bas_pcg_init, dim3(1), dim3(256), 0, st, n_cam, w.rzc, w.rrc, tol,
                               w.state);
        }
        break;
    case SFM_BA_STAGE_ITER:  // -> comm[0, 8 n_cam)
        if (ex) {   // S is replicated: the whole iteration locally, nothing to exchange
            schur_iter(ctx, st, w, k, n_cam, dc, tol);
            break;
        }
        hipLaunchKernelGGL(bas_pcg_point, dim3(w.gblk + w.lblk), dim3(256), 0, st, k, n_pt, n_cam,
                           n_obs, pt_ptr, cam_idx, w.Wp, w.Vinv, w.z, w.pv, w.rzc, w.rrc, tol,
                           w.state, w.u, w.lblk, w.long_list, w.long_cnt);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(bas_pcg_camera, dim3(n_cam), dim3(CC), 0, st, k, n_cam, cam_ptr,
                           cam_obs, w.u, w.Ud, w.z, w.pv, w.state, w.q, w.pq, fused ? 3 : 1,
                           comm, ck.cb, ck.nck, ck.ntot);
        break;
    case SFM_BA_STAGE_ITER_FINISH:
        if (ex) break;   // done by ITER
        if (fused) {
            hipLaunchKernelGGL(bas_pcg_finish_vec, dim3((8 * n_cam + FV - 1) / FV), dim3(FV), 0, st,
                               k, n_cam, w.q, comm, w.pv, w.Mc, dc, w.r, w.z, w.rzc, w.rrc,
                               w.state, ck.cb ? ck.ntot : 0, tol);
            break;
        }
        hipLaunchKernelGGL(bas_pcg_camera, dim3(n_cam), dim3(CC), 0, st, k, n_cam, cam_ptr,
                           cam_obs, w.u, w.Ud, w.z, w.pv, w.state, w.q, w.pq, 2, comm, ck.cb,
                           ck.nck, ck.ntot);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(bas_pcg_vec, dim3(w.vblk), dim3(256), 0, st, k, n_cam, w.Mc, dc, w.r,
                           w.z, w.pv, w.q, w.pq, w.rzc, w.rrc, w.state, tol);
        break;
    case SFM_BA_STAGE_BACKSUB:  // -> comm[0, 2) (chunk mode: [n_chunk][2])
        if (ck.cb) {
            if (solve_backsub(st, w, ck, n_pt, n_obs, pt_ptr, cam_idx, V, gp, dc, dp, true, comm,
                              ex ? W : nullptr) != SFM_OK)
                return SFM_ERR_HIP;
            break;
        }
        hipLaunchKernelGGL(bas_backsub, dim3(w.gblk), dim3(256), 0, st, n_pt, n_obs, pt_ptr,
                           cam_idx, w.Wp, V, w.Vinv, w.vg, gp, dc, dp, w.mpart);
        SFM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(bas_mpart_total, dim3(1), dim3(1024), 0, st, w.gblk, w.mpart, comm);
        break;
    case SFM_BA_STAGE_MODEL:
        // chunk mode: the gathered [n_total][2] model partials' canonical tree, inside bas_model
        hipLaunchKernelGGL(bas_model, dim3(1), dim3(1024), 0, st, n_cam, 1, U, gc, dc,
                           (const double*)comm, w.rrc, w.state, w.bad, info, ck.cb ? ck.nck : 0,
                           ck.cb ? ck.ntot : 0, (const double*)comm);
        break;
    case SFM_BA_STAGE_POLL:
        return solve_poll(ctx, st, w, done);
    }
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}
#undef SFM_SOLVE_ARGS_CHECK

// ---- fixed parameters (gauge / known intrinsics) ------------------------------------------------
//
// Holds the parameters marked in `fixed` [n_cam][8] at their values for the solve: their rows and
// columns of U become those of the identity, their g_c entries and their rows of every W_o are
// zeroed.  The Schur system then decouples them with right-hand side 0, so δ = 0 for them exactly
// and the LM model terms (gᵀδ, δᵀJᵀJδ) do not see them.  Mirrors oracle/ba_lm.py fix_params().
namespace {
// One launch for both halves (blocks [0, ncb): (camera, i, j) of U and g_c; the rest (observation,
// row i of W_o)): a held parameter's U row / column become the identity's, its g_c entry and W rows 0.
__global__ __launch_bounds__(256) void bas_fix(int n_cam, int ncb, int n_obs,
                                               const int32_t* __restrict__ cam_idx,
                                               const uint8_t* __restrict__ fixed,
                                               double* __restrict__ U, double* __restrict__ gc,
                                               double* __restrict__ W) {
    if ((int)blockIdx.x < ncb) {
        const int g = blockIdx.x * blockDim.x + threadIdx.x;  // (camera, i, j)
        if (g >= n_cam * 64) return;
        const int c = g >> 6, i = (g >> 3) & 7, j = g & 7;
        const bool fi = fixed[8 * (size_t)c + i] != 0, fj = fixed[8 * (size_t)c + j] != 0;
        if (fi || fj) U[g] = (i == j) ? 1.0 : 0.0;
        if (j == 0 && fi) gc[8 * (size_t)c + i] = 0.0;
        return;
    }
    const int g = ((int)blockIdx.x - ncb) * blockDim.x + threadIdx.x;  // (observation, row i)
    if (g >= n_obs * 8) return;
    const int o = g >> 3, i = g & 7;
    if (fixed[8 * (size_t)cam_idx[o] + i]) {
        double* w = W + 24 * (size_t)o + 3 * i;
        w[0] = 0.0; w[1] = 0.0; w[2] = 0.0;
    }
}
}  // namespace

extern "C" int sfm_ba_fix_params(sfm_ctx* ctx, int32_t n_cam, int32_t n_obs,
                                 const int32_t* cam_idx, const uint8_t* fixed, double* U,
                                 double* W, double* gc) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ba_fix_params: ctx is NULL");
    SFM_REQUIRE(n_cam >= 0 && n_obs >= 0, "sfm_ba_fix_params: negative size");
    if (n_cam == 0) return SFM_OK;
    SFM_REQUIRE(fixed && U && gc && (n_obs == 0 || (cam_idx && W)),
                "sfm_ba_fix_params: NULL array");
    SFM_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int ncb = (64 * n_cam + 255) / 256, nob = n_obs > 0 ? (8 * n_obs + 255) / 256 : 0;
    hipLaunchKernelGGL(bas_fix, dim3(ncb + nob), dim3(256), 0, st, n_cam, ncb, n_obs, cam_idx,
                       fixed, U, gc, W);
    SFM_HIP_CHECK(hipGetLastError());
    return SFM_OK;
}

extern "C" int sfm_ba_set_schur(sfm_ctx* ctx, int32_t n_slot, const int32_t* slot_cam,
                                int32_t n_seg, const int32_t* seg, int32_t n_inst,
                                const int32_t* inst, const int32_t* row_ptr, int32_t n_ent,
                                const int32_t* row_ent, int32_t n_group, const int32_t* sg_ptr,
                                const int32_t* sg, const int32_t* gk) {
    SFM_REQUIRE(ctx != nullptr, "sfm_ba_set_schur: ctx is NULL");
    SFM_REQUIRE(n_slot >= 0 && n_seg >= 0 && n_inst >= 0 && n_ent >= 0 && n_group >= 0,
                "sfm_ba_set_schur: negative size");
    if (n_slot == 0) {
        ctx->ba_nslot = ctx->ba_nseg = ctx->ba_ninst = ctx->ba_nent = ctx->ba_ngroup = 0;
        ctx->ba_slot_cam = ctx->ba_seg = ctx->ba_inst = ctx->ba_row_ptr = ctx->ba_row_ent = nullptr;
        ctx->ba_sg_ptr = ctx->ba_sg = ctx->ba_gk = nullptr;
        return SFM_OK;
    }
    SFM_REQUIRE(n_seg <= n_group, "sfm_ba_set_schur: more local groups than the problem has");
    SFM_REQUIRE(slot_cam && row_ptr && sg_ptr && (n_seg == 0 || seg) && (n_inst == 0 || inst) &&
                    (n_ent == 0 || row_ent) && (n_group == 0 || (sg && gk)),
                "sfm_ba_set_schur: NULL array");
    ctx->ba_nslot = n_slot;
    ctx->ba_nseg = n_seg;
    ctx->ba_ninst = n_inst;
    ctx->ba_nent = n_ent;
    ctx->ba_ngroup = n_group;
    ctx->ba_slot_cam = slot_cam;
    ctx->ba_seg = seg;
    ctx->ba_inst = inst;
    ctx->ba_row_ptr = row_ptr;
    ctx->ba_row_ent = row_ent;
    ctx->ba_sg_ptr = sg_ptr;
    ctx->ba_sg = sg;
    ctx->ba_gk = gk;
    return SFM_OK;
}
