// Element-wise and reduction kernels of the multi-frame solver (16 frames as the N = 16 columns of the
// MFMA projections in multiframe.hip). Layouts: pixel-major [rows][16] for measurements, weights and
// forward projections (the MFMA B/D fragments), frame-major [16][ld] for solutions and corrections (the
// MFMA A operand of the forward projection), so each frame's solution row is contiguous.
//
// Per-frame semantics are those of the single-frame solver (sart_update.hip) and the reference GPU path
// (reference sartsolver_cuda.cpp:138-354): every frame has its own normalisation, saturation mask,
// convergence history, status and iteration count; finished frames are frozen.
#include "sart_common.hpp"

#include <math.h>
#include <stdexcept>

namespace sart {

constexpr int NF = kMfFrames;

// ghat = fp32(g / s_f); a = [ghat >= 0][len > tau_l] / len; gpos = max(ghat, 0); wo = a * ghat
__global__ __launch_bounds__(256) void k_mf_prep(const double* __restrict__ g, int64_t nrows, int64_t nrows_pad,
                                                 const double* __restrict__ norm, const float* __restrict__ ray_length,
                                                 float len_thres, float* __restrict__ ghat, float* __restrict__ arow,
                                                 float* __restrict__ gpos, float* __restrict__ wo) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // element of [rows_pad][16]
    if (i >= nrows_pad * NF) return;
    const int64_t row = i / NF;
    const int f = (int)(i % NF);
    float gh = 0.f, a = 0.f;
    if (row < nrows) {
        gh = (float)(g[i] / norm[f]);
        const float len = ray_length[row];
        const float inv_len = (len > len_thres) ? 1.f / len : 0.f;
        a = (gh >= 0.f) ? inv_len : 0.f;
    }
    ghat[i] = gh;
    arow[i] = a;
    gpos[i] = gh > 0.f ? gh : 0.f;
    wo[i] = a * gh;
}

// F = sum_s Fsplit[s] (fixed order); W = a F (log) or a (ghat - F) (linear); per-block, per-frame partial
// sums of F^2 in fp64 (deterministic: fixed thread-to-row assignment, fixed tree).
constexpr int kWRows = 256;  // rows per block
__global__ __launch_bounds__(256) void k_mf_weights(const float* __restrict__ Fs, int nsplit, int64_t nrows_pad,
                                                    const float* __restrict__ ghat, const float* __restrict__ arow,
                                                    int logmode, float* __restrict__ W, double* __restrict__ F2part) {
    __shared__ double red[256];
    const int f = threadIdx.x & 15, r16 = threadIdx.x >> 4;  // 16 rows x 16 frames per pass
    const int64_t r0 = (int64_t)blockIdx.x * kWRows;
    double acc = 0.0;
    for (int rr = r16; rr < kWRows; rr += 16) {
        const int64_t row = r0 + rr;
        if (row >= nrows_pad) break;
        const int64_t i = row * NF + f;
        float F = 0.f;
        for (int s = 0; s < nsplit; ++s) F += Fs[(int64_t)s * nrows_pad * NF + i];
        W[i] = logmode ? arow[i] * F : arow[i] * (ghat[i] - F);
        acc += (double)F * (double)F;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off >= 16; off >>= 1) {  // reduce over r16, keep the frame (low 4 bits)
        if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x < 16) F2part[(int64_t)blockIdx.x * NF + threadIdx.x] = red[threadIdx.x];
}

// D[f][v] = scale[v] * sum_s part[s][v][f] (transpose through LDS); block 0 also writes
// F2out[f] = (float) sum_b F2part[b][f] when F2part is given.
__global__ __launch_bounds__(256) void k_mf_collect(const float* __restrict__ part, int nsplit, int64_t ld,
                                                    const float* __restrict__ scale, float* __restrict__ D,
                                                    const double* __restrict__ F2part, int nF2, float* __restrict__ F2out) {
    __shared__ float tile[NF][64 + 1];
    const int64_t v0 = (int64_t)blockIdx.x * 64;
    // load: thread t handles elements t, t+256, t+512, t+768 of the contiguous [64][16] block
    for (int e = threadIdx.x; e < 64 * NF; e += 256) {
        const int64_t v = v0 + e / NF;
        const int f = e % NF;
        float acc = 0.f;
        if (v < ld)
            for (int s = 0; s < nsplit; ++s) acc += part[((int64_t)s * ld + v) * NF + f];
        tile[f][e / NF] = (v < ld && scale) ? acc * scale[v] : acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * NF; e += 256) {
        const int f = e / 64, vv = e % 64;
        const int64_t v = v0 + vv;
        if (v < ld) D[(int64_t)f * ld + v] = tile[f][vv];
    }
    if (F2part && blockIdx.x == 0 && threadIdx.x < NF) {
        double s = 0.0;
        for (int b = 0; b < nF2; ++b) s += F2part[(int64_t)b * NF + threadIdx.x];
        F2out[threadIdx.x] = (float)s;
    }
}

// X[f][v] = max(D0[f][v] * dinv[v], 1e-7) for real voxels of used frames, 0 elsewhere.
__global__ __launch_bounds__(256) void k_mf_init(float* __restrict__ X, const float* __restrict__ D0,
                                                 const float* __restrict__ dinv, int64_t nvox, int64_t ld, int nused) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)NF * ld) return;
    const int f = (int)(i / ld);
    const int64_t v = i % ld;
    float x = 0.f;
    if (f < nused && v < nvox) {
        x = D0[i] * dinv[v];
        x = x > 1e-7f ? x : 1e-7f;
    }
    X[i] = x;
}

// pen[f][v] = beta * sum_j L[v, j] x[f][j] (or log x), one thread per (row, frame), fixed order.
__global__ __launch_bounds__(256) void k_mf_penalty(const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                                                    const float* __restrict__ val, int64_t n, float beta, int logx,
                                                    const float* __restrict__ X, int64_t ld, float* __restrict__ pen,
                                                    const MfState* __restrict__ st) {
    if (st->all_done) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n * NF) return;
    const int f = (int)(i % NF);
    const int64_t r = i / NF;
    if (st->done[f]) return;
    const float* x = X + (int64_t)f * ld;
    float s = 0.f;  // same arithmetic as k_penalty_csr (sart_update.hip)
    for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
        const float xv = x[col[k]];
        s = fmaf(val[k], logx ? logf(xv) : xv, s);
    }
    pen[(int64_t)f * ld + r] = beta * s;
}

// Per-frame decision of sweep s (same rule as k_decide): conv_f = (G_f - F2_f) / G_f; a frame converges
// when s >= 2 and |conv_f - conv_prev_f| < tol; frames done earlier keep their conv_prev.
__global__ void k_mf_decide(MfState* __restrict__ st, const float* __restrict__ F2) {
    __shared__ int alld;
    const int f = threadIdx.x;
    if (st->all_done) return;
    const int s = st->sweep;
    if (f == 0) alld = 1;
    __syncthreads();
    if (f < NF) {
        const double F = (double)F2[f];
        int done = st->done[f];
        if (!isfinite(F)) {
            if (!done) {
                atomicOr(&st->flags, 1 << f);
                st->iters[f] = s;
                done = 1;
            }
        } else if (s >= 1) {
            const double conv = (st->G[f] - F) / st->G[f];
            const bool newly = !done && s >= 2 && fabs(conv - st->conv_prev[f]) < st->tol;
            if (newly) {
                st->status[f] = kSuccess;
                st->iters[f] = s;
            }
            if (!(done && !newly)) st->conv_prev[f] = conv;
            st->conv[f] = conv;
            done = done || newly;
        }
        st->done[f] = done;
        if (!done) atomicAnd(&alld, 0);
    }
    __syncthreads();
    if (f == 0) {
        st->all_done = (alld || s >= st->max_iter) ? 1 : 0;
        st->sweep = s + 1;
    }
}

// Update of the frames that are still running (after the decision of this sweep).
__global__ __launch_bounds__(256) void k_mf_update(float* __restrict__ X, const float* __restrict__ D,
                                                   const float* __restrict__ O, const float* __restrict__ pen,
                                                   float alpha, int logmode, int64_t nvox, int64_t ld,
                                                   const MfState* __restrict__ st) {
    if (st->all_done) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)NF * ld) return;
    const int f = (int)(i / ld);
    const int64_t v = i % ld;
    if (v >= nvox || st->done[f]) return;
    const float p = pen ? pen[i] : 0.f;
    if (logmode) {
        const float eps = 1e-7f;  // reference EPSILON_LOG_CUDA (sart_kernels.cu:17-19)
        float r = powf((O[i] + eps) / (D[i] + eps), alpha);
        if (pen) r *= expf(-p);
        X[i] = X[i] * r;
    } else {
        const float x = X[i] + D[i] - p;
        X[i] = x > 0.f ? x : 0.f;
    }
}

__global__ void k_mf_state_begin(MfState* __restrict__ st, const double* __restrict__ G, int nused, double tol,
                                 int max_iter) {
    const int f = threadIdx.x;
    if (f < NF) {
        st->G[f] = G[f];
        st->conv_prev[f] = 0.0;
        st->conv[f] = 0.0;
        st->done[f] = f < nused ? 0 : 1;
        st->status[f] = kMaxIterationsExceeded;
        st->iters[f] = max_iter;
    }
    if (f == 0) {
        st->sweep = 0;
        st->max_iter = max_iter;
        st->all_done = nused > 0 ? 0 : 1;
        st->flags = 0;
        st->tol = tol;
    }
}

static inline unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }

void launch_mf_prep(const double* g, int64_t nrows, int64_t nrows_pad, const double* norm, const float* ray_length,
                    float len_thres, float* ghat, float* arow, float* gpos, float* wo, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_prep, dim3(nb(nrows_pad * NF)), dim3(256), 0, stream, g, nrows, nrows_pad, norm,
                       ray_length, len_thres, ghat, arow, gpos, wo);
    check_launch("k_mf_prep");
}

int mf_weights_num_blocks(int64_t nrows_pad) { return (int)((nrows_pad + kWRows - 1) / kWRows); }

void launch_mf_weights(const float* Fs, int nsplit, int64_t nrows_pad, const float* ghat, const float* arow,
                       bool logmode, float* W, double* F2part, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_weights, dim3((unsigned)mf_weights_num_blocks(nrows_pad)), dim3(256), 0, stream, Fs,
                       nsplit, nrows_pad, ghat, arow, logmode ? 1 : 0, W, F2part);
    check_launch("k_mf_weights");
}

void launch_mf_collect(const float* part, int nsplit, int64_t ld, const float* scale, float* D, const double* F2part,
                       int nF2, float* F2out, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_collect, dim3((unsigned)((ld + 63) / 64)), dim3(256), 0, stream, part, nsplit, ld, scale,
                       D, F2part, nF2, F2out);
    check_launch("k_mf_collect");
}

void launch_mf_init(float* X, const float* D0, const float* dinv, int64_t nvox, int64_t ld, int nused,
                    hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_init, dim3(nb((int64_t)NF * ld)), dim3(256), 0, stream, X, D0, dinv, nvox, ld, nused);
    check_launch("k_mf_init");
}

void launch_mf_penalty(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t n, float beta, bool logx,
                       const float* X, int64_t ld, float* pen, const MfState* st, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_penalty, dim3(nb(n * NF)), dim3(256), 0, stream, row_ptr, col, val, n, beta,
                       logx ? 1 : 0, X, ld, pen, st);
    check_launch("k_mf_penalty");
}

void launch_mf_decide(MfState* st, const float* F2, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_decide, dim3(1), dim3(64), 0, stream, st, F2);
    check_launch("k_mf_decide");
}

void launch_mf_update(float* X, const float* D, const float* O, const float* pen, float alpha, bool logmode,
                      int64_t nvox, int64_t ld, const MfState* st, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_update, dim3(nb((int64_t)NF * ld)), dim3(256), 0, stream, X, D, O, pen, alpha,
                       logmode ? 1 : 0, nvox, ld, st);
    check_launch("k_mf_update");
}

void launch_mf_state_begin(MfState* st, const double* G, int nused, double tol, int max_iter, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_state_begin, dim3(1), dim3(64), 0, stream, st, G, nused, tol, max_iter);
    check_launch("k_mf_state_begin");
}

}  // namespace sart
