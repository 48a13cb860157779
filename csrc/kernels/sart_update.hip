// Per-frame preparation, Laplacian penalty (CSR SpMV), device-side convergence decision and the
// fused SART solution updates for gfx950.
//
// Reference counterparts:
//   * measurement normalisation / masks / initial-guess weights, done on the host per frame
//     (reference sartsolver_cuda.cpp:138-194) -> k_prep_rows, k_init_solution.
//   * GradPenaltyKernel / LogGradPenaltyKernel: COO with 64-bit div/mod and fp32 atomics
//     (reference sart_kernels.cu:179-202) -> k_penalty_csr: one thread per Laplacian row, fixed order,
//     written not accumulated (no memset, no atomics).
//   * UpdateSolutionKernel / UpdateLogSolutionKernel (reference sart_kernels.cu:205-224) ->
//     k_update_linear / k_update_log, gated by the device-side decision.
//   * host convergence test `|conv - conv_prev| < tol` after cublasSdot + MPI_Allreduce
//     (reference sartsolver_cuda.cpp:250-261) -> k_decide, a single-lane kernel on the stream, so
//     a frame solve never synchronises with the host.
#include "sart_common.hpp"

#include <math.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace sart {


// ghat = fp32(g / s); a = [ghat >= 0][len > tau_l] / len; gpos = max(ghat, 0); wo = a * ghat
// A non-finite pixel (NaN / Inf from a broken detector channel) is masked like a saturated one (g < 0):
// with a = 0 it contributes nothing; unmasked, 0 * NaN would turn every correction into NaN.
__global__ __launch_bounds__(256) void k_prep_rows(const double* __restrict__ g, int64_t nrows, int64_t nrows_pad,
                                                   double inv_s, const float* __restrict__ ray_length,
                                                   float len_thres, float* __restrict__ ghat, float* __restrict__ arow,
                                                   float* __restrict__ gpos, float* __restrict__ wo) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nrows_pad) return;
    float gh = 0.f, a = 0.f;
    if (i < nrows) {
        const double gv = g[i];
        gh = isfinite(gv) ? (float)(gv * inv_s) : -1.f;
        const float len = ray_length[i];
        const float inv_len = (len > len_thres) ? 1.f / len : 0.f;
        a = (gh >= 0.f) ? inv_len : 0.f;
    }
    ghat[i] = gh;
    arow[i] = a;
    if (gpos) gpos[i] = (gh > 0.f) ? gh : 0.f;
    if (wo) wo[i] = a * gh;
}

// x = max(src, 1e-7) on [0, n), 0 on the padding (reference sartsolver_cuda.cpp:180).
// src_f32 (device, already scaled) or src_f64 * scale (warm start x_prev / s).
__global__ __launch_bounds__(256) void k_init_solution(float* __restrict__ x, int64_t n, int64_t n_pad,
                                                       const float* __restrict__ src_f32,
                                                       const double* __restrict__ src_f64, double scale) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_pad) return;
    float v = 0.f;
    if (i < n) {
        v = src_f32 ? src_f32[i] : (float)(src_f64[i] * scale);
        if (v < kEpsLog) v = kEpsLog;
    }
    x[i] = v;
}

// Warm start from the solution still on the device (x normalised by the previous frame's norm a): x = fp32((x a) b)
// with b = 1 / the new norm, in double and in the order of the host path (de-normalise to the fp64 output, then
// normalise the start value), so the bits equal a host round trip; clamped like k_init_solution.
__global__ __launch_bounds__(256) void k_rescale_solution(float* __restrict__ x, int64_t n, int64_t n_pad, double a,
                                                          double b) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_pad) return;
    float v = 0.f;
    if (i < n) {
        v = (float)(((double)x[i] * a) * b);
        if (v < kEpsLog) v = kEpsLog;
    }
    x[i] = v;
}

// pen[i] = beta * sum_k val[k] * h(x[col[k]]), h = identity (linear) or log (logarithmic SART).
template <bool LOGX>
__global__ __launch_bounds__(256) void k_penalty_csr(const int64_t* __restrict__ row_ptr,
                                                     const int32_t* __restrict__ col,
                                                     const float* __restrict__ val, int64_t n, float beta,
                                                     const float* __restrict__ x, float* __restrict__ pen,
                                                     const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t k0 = row_ptr[i], k1 = row_ptr[i + 1];
    float acc = 0.f;
    for (int64_t k = k0; k < k1; ++k) {
        const float xv = x[col[k]];
        acc = fmaf(val[k], LOGX ? logf(xv) : xv, acc);
    }
    pen[i] = beta * acc;
}

// decide_next: sart_common.hpp (shared with the P2P all-reduce's fused update, p2p_allreduce.hip)

__global__ void k_decide(SartState* __restrict__ st, const float* __restrict__ Fslot) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    SartState s = *st;
    decide_next(s, Fslot);
    *st = s;
}

// k_decide and k_update_linear / k_update_log in ONE launch (one kernel boundary less per SART iteration): every
// workgroup evaluates the decision itself from the state before it, applies the update to its voxels when the
// frame continues, then takes a ticket; the last workgroup to arrive writes the new state (every other one has
// read the old state before its ticket) and re-arms the ticket for the next sweep.
template <bool LOGV>
__global__ __launch_bounds__(256) void k_decide_update(SartState* __restrict__ st, const float* __restrict__ Fslot,
                                                       float* __restrict__ x, const float* __restrict__ d,
                                                       const float* __restrict__ O, const float* __restrict__ pen,
                                                       float alpha, int64_t n, unsigned* __restrict__ xcnt,
                                                       float* __restrict__ xprev, unsigned* __restrict__ ticket) {
    __shared__ SartState s_next;
    __shared__ int s_apply;
    if (threadIdx.x == 0) {
        SartState s = *st;
        decide_next(s, Fslot);
        s_next = s;
        s_apply = !s.done;
    }
    if (xcnt && blockIdx.x == 0 && threadIdx.x < 16) xcnt[threadIdx.x] = 0u;  // see k_update_linear
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s_apply && i < n) {
        const float x0 = x[i];
        if (xprev) xprev[i] = x0;
        if constexpr (LOGV) {
            float r = powf((O[i] + kEpsLog) / (d[i] + kEpsLog), alpha);
            if (pen) r *= expf(-pen[i]);
            x[i] = x0 * r;
        } else {
            float v = x0 + d[i];
            if (pen) v -= pen[i];
            x[i] = (v > 0.f) ? v : 0.f;
        }
    }
    if (threadIdx.x == 0) {
        const unsigned t = atomicAdd(ticket, 1u);  // after this workgroup's read of *st (its value is consumed above)
        if (t == gridDim.x - 1) {
            *st = s_next;
            *ticket = 0u;
        }
    }
}

// One rank (nothing to all-reduce between the sweep and the update): k_reduce_partials and k_decide_update in ONE
// launch, so a SART iteration is the sweep plus this kernel. Every workgroup sums the sweep's Fpart[0:nF] itself in
// k_reduce_partials' order (nF is the sweep's grid, a few hundred doubles: L2 hits), evaluates the decision, sums
// its voxels' partial rows in k_reduce_partials' order and applies k_decide_update's update. Contraction is off so
// the correction is rounded before it is added, as when it went through memory: x is bitwise the three-kernel x.
template <int VEC>
__device__ __forceinline__ void load_v(const float* __restrict__ p, float (&v)[VEC]) {
    if constexpr (VEC == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x, v[1] = t.y, v[2] = t.z, v[3] = t.w;
    } else {
#pragma unroll
        for (int c = 0; c < VEC; ++c) v[c] = p[c];
    }
}

// VEC consecutive voxels per thread (4: float4 accesses; every array is ld long, ld % 64 == 0, stores guarded by n).
// Fslot != nullptr: k_decide_update's inputs (d = partial with nsplit 1 and no scale, Fslot = the all-reduced
// {||A x||^2, error word}), for N > 1 where the reduction happened before the all-reduce.
template <bool LOGV, int VEC>
__global__ __launch_bounds__(256) void k_reduce_decide_update(SartState* __restrict__ st,
                                                              const float* __restrict__ partial, int64_t ld,
                                                              int nsplit, const float* __restrict__ scale,
                                                              const double* __restrict__ Fpart, int64_t nF,
                                                              float* __restrict__ x, const float* __restrict__ O,
                                                              const float* __restrict__ pen, float alpha, int64_t n,
                                                              unsigned* __restrict__ xcnt, float* __restrict__ xprev,
                                                              unsigned* __restrict__ ticket,
                                                              const float* __restrict__ Fslot) {
#pragma clang fp contract(off)
    __shared__ double red[4];
    __shared__ SartState s_next;
    __shared__ int s_apply;
    // this thread's voxel operands first (independent of the decision; stale but finite once the frame is done),
    // so their latency overlaps the Fpart reduction
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC;
    const bool mine = i0 < n;
    float d[VEC], x0[VEC], o[VEC], pn[VEC], t[VEC];
    if (mine) {
        load_v<VEC>(partial + i0, d);
        for (int k = 1; k < nsplit; ++k) {
            load_v<VEC>(partial + (int64_t)k * ld + i0, t);
#pragma unroll
            for (int c = 0; c < VEC; ++c) d[c] += t[c];
        }
        if (scale != nullptr) {
            load_v<VEC>(scale + i0, t);
#pragma unroll
            for (int c = 0; c < VEC; ++c) d[c] *= t[c];
        }
        load_v<VEC>(x + i0, x0);
        if constexpr (LOGV) load_v<VEC>(O + i0, o);
        if (pen) load_v<VEC>(pen + i0, pn);
    }
    if (Fslot == nullptr) {  // uniform: ||A x||^2 from the sweep partials, the error word from the state
        double acc = 0.0;
        for (int64_t i = threadIdx.x; i < nF; i += 256) acc += Fpart[i];
        acc = wave_sum(acc);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    }
    if (xcnt && blockIdx.x == 0 && threadIdx.x < 16) xcnt[threadIdx.x] = 0u;  // see k_update_linear
    __syncthreads();
    if (threadIdx.x == 0) {
        SartState s = *st;
        float F[2];
        if (Fslot != nullptr) {  // all-reduced {||A x||^2, error word} (k_decide_update's input)
            F[0] = Fslot[0];
            F[1] = Fslot[1];
        } else {
            F[0] = (float)(((red[0] + red[1]) + red[2]) + red[3]);
            F[1] = (float)s.error;
        }
        decide_next(s, F);
        s_next = s;
        s_apply = !s.done;
    }
    __syncthreads();
    if (s_apply && mine) {
#pragma unroll
        for (int c = 0; c < VEC; ++c) t[c] = sart_update_voxel<LOGV>(x0[c], d[c], LOGV ? o[c] : 0.f, pen, pen ? pn[c] : 0.f, alpha);
        if (VEC == 4 && i0 + 4 <= n) {
            if (xprev) *reinterpret_cast<float4*>(xprev + i0) = make_float4(x0[0], x0[1], x0[2], x0[3]);
            *reinterpret_cast<float4*>(x + i0) = make_float4(t[0], t[1], t[2], t[3]);
        } else {
            for (int c = 0; c < VEC && i0 + c < n; ++c) {
                if (xprev) xprev[i0 + c] = x0[c];
                x[i0 + c] = t[c];
            }
        }
    }
    if (threadIdx.x == 0) {
        const unsigned tk = atomicAdd(ticket, 1u);  // after this workgroup's read of *st
        if (tk == gridDim.x - 1) {
            *st = s_next;
            *ticket = 0u;
        }
    }
}

// x = max(x + d - pen, 0)
// xcnt (optional): the per-XCD ticket counters of the next fused sweep (variant 6), zeroed here so the
// sweep loop needs no separate memset launch per iteration (the sweep that used them has completed).
// xprev (optional): receives the iterate before the update (the rollback point of the NaN/Inf guard);
// one extra vector store per voxel, against a full pass over the shard per sweep.
__global__ __launch_bounds__(256) void k_update_linear(float* __restrict__ x, const float* __restrict__ d,
                                                       const float* __restrict__ pen, int64_t n,
                                                       const SartState* __restrict__ st, unsigned* __restrict__ xcnt,
                                                       float* __restrict__ xprev) {
    if (xcnt && blockIdx.x == 0 && threadIdx.x < 16) xcnt[threadIdx.x] = 0u;
    if (st->done) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x0 = x[i];
    if (xprev) xprev[i] = x0;
    float v = x0 + d[i];
    if (pen) v -= pen[i];
    x[i] = (v > 0.f) ? v : 0.f;
}

// x *= ((O + eps) / (Fv + eps))^alpha * exp(-pen)
__global__ __launch_bounds__(256) void k_update_log(float* __restrict__ x, const float* __restrict__ O,
                                                    const float* __restrict__ Fv, const float* __restrict__ pen,
                                                    float alpha, int64_t n, const SartState* __restrict__ st,
                                                    unsigned* __restrict__ xcnt, float* __restrict__ xprev) {
    if (xcnt && blockIdx.x == 0 && threadIdx.x < 16) xcnt[threadIdx.x] = 0u;  // see k_update_linear
    if (st->done) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float r = powf((O[i] + kEpsLog) / (Fv[i] + kEpsLog), alpha);
    if (pen) r *= expf(-pen[i]);
    const float x0 = x[i];
    if (xprev) xprev[i] = x0;
    x[i] = x0 * r;
}

// Device-side state initialisation for a new frame (keeps the epoch counter monotonic).
__global__ void k_state_begin(SartState* __restrict__ st, double G, double tol, int max_iter) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    st->G = G;
    st->conv_prev = 0.0;
    st->conv_last = 0.0;
    st->F_last = 0.0;
    st->sweep = 0;
    st->done = 0;
    st->status = kRunning;
    st->iterations = 0;
    st->max_iter = max_iter;
    st->error = 0;
    st->flags = 0;
    st->tol = tol;
    if (st->epoch <= 0) st->epoch = 1;
}

// Per-voxel scales from the global fp64 ray density, with the reference's fp32 semantics: the density is
// converted to fp32 first and compared with the fp32 threshold (reference sartsolver_cuda.cpp:118-124,
// sart_kernels.cu:82,86): dinv = [rho > t] / rho (cold start), dscale = [rho > t] alpha / rho (linear
// correction), dmask = [rho > t] (log back-projections). Padding voxels get zeros.
__global__ void k_density_scales(const double* __restrict__ rho, int64_t n, int64_t n_pad, float thres, float alpha,
                                 float* __restrict__ dinv, float* __restrict__ dscale, float* __restrict__ dmask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    const float r = i < n ? (float)rho[i] : 0.f;
    const bool valid = i < n && r > thres;
    dinv[i] = valid ? 1.0f / r : 0.f;
    dscale[i] = valid ? alpha / r : 0.f;
    dmask[i] = valid ? 1.f : 0.f;
}

__global__ void k_f64_to_f32(const double* __restrict__ src, float* __restrict__ dst, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = (float)src[i];
}

// Column-shard sweep (Engine with EngineConfig::column_shard): after the all-reduce of the partial forward
// projections, every rank holds the complete f and forms the SART weight of every pixel, exactly as the
// epilogue of k_forward does for a row shard (projection.hip): w = a (ghat - f) | a f, and the fp64 sum of
// f^2 per block (fixed thread order -> deterministic and identical on all ranks).
__global__ __launch_bounds__(256) void k_weights(int logmode, const float* __restrict__ f,
                                                 const float* __restrict__ ghat, const float* __restrict__ arow,
                                                 int64_t nrows, int64_t nrows_pad, float* __restrict__ w,
                                                 double* __restrict__ Fpart, const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    __shared__ double red[4];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double f2 = 0.0;
    if (i < nrows_pad) {
        float wv = 0.f;
        if (i < nrows) {
            const float fv = f[i];
            wv = logmode ? arow[i] * fv : arow[i] * (ghat[i] - fv);
            f2 = (double)fv * (double)fv;
        }
        w[i] = wv;
    }
    f2 = wave_sum(f2);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = f2;
    __syncthreads();
    if (threadIdx.x == 0) Fpart[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(256) void k_copy_slice(const float* __restrict__ src, int64_t n, float* __restrict__ dst,
                                                    int64_t offset) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[offset + i] = src[i];
}

static inline unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }

int weights_num_blocks(int64_t nrows_pad) { return (int)nb(nrows_pad); }

void launch_weights(bool logmode, const float* f, const float* ghat, const float* arow, int64_t nrows,
                    int64_t nrows_pad, float* w, double* Fpart, const SartState* st, hipStream_t stream) {
    hipLaunchKernelGGL(k_weights, dim3(nb(nrows_pad)), dim3(256), 0, stream, logmode ? 1 : 0, f, ghat, arow, nrows,
                       nrows_pad, w, Fpart, st);
    check_launch("k_weights");
}

void launch_copy_slice(const float* src, int64_t n, float* dst, int64_t offset, hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_copy_slice, dim3(nb(n)), dim3(256), 0, stream, src, n, dst, offset);
    check_launch("k_copy_slice");
}

void launch_density_scales(const double* rho, int64_t n, int64_t n_pad, float thres, float alpha, float* dinv,
                           float* dscale, float* dmask, hipStream_t stream) {
    hipLaunchKernelGGL(k_density_scales, dim3(nb(n_pad)), dim3(256), 0, stream, rho, n, n_pad, thres, alpha, dinv,
                       dscale, dmask);
    check_launch("k_density_scales");
}

void launch_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_f64_to_f32, dim3(nb(n)), dim3(256), 0, stream, src, dst, n);
    check_launch("k_f64_to_f32");
}

void launch_prep_rows(const double* g, int64_t nrows, int64_t nrows_pad, double inv_s, const float* ray_length,
                      float len_thres, float* ghat, float* arow, float* gpos, float* wo, hipStream_t stream) {
    hipLaunchKernelGGL(k_prep_rows, dim3(nb(nrows_pad)), dim3(256), 0, stream, g, nrows, nrows_pad, inv_s, ray_length,
                       len_thres, ghat, arow, gpos, wo);
    check_launch("k_prep_rows");
}

void launch_init_solution(float* x, int64_t n, int64_t n_pad, const float* src_f32, const double* src_f64,
                          double scale, hipStream_t stream) {
    hipLaunchKernelGGL(k_init_solution, dim3(nb(n_pad)), dim3(256), 0, stream, x, n, n_pad, src_f32, src_f64, scale);
    check_launch("k_init_solution");
}

void launch_rescale_solution(float* x, int64_t n, int64_t n_pad, double a, double b, hipStream_t stream) {
    hipLaunchKernelGGL(k_rescale_solution, dim3(nb(n_pad)), dim3(256), 0, stream, x, n, n_pad, a, b);
    check_launch("k_rescale_solution");
}

void launch_penalty(bool logx, const int64_t* row_ptr, const int32_t* col, const float* val, int64_t n, float beta,
                    const float* x, float* pen, const SartState* st, hipStream_t stream) {
    if (logx)
        hipLaunchKernelGGL(k_penalty_csr<true>, dim3(nb(n)), dim3(256), 0, stream, row_ptr, col, val, n, beta, x, pen,
                           st);
    else
        hipLaunchKernelGGL(k_penalty_csr<false>, dim3(nb(n)), dim3(256), 0, stream, row_ptr, col, val, n, beta, x, pen,
                           st);
    check_launch("k_penalty_csr");
}

// SART_TAIL_VEC=1: one voxel per thread in the decide / update kernels (A/B); default 4 (float4 accesses, a
// quarter of the workgroups: 5.7 instead of 7.3 us per iteration at 65536 voxels)
int tail_vec() {
    static const int vec = [] {
        const char* e = std::getenv("SART_TAIL_VEC");
        return (e && *e && std::atoi(e) == 1) ? 1 : 4;
    }();
    return vec;
}

void launch_decide(SartState* st, const float* Fslot, hipStream_t stream) {
    hipLaunchKernelGGL(k_decide, dim3(1), dim3(64), 0, stream, st, Fslot);
    check_launch("k_decide");
}

void launch_decide_update(bool logmode, SartState* st, const float* Fslot, float* x, const float* d, const float* O,
                          const float* pen, float alpha, int64_t n, unsigned* xcnt, float* xprev, unsigned* ticket,
                          hipStream_t stream) {
    if (tail_vec() == 4) {  // the float4 tail kernel on k_decide_update's inputs (bitwise the same x and state)
        const unsigned b4 = (unsigned)std::max<int64_t>(1, (n + 1023) / 1024);
        if (logmode)
            hipLaunchKernelGGL((k_reduce_decide_update<true, 4>), dim3(b4), dim3(256), 0, stream, st, d, (int64_t)0, 1,
                               nullptr, nullptr, (int64_t)0, x, O, pen, alpha, n, xcnt, xprev, ticket, Fslot);
        else
            hipLaunchKernelGGL((k_reduce_decide_update<false, 4>), dim3(b4), dim3(256), 0, stream, st, d, (int64_t)0,
                               1, nullptr, nullptr, (int64_t)0, x, O, pen, alpha, n, xcnt, xprev, ticket, Fslot);
        check_launch("k_reduce_decide_update (decide_update)");
        return;
    }
    const unsigned blocks = nb(n > 0 ? n : 1);
    if (logmode)
        hipLaunchKernelGGL(k_decide_update<true>, dim3(blocks), dim3(256), 0, stream, st, Fslot, x, d, O, pen, alpha, n,
                           xcnt, xprev, ticket);
    else
        hipLaunchKernelGGL(k_decide_update<false>, dim3(blocks), dim3(256), 0, stream, st, Fslot, x, d, O, pen, alpha,
                           n, xcnt, xprev, ticket);
    check_launch("k_decide_update");
}

void launch_reduce_decide_update(bool logmode, SartState* st, const float* partial, int64_t ld, int nsplit,
                                 const float* scale, const double* Fpart, int64_t nF, float* x, const float* O,
                                 const float* pen, float alpha, int64_t n, unsigned* xcnt, float* xprev,
                                 unsigned* ticket, hipStream_t stream) {
    if (n > ld || nsplit < 1 || nF < 0)
        throw std::runtime_error("launch_reduce_decide_update: bad arguments (n > ld, nsplit < 1 or nF < 0)");
    const int vec = tail_vec();
    const unsigned blocks = (unsigned)std::max<int64_t>(1, (n + 256 * vec - 1) / (256 * vec));
#define SART_RDU(L, V)                                                                                                 \
    hipLaunchKernelGGL((k_reduce_decide_update<L, V>), dim3(blocks), dim3(256), 0, stream, st, partial, ld, nsplit,   \
                       scale, Fpart, nF, x, O, pen, alpha, n, xcnt, xprev, ticket, nullptr)
    if (vec == 4) {
        if (logmode) SART_RDU(true, 4); else SART_RDU(false, 4);
    } else {
        if (logmode) SART_RDU(true, 1); else SART_RDU(false, 1);
    }
#undef SART_RDU
    check_launch("k_reduce_decide_update");
}

void launch_update_linear(float* x, const float* d, const float* pen, int64_t n, const SartState* st,
                          hipStream_t stream, unsigned* xcnt, float* xprev) {
    hipLaunchKernelGGL(k_update_linear, dim3(nb(n)), dim3(256), 0, stream, x, d, pen, n, st, xcnt, xprev);
    check_launch("k_update_linear");
}

void launch_update_log(float* x, const float* O, const float* Fv, const float* pen, float alpha, int64_t n,
                       const SartState* st, hipStream_t stream, unsigned* xcnt, float* xprev) {
    hipLaunchKernelGGL(k_update_log, dim3(nb(n)), dim3(256), 0, stream, x, O, Fv, pen, alpha, n, st, xcnt, xprev);
    check_launch("k_update_log");
}

void launch_state_begin(SartState* st, double G, double tol, int max_iter, hipStream_t stream) {
    hipLaunchKernelGGL(k_state_begin, dim3(1), dim3(64), 0, stream, st, G, tol, max_iter);
    check_launch("k_state_begin");
}

}  // namespace sart
