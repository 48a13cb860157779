// Two-pass projection kernels for gfx950: forward projection (row dot, A.x) with fused per-pixel
// epilogues and deterministic split-K back-projection (column accumulate, A^T.w).
//
// Reference behaviour being replaced:
//   * forward projection: cublasSgemv(OP_T) + cublasSdot to a host pointer
//     (reference sartsolver_cuda.cpp:188-189, 248-253) -> k_forward with the per-pixel SART weight,
//     ||f||^2 partials and the fitted image produced in the same pass (no second pass over f).
//   * back-projection: PropagateKernel / LogPropagateKernel / InitialGuessKernel with fp32 atomicAdd
//     (reference sart_kernels.cu:22-176) -> k_backproject writing per-split partial slabs that a
//     fixed-order second stage reduces, so results are bitwise reproducible run to run.
//   * ray density / ray length computed on the CPU in fp64 (reference sartsolver.cpp:38-56) ->
//     k_colsum_f64 / k_rowsum_f64 on the device with fp64 accumulation.
//
// All loads are 16 B per lane (float4); one wave instruction moves 1 KiB of a row.
#include "sart_common.hpp"

#include <stdexcept>
#include <string>

namespace sart {

void hip_call(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void check_launch(const char* what) {
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        throw std::runtime_error(std::string("HIP launch failed (") + what + "): " + hipGetErrorString(err));
    }
}

enum FwdEpilogue : int {
    kEpiPlain = 0,   // f only
    kEpiLinear = 1,  // w = a * (ghat - f)          (linear SART weight, reference sart_kernels.cu:79-81)
    kEpiLog = 2,     // w = a * f                   (fitted half of LogPropagateKernel, :134-146)
};

// ---------------------------------------------------------------------------------------------
// Forward projection: each workgroup owns RPB consecutive rows; 256 threads stride the columns
// with float4 loads. x is re-read from L2 once per RPB rows.
// ---------------------------------------------------------------------------------------------
template <int RPB, int EPI>
__global__ __launch_bounds__(256) void k_forward(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                 const float* __restrict__ x,
                                                 const float* __restrict__ ghat,
                                                 const float* __restrict__ arow,
                                                 float* __restrict__ out_f,
                                                 float* __restrict__ out_w,
                                                 double* __restrict__ Fpart,
                                                 const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    __shared__ float red[4][RPB];

    const int tid = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * RPB;
    const int64_t ld4 = ld >> 2;
    const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x);
    const float4* __restrict__ a4 = reinterpret_cast<const float4*>(A + row0 * ld);

    float acc[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) acc[r] = 0.f;

#pragma unroll 2
    for (int64_t c = tid; c < ld4; c += 256) {
        const float4 xv = x4[c];
        float4 av[RPB];
#pragma unroll
        for (int r = 0; r < RPB; ++r) av[r] = load_stream(a4 + r * ld4 + c);
#pragma unroll
        for (int r = 0; r < RPB; ++r) acc[r] += dot4(av[r], xv);
    }

    const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        const float s = wave_sum(acc[r]);
        if (lane == 0) red[wid][r] = s;
    }
    __syncthreads();

    if (tid < 64) {
        double f2 = 0.0;
        if (tid < RPB) {
            const int64_t row = row0 + tid;
            const float f = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
            if (row < nrows) {
                if (out_f) out_f[row] = f;
                if (EPI == kEpiLinear) out_w[row] = arow[row] * (ghat[row] - f);
                if (EPI == kEpiLog) out_w[row] = arow[row] * f;
                f2 = (double)f * (double)f;
            }
        }
        if (Fpart != nullptr) {
            f2 = wave_sum(f2);
            if (tid == 0) Fpart[blockIdx.x] = f2;
        }
    }
}

// fp64 row sums (ray length, reference sartsolver.cpp:49-56).
__global__ __launch_bounds__(256) void k_rowsum_f64(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                    double* __restrict__ out) {
    __shared__ double red[4];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    const int64_t ld4 = ld >> 2;
    const float4* __restrict__ a4 = reinterpret_cast<const float4*>(A + row * ld);
    double acc = 0.0;
    for (int64_t c = tid; c < ld4; c += 256) {
        const float4 a = a4[c];
        acc += ((double)a.x + (double)a.y) + ((double)a.z + (double)a.w);
    }
    acc = wave_sum(acc);
    if ((tid & 63) == 0) red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0 && row < nrows) out[row] = ((red[0] + red[1]) + red[2]) + red[3];
}

// ---------------------------------------------------------------------------------------------
// Back-projection, split-K over rows: block (cb, s) owns 1024 columns (256 lanes x float4) and the
// row range of split s. The per-row weight is wave-uniform, so it is fetched by scalar loads.
// partial[s][c] is written (not accumulated), the second stage k_reduce_partials sums the splits
// in a fixed order.
// ---------------------------------------------------------------------------------------------
template <int UNR>
__global__ __launch_bounds__(256) void k_backproject(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                     const float* __restrict__ w, int64_t rows_per_split,
                                                     float* __restrict__ partial,
                                                     const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    const int64_t c4 = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 column index
    const int64_t ld4 = ld >> 2;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows) r_end = nrows;
    if (c4 >= ld4) return;

    const float4* __restrict__ a4 = reinterpret_cast<const float4*>(A) + c4;
    float4 acc0 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc1 = acc0;

    int64_t r = r_begin;
    for (; r + UNR <= r_end; r += UNR) {
        float4 av[UNR];
        float wv[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) av[u] = load_stream(a4 + (r + u) * ld4);
#pragma unroll
        for (int u = 0; u < UNR; ++u) wv[u] = w[r + u];
#pragma unroll
        for (int u = 0; u < UNR; u += 2) {
            fma4(acc0, av[u], wv[u]);
            fma4(acc1, av[u + 1], wv[u + 1]);
        }
    }
    for (; r < r_end; ++r) fma4(acc0, load_stream(a4 + r * ld4), w[r]);

    acc0.x += acc1.x;
    acc0.y += acc1.y;
    acc0.z += acc1.z;
    acc0.w += acc1.w;
    reinterpret_cast<float4*>(partial + (int64_t)blockIdx.y * ld)[c4] = acc0;
}

// fp64 column sums (ray density, reference sartsolver.cpp:38-47), same split-K structure.
__global__ __launch_bounds__(256) void k_colsum_f64(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                    int64_t rows_per_split, double* __restrict__ partial) {
    const int64_t c4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t ld4 = ld >> 2;
    if (c4 >= ld4) return;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows) r_end = nrows;
    const float4* __restrict__ a4 = reinterpret_cast<const float4*>(A) + c4;
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int64_t r = r_begin; r < r_end; ++r) {
        const float4 a = a4[r * ld4];
        s0 += a.x;
        s1 += a.y;
        s2 += a.z;
        s3 += a.w;
    }
    double* out = partial + (int64_t)blockIdx.y * ld + c4 * 4;
    out[0] = s0;
    out[1] = s1;
    out[2] = s2;
    out[3] = s3;
}

// out[c] = scale[c] * sum_s partial[s][c]   (fixed summation order -> deterministic)
// scale == nullptr means 1. Optionally also writes the sum of Fpart[0:nF] (fp64) to *Fout as
// fp32, the value that is all-reduced with the correction vector (piggyback, one collective).
__global__ __launch_bounds__(256) void k_reduce_partials(const float* __restrict__ partial, int64_t ld, int nsplit,
                                                         const float* __restrict__ scale, float* __restrict__ out,
                                                         const double* __restrict__ Fpart, int64_t nF,
                                                         float* __restrict__ Fout,
                                                         const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    const int64_t c4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t ld4 = ld >> 2;
    if (c4 < ld4) {
        const float4* __restrict__ p4 = reinterpret_cast<const float4*>(partial) + c4;
        float4 s = p4[0];
        for (int k = 1; k < nsplit; ++k) {
            const float4 v = p4[(int64_t)k * ld4];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        if (scale != nullptr) {
            const float4 sc = reinterpret_cast<const float4*>(scale)[c4];
            s.x *= sc.x;
            s.y *= sc.y;
            s.z *= sc.z;
            s.w *= sc.w;
        }
        reinterpret_cast<float4*>(out)[c4] = s;
    }
    if (Fout != nullptr && blockIdx.x == 0) {
        __shared__ double red[4];
        double acc = 0.0;
        for (int64_t i = threadIdx.x; i < nF; i += 256) acc += Fpart[i];
        acc = wave_sum(acc);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) *Fout = (float)(((red[0] + red[1]) + red[2]) + red[3]);
    }
}

__global__ __launch_bounds__(256) void k_reduce_partials_f64(const double* __restrict__ partial, int64_t ld,
                                                             int nsplit, double* __restrict__ out) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= ld) return;
    double s = partial[c];
    for (int k = 1; k < nsplit; ++k) s += partial[(int64_t)k * ld + c];
    out[c] = s;
}

// ---------------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------------
template <int EPI>
static void launch_forward_epi(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                               const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                               const SartState* st, hipStream_t stream) {
    constexpr int RPB = 8;
    const int64_t nblk = (nrows_pad + RPB - 1) / RPB;
    hipLaunchKernelGGL((k_forward<RPB, EPI>), dim3((unsigned)nblk), dim3(256), 0, stream, A, ld, nrows, x, ghat, arow,
                       out_f, out_w, Fpart, st);
}

int64_t forward_num_blocks(int64_t nrows_pad) { return (nrows_pad + 7) / 8; }

void launch_forward(int epi, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                    const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                    const SartState* st, hipStream_t stream) {
    if (nrows_pad % 8 != 0) throw std::runtime_error("forward: padded row count must be a multiple of 8");
    if (ld % 64 != 0) throw std::runtime_error("forward: ld must be a multiple of 64");
    switch (epi) {
        case kEpiPlain:
            launch_forward_epi<kEpiPlain>(A, ld, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream);
            break;
        case kEpiLinear:
            launch_forward_epi<kEpiLinear>(A, ld, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream);
            break;
        case kEpiLog:
            launch_forward_epi<kEpiLog>(A, ld, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream);
            break;
        default:
            throw std::runtime_error("forward: unknown epilogue");
    }
    check_launch("k_forward");
}

void launch_rowsum_f64(const float* A, int64_t ld, int64_t nrows, double* out, hipStream_t stream) {
    if (nrows <= 0) return;
    hipLaunchKernelGGL(k_rowsum_f64, dim3((unsigned)nrows), dim3(256), 0, stream, A, ld, nrows, out);
    check_launch("k_rowsum_f64");
}

// Choose the number of row splits so that the grid has >= ~2048 workgroups (8 per CU on 256 CUs)
// while each split still streams >= 32 rows.
int backproject_num_splits(int64_t ld, int64_t nrows) {
    const int64_t ncb = (ld / 4 + 255) / 256;
    int64_t s = (2048 + ncb - 1) / ncb;
    const int64_t smax = (nrows + 31) / 32;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    if (s > 4096) s = 4096;
    return (int)s;
}

void launch_backproject(const float* A, int64_t ld, int64_t nrows, const float* w, int nsplit, float* partial,
                        const SartState* st, hipStream_t stream) {
    if (ld % 64 != 0) throw std::runtime_error("backproject: ld must be a multiple of 64");
    if (nsplit < 1) throw std::runtime_error("backproject: nsplit must be >= 1");
    const int64_t ncb = (ld / 4 + 255) / 256;
    const int64_t rps = (nrows + nsplit - 1) / nsplit;
    hipLaunchKernelGGL((k_backproject<8>), dim3((unsigned)ncb, (unsigned)nsplit), dim3(256), 0, stream, A, ld, nrows,
                       w, rps, partial, st);
    check_launch("k_backproject");
}

void launch_colsum_f64(const float* A, int64_t ld, int64_t nrows, int nsplit, double* partial, hipStream_t stream) {
    const int64_t ncb = (ld / 4 + 255) / 256;
    const int64_t rps = (nrows + nsplit - 1) / nsplit;
    hipLaunchKernelGGL(k_colsum_f64, dim3((unsigned)ncb, (unsigned)nsplit), dim3(256), 0, stream, A, ld, nrows, rps,
                       partial);
    check_launch("k_colsum_f64");
}

void launch_reduce_partials(const float* partial, int64_t ld, int nsplit, const float* scale, float* out,
                            const double* Fpart, int64_t nF, float* Fout, const SartState* st, hipStream_t stream) {
    const int64_t nblk = (ld / 4 + 255) / 256;
    hipLaunchKernelGGL(k_reduce_partials, dim3((unsigned)nblk), dim3(256), 0, stream, partial, ld, nsplit, scale, out,
                       Fpart, nF, Fout, st);
    check_launch("k_reduce_partials");
}

void launch_reduce_partials_f64(const double* partial, int64_t ld, int nsplit, double* out, hipStream_t stream) {
    const int64_t nblk = (ld + 255) / 256;
    hipLaunchKernelGGL(k_reduce_partials_f64, dim3((unsigned)nblk), dim3(256), 0, stream, partial, ld, nsplit, out);
    check_launch("k_reduce_partials_f64");
}

}  // namespace sart
