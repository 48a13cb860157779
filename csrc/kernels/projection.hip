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
// All loads are 16 B per lane (4 fp32 or 8 bf16 columns); one wave instruction moves 1 KiB of a row. The
// kernels are templated on the RTM storage type (RtmVec, sart_common.hpp): fp32, or bf16 storage with fp32
// products and sums (opt-in, half the bytes per sweep).
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
template <int RPB, int EPI, typename AT>
__global__ __launch_bounds__(256) void k_forward(const AT* __restrict__ A, int64_t ld, int64_t nrows,
                                                 const float* __restrict__ x,
                                                 const float* __restrict__ ghat,
                                                 const float* __restrict__ arow,
                                                 float* __restrict__ out_f,
                                                 float* __restrict__ out_w,
                                                 double* __restrict__ Fpart,
                                                 const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    __shared__ float red[4][RPB];

    using L = RtmVec<AT>;
    constexpr int NF4 = L::NF4;
    const int tid = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * RPB;
    const int64_t ldv = ld / (4 * NF4);  // 16-byte vectors per row
    const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x);
    const AT* __restrict__ a0 = A + row0 * ld;

    float acc[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) acc[r] = 0.f;

#pragma unroll 2
    for (int64_t c = tid; c < ldv; c += 256) {
        float4 xv[NF4];
#pragma unroll
        for (int j = 0; j < NF4; ++j) xv[j] = x4[c * NF4 + j];
        float4 av[RPB][NF4];
#pragma unroll
        for (int r = 0; r < RPB; ++r) L::load(a0 + r * ld, c, av[r]);
#pragma unroll
        for (int r = 0; r < RPB; ++r)
#pragma unroll
            for (int j = 0; j < NF4; ++j) acc[r] += dot4(av[r][j], xv[j]);
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
template <typename AT>
__global__ __launch_bounds__(256) void k_rowsum_f64(const AT* __restrict__ A, int64_t ld, int64_t nrows,
                                                    double* __restrict__ out) {
    using L = RtmVec<AT>;
    __shared__ double red[4];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    const int64_t ldv = ld / (4 * L::NF4);
    double acc = 0.0;
    for (int64_t c = tid; c < ldv; c += 256) {
        float4 av[L::NF4];
        L::load(A + row * ld, c, av);
#pragma unroll
        for (int j = 0; j < L::NF4; ++j) {
            const float4 a = av[j];
            acc += ((double)a.x + (double)a.y) + ((double)a.z + (double)a.w);
        }
    }
    acc = wave_sum(acc);
    if ((tid & 63) == 0) red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0 && row < nrows) out[row] = ((red[0] + red[1]) + red[2]) + red[3];
}

// ---------------------------------------------------------------------------------------------
// Back-projection, split-K over rows: block (cb, s) owns 1024 fp32 / 2048 bf16 columns (256 lanes x one
// 16-byte vector) and the
// row range of split s. The per-row weight is wave-uniform, so it is fetched by scalar loads.
// partial[s][c] is written (not accumulated), the second stage k_reduce_partials sums the splits
// in a fixed order.
// ---------------------------------------------------------------------------------------------
template <int UNR, typename AT>
__global__ __launch_bounds__(256) void k_backproject(const AT* __restrict__ A, int64_t ld, int64_t nrows,
                                                     const float* __restrict__ w, int64_t rows_per_split,
                                                     float* __restrict__ partial,
                                                     const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    using L = RtmVec<AT>;
    constexpr int NF4 = L::NF4;
    const int64_t cv = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 16-byte vector column index
    const int64_t ldv = ld / (4 * NF4);
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows) r_end = nrows;
    if (cv >= ldv) return;

    float4 acc0[NF4], acc1[NF4];
#pragma unroll
    for (int j = 0; j < NF4; ++j) acc0[j] = acc1[j] = make_float4(0.f, 0.f, 0.f, 0.f);

    int64_t r = r_begin;
    for (; r + UNR <= r_end; r += UNR) {
        float4 av[UNR][NF4];
        float wv[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) L::load(A + (r + u) * ld, cv, av[u]);
#pragma unroll
        for (int u = 0; u < UNR; ++u) wv[u] = w[r + u];
#pragma unroll
        for (int u = 0; u < UNR; u += 2) {
#pragma unroll
            for (int j = 0; j < NF4; ++j) {
                fma4(acc0[j], av[u][j], wv[u]);
                fma4(acc1[j], av[u + 1][j], wv[u + 1]);
            }
        }
    }
    for (; r < r_end; ++r) {
        float4 av[NF4];
        L::load(A + r * ld, cv, av);
#pragma unroll
        for (int j = 0; j < NF4; ++j) fma4(acc0[j], av[j], w[r]);
    }

    float4* out = reinterpret_cast<float4*>(partial + (int64_t)blockIdx.y * ld) + cv * NF4;
#pragma unroll
    for (int j = 0; j < NF4; ++j) {
        acc0[j].x += acc1[j].x;
        acc0[j].y += acc1[j].y;
        acc0[j].z += acc1[j].z;
        acc0[j].w += acc1[j].w;
        out[j] = acc0[j];
    }
}

// fp64 column sums (ray density, reference sartsolver.cpp:38-47), same split-K structure.
template <typename AT>
__global__ __launch_bounds__(256) void k_colsum_f64(const AT* __restrict__ A, int64_t ld, int64_t nrows,
                                                    int64_t rows_per_split, double* __restrict__ partial) {
    using L = RtmVec<AT>;
    constexpr int NF4 = L::NF4;
    const int64_t cv = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t ldv = ld / (4 * NF4);
    if (cv >= ldv) return;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows) r_end = nrows;
    double s[4 * NF4];
#pragma unroll
    for (int j = 0; j < 4 * NF4; ++j) s[j] = 0.0;
    for (int64_t r = r_begin; r < r_end; ++r) {
        float4 av[NF4];
        L::load(A + r * ld, cv, av);
#pragma unroll
        for (int j = 0; j < NF4; ++j) {
            s[4 * j + 0] += av[j].x;
            s[4 * j + 1] += av[j].y;
            s[4 * j + 2] += av[j].z;
            s[4 * j + 3] += av[j].w;
        }
    }
    double* out = partial + (int64_t)blockIdx.y * ld + cv * 4 * NF4;
#pragma unroll
    for (int j = 0; j < 4 * NF4; ++j) out[j] = s[j];
}

// fp32 -> bf16 with round-to-nearest-even (NaN stays NaN): bf16 storage of an RTM loaded or generated in
// fp32 blocks. n must be a multiple of 4.
__global__ __launch_bounds__(256) void k_f32_to_bf16(const float* __restrict__ src, int64_t n4,
                                                     bf16_t* __restrict__ dst) {
    auto cvt = [](float f) -> unsigned {
        const unsigned u = __float_as_uint(f);
        if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
        return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
    };
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 v = reinterpret_cast<const float4*>(src)[i];
        uint2 o;
        o.x = cvt(v.x) | (cvt(v.y) << 16);
        o.y = cvt(v.z) | (cvt(v.w) << 16);
        reinterpret_cast<uint2*>(dst)[i] = o;
    }
}

// out[c] = scale[c] * sum_s partial[s][c]   (fixed summation order -> deterministic)
// scale == nullptr means 1. Optionally also writes the sum of Fpart[0:nF] (fp64) to Fout[0] as
// fp32, the value that is all-reduced with the correction vector (piggyback, one collective), and the
// sweep's error word st->error to Fout[1] (so a protocol timeout on one rank reaches every rank's k_decide).
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
        if (threadIdx.x == 0) {
            Fout[0] = (float)(((red[0] + red[1]) + red[2]) + red[3]);
            Fout[1] = st != nullptr ? (float)st->error : 0.f;  // error word, all-reduced with ||A x||^2
        }
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
template <typename AT>
static constexpr int64_t cols_per_vec() {
    return 4 * RtmVec<AT>::NF4;
}

template <int EPI, typename AT>
static void launch_forward_epi(const AT* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                               const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                               const SartState* st, hipStream_t stream) {
    constexpr int RPB = 8;
    const int64_t nblk = (nrows_pad + RPB - 1) / RPB;
    hipLaunchKernelGGL((k_forward<RPB, EPI, AT>), dim3((unsigned)nblk), dim3(256), 0, stream, A, ld, nrows, x, ghat,
                       arow, out_f, out_w, Fpart, st);
}

int64_t forward_num_blocks(int64_t nrows_pad) { return (nrows_pad + 7) / 8; }

template <typename AT>
static void launch_forward_t(int epi, const AT* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
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

void launch_forward(int epi, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                    const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                    const SartState* st, hipStream_t stream) {
    launch_forward_t(epi, A, ld, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream);
}

void launch_forward(int epi, const bf16_t* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* x,
                    const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                    const SartState* st, hipStream_t stream) {
    launch_forward_t(epi, A, ld, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream);
}

template <typename AT>
static void launch_rowsum_t(const AT* A, int64_t ld, int64_t nrows, double* out, hipStream_t stream) {
    if (nrows <= 0) return;
    if (ld % 64 != 0) throw std::runtime_error("rowsum: ld must be a multiple of 64");
    hipLaunchKernelGGL((k_rowsum_f64<AT>), dim3((unsigned)nrows), dim3(256), 0, stream, A, ld, nrows, out);
    check_launch("k_rowsum_f64");
}

void launch_rowsum_f64(const float* A, int64_t ld, int64_t nrows, double* out, hipStream_t stream) {
    launch_rowsum_t(A, ld, nrows, out, stream);
}

void launch_rowsum_f64(const bf16_t* A, int64_t ld, int64_t nrows, double* out, hipStream_t stream) {
    launch_rowsum_t(A, ld, nrows, out, stream);
}

// Choose the number of row splits so that the grid has >= ~2048 workgroups (8 per CU on 256 CUs)
// while each split still streams >= 32 rows. elem_bytes: 4 (fp32) or 2 (bf16 storage, 8 columns per lane).
int backproject_num_splits(int64_t ld, int64_t nrows, int elem_bytes) {
    const int64_t cpv = elem_bytes == 2 ? 8 : 4;
    const int64_t ncb = (ld / cpv + 255) / 256;
    int64_t s = (2048 + ncb - 1) / ncb;
    const int64_t smax = (nrows + 31) / 32;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    if (s > 4096) s = 4096;
    return (int)s;
}

template <typename AT>
static void launch_backproject_t(const AT* A, int64_t ld, int64_t nrows, const float* w, int nsplit, float* partial,
                                 const SartState* st, hipStream_t stream) {
    if (ld % 64 != 0) throw std::runtime_error("backproject: ld must be a multiple of 64");
    if (nsplit < 1) throw std::runtime_error("backproject: nsplit must be >= 1");
    const int64_t ncb = (ld / cols_per_vec<AT>() + 255) / 256;
    const int64_t rps = (nrows + nsplit - 1) / nsplit;
    hipLaunchKernelGGL((k_backproject<8, AT>), dim3((unsigned)ncb, (unsigned)nsplit), dim3(256), 0, stream, A, ld,
                       nrows, w, rps, partial, st);
    check_launch("k_backproject");
}

void launch_backproject(const float* A, int64_t ld, int64_t nrows, const float* w, int nsplit, float* partial,
                        const SartState* st, hipStream_t stream) {
    launch_backproject_t(A, ld, nrows, w, nsplit, partial, st, stream);
}

void launch_backproject(const bf16_t* A, int64_t ld, int64_t nrows, const float* w, int nsplit, float* partial,
                        const SartState* st, hipStream_t stream) {
    launch_backproject_t(A, ld, nrows, w, nsplit, partial, st, stream);
}

template <typename AT>
static void launch_colsum_t(const AT* A, int64_t ld, int64_t nrows, int nsplit, double* partial,
                            hipStream_t stream) {
    if (ld % 64 != 0) throw std::runtime_error("colsum: ld must be a multiple of 64");
    const int64_t ncb = (ld / cols_per_vec<AT>() + 255) / 256;
    const int64_t rps = (nrows + nsplit - 1) / nsplit;
    hipLaunchKernelGGL((k_colsum_f64<AT>), dim3((unsigned)ncb, (unsigned)nsplit), dim3(256), 0, stream, A, ld, nrows,
                       rps, partial);
    check_launch("k_colsum_f64");
}

void launch_colsum_f64(const float* A, int64_t ld, int64_t nrows, int nsplit, double* partial, hipStream_t stream) {
    launch_colsum_t(A, ld, nrows, nsplit, partial, stream);
}

void launch_colsum_f64(const bf16_t* A, int64_t ld, int64_t nrows, int nsplit, double* partial, hipStream_t stream) {
    launch_colsum_t(A, ld, nrows, nsplit, partial, stream);
}

void launch_f32_to_bf16(const float* src, int64_t n, bf16_t* dst, hipStream_t stream) {
    if (n <= 0) return;
    if (n % 4 != 0) throw std::runtime_error("f32_to_bf16: n must be a multiple of 4");
    const int64_t n4 = n / 4;
    int64_t nblk = (n4 + 255) / 256;
    if (nblk > 8192) nblk = 8192;
    hipLaunchKernelGGL(k_f32_to_bf16, dim3((unsigned)nblk), dim3(256), 0, stream, src, n4, dst);
    check_launch("k_f32_to_bf16");
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
