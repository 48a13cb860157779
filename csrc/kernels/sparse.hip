// Sparse RTM projections for gfx950 (the sparse COO datasets of the input schema, manual.pdf p.5-8, kept sparse on
// the device instead of expanded into a dense shard).
//
// Reference behaviour being replaced: the reference scatters a sparse COO RTM into its dense host shard
// (raytransfer.cpp:67-91) and then runs the dense kernels, so a few-MB no-reflection matrix costs the
// same HBM stream per iteration as a dense one (reference sartsolver_cuda.cpp:239-249). Here the shard stays
// sparse: CSR rows for the forward projection and CSC columns for the back-projection, both gathers with one
// writer per output, so there are no atomics and results are bitwise reproducible.
//
// Layout of the work: 32 lanes per row (column), 8 rows (columns) per 256-thread workgroup. Each lane sums every
// 32nd entry of its row in fp32 (the reference's precision), the 32 lane sums are combined by a fixed xor tree, so
// a row's sum depends only on its entries. The epilogues and the fp64 ||f||^2 partials (one per 8 rows) are those
// of the dense k_forward (projection.hip), so the engine's reduction, all-reduce, decision and update kernels are
// shared with the dense path.
#include "sart_common.hpp"
#include "launchers.hpp"

#include <stdexcept>

namespace sart {

namespace {

constexpr int kLanesPerRow = 32;
constexpr int kRowsPerBlock = 256 / kLanesPerRow;  // = 8, the dense forward's rows per Fpart block

__device__ __forceinline__ float sum32(float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, kLanesPerRow);
    return v;
}
__device__ __forceinline__ double sum32(double v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, kLanesPerRow);
    return v;
}

}  // namespace

template <int EPI>
__global__ __launch_bounds__(256) void k_csr_forward(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                     const float* __restrict__ val, int64_t nrows,
                                                     const float* __restrict__ x, const float* __restrict__ ghat,
                                                     const float* __restrict__ arow, float* __restrict__ out_f,
                                                     float* __restrict__ out_w, double* __restrict__ Fpart,
                                                     const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    const int sub = threadIdx.x & (kLanesPerRow - 1), r8 = threadIdx.x / kLanesPerRow;
    const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + r8;
    float acc = 0.f;
    if (row < nrows) {
        const int64_t k1 = rp[row + 1];
        for (int64_t k = rp[row] + sub; k < k1; k += kLanesPerRow) acc = __builtin_fmaf(val[k], x[col[k]], acc);
    }
    const float f = sum32(acc);
    double f2 = 0.0;
    if (sub == 0 && row < nrows) {
        if (out_f) out_f[row] = f;
        if (EPI == 1) out_w[row] = arow[row] * (ghat[row] - f);  // kEpiLinear
        if (EPI == 2) out_w[row] = arow[row] * f;                // kEpiLog
        f2 = (double)f * (double)f;
    }
    if (Fpart != nullptr) {
        __shared__ double red[kRowsPerBlock];
        if (sub == 0) red[r8] = f2;
        __syncthreads();
        if (threadIdx.x == 0) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < kRowsPerBlock; ++i) s += red[i];
            Fpart[blockIdx.x] = s;
        }
    }
}

__global__ __launch_bounds__(256) void k_csc_backproject(const int64_t* __restrict__ cp, const int32_t* __restrict__ row,
                                                         const float* __restrict__ val, int64_t ncols,
                                                         const float* __restrict__ w, float* __restrict__ out,
                                                         const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    const int sub = threadIdx.x & (kLanesPerRow - 1);
    const int64_t c = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kLanesPerRow;
    float acc = 0.f;
    if (c < ncols) {
        const int64_t k1 = cp[c + 1];
        for (int64_t k = cp[c] + sub; k < k1; k += kLanesPerRow) acc = __builtin_fmaf(val[k], w[row[k]], acc);
    }
    acc = sum32(acc);
    if (sub == 0 && c < ncols) out[c] = acc;
}

// fp64 sums of the entries of each row (CSR) or column (CSC): ray lengths / ray densities
__global__ __launch_bounds__(256) void k_sparse_sum_f64(const int64_t* __restrict__ ptr, const float* __restrict__ val,
                                                        int64_t n, double* __restrict__ out) {
    const int sub = threadIdx.x & (kLanesPerRow - 1);
    const int64_t i = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kLanesPerRow;
    double acc = 0.0;
    if (i < n) {
        const int64_t k1 = ptr[i + 1];
        for (int64_t k = ptr[i] + sub; k < k1; k += kLanesPerRow) acc += (double)val[k];
    }
    acc = sum32(acc);
    if (sub == 0 && i < n) out[i] = acc;
}

static unsigned blocks_for(int64_t n) { return (unsigned)((n + kRowsPerBlock - 1) / kRowsPerBlock); }

static void check_sparse(const SparseRtm& s, const char* what) {
    if (!s.row_ptr || !s.col_ptr || (s.nnz > 0 && (!s.col || !s.val || !s.row || !s.cval)))
        throw std::runtime_error(std::string(what) + ": incomplete sparse RTM (CSR and CSC arrays required)");
}

void launch_csr_forward(int epi, const SparseRtm& s, int64_t nrows, int64_t nrows_pad, const float* x,
                        const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                        const SartState* st, hipStream_t stream) {
    check_sparse(s, "csr_forward");
    if (nrows_pad % kRowsPerBlock != 0 || nrows_pad < nrows)
        throw std::runtime_error("csr_forward: padded row count must be a multiple of 8 covering the rows");
    // one Fpart entry per 8 padded rows, as forward_num_blocks(nrows_pad)
    const dim3 grid(blocks_for(nrows_pad));
    switch (epi) {
        case 0:
            hipLaunchKernelGGL(k_csr_forward<0>, grid, dim3(256), 0, stream, s.row_ptr, s.col, s.val, nrows, x, ghat,
                               arow, out_f, out_w, Fpart, st);
            break;
        case 1:
            hipLaunchKernelGGL(k_csr_forward<1>, grid, dim3(256), 0, stream, s.row_ptr, s.col, s.val, nrows, x, ghat,
                               arow, out_f, out_w, Fpart, st);
            break;
        case 2:
            hipLaunchKernelGGL(k_csr_forward<2>, grid, dim3(256), 0, stream, s.row_ptr, s.col, s.val, nrows, x, ghat,
                               arow, out_f, out_w, Fpart, st);
            break;
        default:
            throw std::runtime_error("csr_forward: unknown epilogue");
    }
    check_launch("k_csr_forward");
}

void launch_csc_backproject(const SparseRtm& s, int64_t nvoxel, const float* w, float* out, const SartState* st,
                            hipStream_t stream) {
    check_sparse(s, "csc_backproject");
    if (nvoxel <= 0) return;
    hipLaunchKernelGGL(k_csc_backproject, dim3(blocks_for(nvoxel)), dim3(256), 0, stream, s.col_ptr, s.row, s.cval,
                       nvoxel, w, out, st);
    check_launch("k_csc_backproject");
}

void launch_csr_rowsum_f64(const SparseRtm& s, int64_t nrows, double* out, hipStream_t stream) {
    check_sparse(s, "csr_rowsum");
    if (nrows <= 0) return;
    hipLaunchKernelGGL(k_sparse_sum_f64, dim3(blocks_for(nrows)), dim3(256), 0, stream, s.row_ptr, s.val, nrows, out);
    check_launch("k_sparse_sum_f64 (rows)");
}

void launch_csc_colsum_f64(const SparseRtm& s, int64_t nvoxel, double* out, hipStream_t stream) {
    check_sparse(s, "csc_colsum");
    if (nvoxel <= 0) return;
    hipLaunchKernelGGL(k_sparse_sum_f64, dim3(blocks_for(nvoxel)), dim3(256), 0, stream, s.col_ptr, s.cval, nvoxel,
                       out);
    check_launch("k_sparse_sum_f64 (columns)");
}

}  // namespace sart
