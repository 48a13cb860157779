// Sparse RTM projections for gfx950 (the sparse COO datasets of the input schema, manual.pdf p.5-8, kept sparse on
// the device instead of expanded into a dense shard).
//
// Reference behaviour being replaced: the reference scatters a sparse COO RTM into its dense host shard
// (raytransfer.cpp:67-91) and then runs the dense kernels, so a few-MB no-reflection matrix costs the
// same HBM stream per iteration as a dense one (reference sartsolver_cuda.cpp:239-249). Here the shard stays
// sparse: CSR rows for the forward projection and CSC columns for the back-projection, both gathers with one
// writer per output, so there are no atomics and results are bitwise reproducible.
//
// Layout of the work: a group of L lanes (4 .. 32, a power of two: SparseRtm::lanes_rows / lanes_cols) per row
// (column), 256 / L rows per 256-thread workgroup. Each lane sums every L-th entry of its row in fp32 (the
// reference's precision), the L lane sums are combined by a fixed xor tree, so a row's sum depends only on its
// entries and L. Short rows (a ray crosses O(grid) voxels) take few lanes, so a wave serves several rows and the
// dependent loads (offsets -> indices -> the gathered vector) of many rows are in flight at once. The epilogues are
// those of the dense k_forward (projection.hip); the fp64 ||f||^2 partials are one per workgroup, summed in row
// order, so the engine's reduction, all-reduce, decision and update kernels are shared with the dense path.
#include "sart_common.hpp"
#include "launchers.hpp"

#include <cstdlib>
#include <stdexcept>
#include <string>

namespace sart {

namespace {

template <int L, typename T>
__device__ __forceinline__ T group_sum(T v) {
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, L);
    return v;
}

// sum over k = k0, k0 + L, ... < k1 of val[k] * v[idx[k]] in that order (fp32 fma chain), four entries' loads issued
// before their products: the index -> gather dependency of one entry then overlaps the loads of the next three
template <int L>
__device__ __forceinline__ float gather_dot(const int32_t* __restrict__ idx, const float* __restrict__ val,
                                            const float* __restrict__ v, int64_t k0, int64_t k1) {
    float acc = 0.f;
    int64_t k = k0;
    for (; k + 3 * L < k1; k += 4 * L) {
        const int32_t i0 = idx[k], i1 = idx[k + L], i2 = idx[k + 2 * L], i3 = idx[k + 3 * L];
        const float a0 = val[k], a1 = val[k + L], a2 = val[k + 2 * L], a3 = val[k + 3 * L];
        const float x0 = v[i0], x1 = v[i1], x2 = v[i2], x3 = v[i3];
        acc = __builtin_fmaf(a0, x0, acc);
        acc = __builtin_fmaf(a1, x1, acc);
        acc = __builtin_fmaf(a2, x2, acc);
        acc = __builtin_fmaf(a3, x3, acc);
    }
    for (; k < k1; k += L) acc = __builtin_fmaf(val[k], v[idx[k]], acc);
    return acc;
}

}  // namespace

template <int L, int EPI>
__global__ __launch_bounds__(256) void k_csr_forward(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                     const float* __restrict__ val, int64_t nrows,
                                                     const float* __restrict__ x, const float* __restrict__ ghat,
                                                     const float* __restrict__ arow, float* __restrict__ out_f,
                                                     float* __restrict__ out_w, double* __restrict__ Fpart,
                                                     const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    constexpr int RPB = 256 / L;
    const int sub = threadIdx.x & (L - 1), rl = threadIdx.x / L;
    const int64_t row = (int64_t)blockIdx.x * RPB + rl;
    const float acc = row < nrows ? gather_dot<L>(col, val, x, rp[row] + sub, rp[row + 1]) : 0.f;
    const float f = group_sum<L>(acc);
    double f2 = 0.0;
    if (sub == 0 && row < nrows) {
        if (out_f) out_f[row] = f;
        if (EPI == 1) out_w[row] = arow[row] * (ghat[row] - f);  // kEpiLinear
        if (EPI == 2) out_w[row] = arow[row] * f;                // kEpiLog
        f2 = (double)f * (double)f;
    }
    if (Fpart != nullptr) {
        __shared__ double red[RPB];
        if (sub == 0) red[rl] = f2;
        __syncthreads();
        if (threadIdx.x == 0) {
            double s = 0.0;
            for (int i = 0; i < RPB; ++i) s += red[i];  // row order
            Fpart[blockIdx.x] = s;
        }
    }
}

template <int L>
__global__ __launch_bounds__(256) void k_csc_backproject(const int64_t* __restrict__ cp, const int32_t* __restrict__ row,
                                                         const float* __restrict__ val, int64_t ncols,
                                                         const float* __restrict__ w, float* __restrict__ out,
                                                         const SartState* __restrict__ st) {
    if (st != nullptr && st->done) return;
    const int sub = threadIdx.x & (L - 1);
    const int64_t c = (int64_t)blockIdx.x * (256 / L) + threadIdx.x / L;
    float acc = c < ncols ? gather_dot<L>(row, val, w, cp[c] + sub, cp[c + 1]) : 0.f;
    acc = group_sum<L>(acc);
    if (sub == 0 && c < ncols) out[c] = acc;
}

// fp64 sums of the entries of each row (CSR) or column (CSC): ray lengths / ray densities
__global__ __launch_bounds__(256) void k_sparse_sum_f64(const int64_t* __restrict__ ptr, const float* __restrict__ val,
                                                        int64_t n, double* __restrict__ out) {
    const int sub = threadIdx.x & 31;
    const int64_t i = (int64_t)blockIdx.x * 8 + threadIdx.x / 32;
    double acc = 0.0;
    if (i < n) {
        const int64_t k1 = ptr[i + 1];
        for (int64_t k = ptr[i] + sub; k < k1; k += 32) acc += (double)val[k];
    }
    acc = group_sum<32>(acc);
    if (sub == 0 && i < n) out[i] = acc;
}

int sparse_lanes(double avg) {
    if (const char* e = std::getenv("SART_SPARSE_LANES"); e && *e) {
        const int l = std::atoi(e);
        if (l == 4 || l == 8 || l == 16 || l == 32) return l;
    }
    // the largest group with >= 4 entries per lane (one unrolled step of gather_dot), 4 .. 32 lanes: rows of ~48
    // entries run best on 8 lanes (27.3k it/s at 64k x 64k; 4 / 16 / 32 lanes: 24.1k / 25.8k / 21.1k;
    // profiles/sparse_r5_lanes.jsonl)
    int l = 4;
    while (l < 32 && 2 * l * 4 <= avg) l *= 2;
    return l;
}

static int lanes_or(int l, double avg) { return l ? l : sparse_lanes(avg); }

int64_t csr_forward_num_blocks(const SparseRtm& s, int64_t nrows_pad) {
    const int L = lanes_or(s.lanes_rows, nrows_pad ? (double)s.nnz / (double)nrows_pad : 0.0);
    const int64_t rpb = 256 / L;
    return (nrows_pad + rpb - 1) / rpb;
}

static void check_sparse(const SparseRtm& s, const char* what) {
    if (!s.row_ptr || !s.col_ptr || (s.nnz > 0 && (!s.col || !s.val || !s.row || !s.cval)))
        throw std::runtime_error(std::string(what) + ": incomplete sparse RTM (CSR and CSC arrays required)");
}

template <int L>
static void csr_forward_l(int epi, const SparseRtm& s, int64_t nrows, int64_t nrows_pad, const float* x,
                          const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                          const SartState* st, hipStream_t stream) {
    const dim3 grid((unsigned)((nrows_pad + 256 / L - 1) / (256 / L)));
    switch (epi) {
        case 0:
            hipLaunchKernelGGL((k_csr_forward<L, 0>), grid, dim3(256), 0, stream, s.row_ptr, s.col, s.val, nrows, x,
                               ghat, arow, out_f, out_w, Fpart, st);
            break;
        case 1:
            hipLaunchKernelGGL((k_csr_forward<L, 1>), grid, dim3(256), 0, stream, s.row_ptr, s.col, s.val, nrows, x,
                               ghat, arow, out_f, out_w, Fpart, st);
            break;
        case 2:
            hipLaunchKernelGGL((k_csr_forward<L, 2>), grid, dim3(256), 0, stream, s.row_ptr, s.col, s.val, nrows, x,
                               ghat, arow, out_f, out_w, Fpart, st);
            break;
        default:
            throw std::runtime_error("csr_forward: unknown epilogue");
    }
}

void launch_csr_forward(int epi, const SparseRtm& s, int64_t nrows, int64_t nrows_pad, const float* x,
                        const float* ghat, const float* arow, float* out_f, float* out_w, double* Fpart,
                        const SartState* st, hipStream_t stream) {
    check_sparse(s, "csr_forward");
    if (nrows_pad < nrows) throw std::runtime_error("csr_forward: padded row count below the row count");
    switch (lanes_or(s.lanes_rows, nrows_pad ? (double)s.nnz / (double)nrows_pad : 0.0)) {
        case 4: csr_forward_l<4>(epi, s, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream); break;
        case 8: csr_forward_l<8>(epi, s, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream); break;
        case 16: csr_forward_l<16>(epi, s, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream); break;
        default: csr_forward_l<32>(epi, s, nrows, nrows_pad, x, ghat, arow, out_f, out_w, Fpart, st, stream); break;
    }
    check_launch("k_csr_forward");
}

void launch_csc_backproject(const SparseRtm& s, int64_t nvoxel, const float* w, float* out, const SartState* st,
                            hipStream_t stream) {
    check_sparse(s, "csc_backproject");
    if (nvoxel <= 0) return;
    auto go = [&](auto lc) {
        constexpr int L = decltype(lc)::value;
        hipLaunchKernelGGL(k_csc_backproject<L>, dim3((unsigned)((nvoxel + 256 / L - 1) / (256 / L))), dim3(256), 0,
                           stream, s.col_ptr, s.row, s.cval, nvoxel, w, out, st);
    };
    switch (lanes_or(s.lanes_cols, (double)s.nnz / (double)nvoxel)) {
        case 4: go(std::integral_constant<int, 4>{}); break;
        case 8: go(std::integral_constant<int, 8>{}); break;
        case 16: go(std::integral_constant<int, 16>{}); break;
        default: go(std::integral_constant<int, 32>{}); break;
    }
    check_launch("k_csc_backproject");
}

void launch_csr_rowsum_f64(const SparseRtm& s, int64_t nrows, double* out, hipStream_t stream) {
    check_sparse(s, "csr_rowsum");
    if (nrows <= 0) return;
    hipLaunchKernelGGL(k_sparse_sum_f64, dim3((unsigned)((nrows + 7) / 8)), dim3(256), 0, stream, s.row_ptr, s.val,
                       nrows, out);
    check_launch("k_sparse_sum_f64 (rows)");
}

void launch_csc_colsum_f64(const SparseRtm& s, int64_t nvoxel, double* out, hipStream_t stream) {
    check_sparse(s, "csc_colsum");
    if (nvoxel <= 0) return;
    hipLaunchKernelGGL(k_sparse_sum_f64, dim3((unsigned)((nvoxel + 7) / 8)), dim3(256), 0, stream, s.col_ptr, s.cval,
                       nvoxel, out);
    check_launch("k_sparse_sum_f64 (columns)");
}

}  // namespace sart
