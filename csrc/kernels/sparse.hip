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

static void check_sparse(const SparseRtm& s, const char* what) {
    if (!s.row_ptr || !s.col_ptr || (s.nnz > 0 && (!s.col || !s.val || !s.row || !s.cval)))
        throw std::runtime_error(std::string(what) + ": incomplete sparse RTM (CSR and CSC arrays required)");
}

// ------------------------------------------------------------------------------------------- multi-frame (SpMM)
// The multi-frame engine's projections of a sparse shard (MultiFrameEngine sparse mode): one wave per row
// (column), the frames of one plane across the lanes (PW < 64: 64 / PW entries of the row in flight per wave, combined
// by a fixed xor tree), so each entry's operand row (PW consecutive fp32 of the voxel-major copy of X, or of W) is one
// coalesced load. fp32 fma chains in entry order per lane. A batch of nf > PW frames runs as nf / PW planes of PW
// frames (grid.y): a launch then gathers from the working set of one plane (the interleaved [n][128] rows of a
// 128-frame batch ran at 83.1k frame-it/s, two 64-frame planes at 183k; mf_sparse_plane_width).

int mf_sparse_plane_width(int nf) {
    int pw = 64;
    if (const char* e = std::getenv("SART_MF_SPARSE_PW"); e && *e) pw = std::atoi(e);
    if (pw != 16 && pw != 32 && pw != 64) throw std::runtime_error("SART_MF_SPARSE_PW must be 16, 32 or 64");
    return nf < pw ? nf : pw;
}

// The back-projection reads W in its slot layout only for one plane of <= 32 frames: there the 16 lanes of each quarter
// wave (one pass of the address path) still touch a single 128-B line. At 64 frames the slot order spreads them over
// the whole 256-B row, twice the lines per gather (113.5k against 183.5k frame-it/s per 64-frame plane,
// profiles/sparse_r5_plane_width.txt), so W is re-laid in frame order first (launch_mf_w_planes).
bool mf_sparse_needs_w_planes(int nf, int pw) { return pw < nf || pw > 32; }

static void check_pw(int nf, int pw, const char* what) {
    if ((pw != 16 && pw != 32 && pw != 64) || pw > nf || nf % pw != 0)
        throw std::runtime_error(std::string(what) + ": plane width must be 16, 32 or 64 and divide nf");
}

// W's back-projection layout [rows][16][nf / 16] (multiframe_glue.hip::mf_bp_slot)
__device__ __forceinline__ int mf_bp_slot_s(int f, int nf) { return (f & 15) * (nf >> 4) + (f >> 4); }

// X [nf][ld] (frame-major) -> Xt [nf / pw][ld][pw] (voxel-major planes of pw frames), 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void k_mf_transpose_x(const float* __restrict__ X, int64_t ld, int nf, int pw,
                                                        float* __restrict__ Xt, const int* __restrict__ skip) {
    if (skip && *skip) return;
    __shared__ float t[64][65];
    const int64_t v0 = (int64_t)blockIdx.x * 64;
    const int f0 = blockIdx.y * 64;
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int ff = i >> 6, vv = i & 63;
        if (f0 + ff < nf) t[ff][vv] = X[(int64_t)(f0 + ff) * ld + v0 + vv];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int vv = i >> 6, ff = i & 63, f = f0 + ff;
        if (f < nf) Xt[((int64_t)(f / pw) * ld + v0 + vv) * pw + f % pw] = t[ff][vv];
    }
}

// W [rows][nf] in the back-projection slot layout -> Wt [nf / pw][rows][pw] in frame order
__global__ __launch_bounds__(256) void k_mf_w_planes(const float* __restrict__ W, int64_t rows, int nf, int pw,
                                                     float* __restrict__ Wt, const int* __restrict__ skip) {
    if (skip && *skip) return;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (plane, row, frame) in Wt order
    if (e >= rows * nf) return;
    const int64_t p = (e / pw) % rows;
    const int f = (int)(e % pw) + pw * (int)(e / (rows * pw));
    Wt[e] = W[p * nf + mf_bp_slot_s(f, nf)];
}

// PW frames per plane (16, 32, 64); SLOT: W in the slot layout of a PW-frame batch (a one-plane back-projection);
// plane blockIdx.y: Y + blockIdx.y * yplane, outputs at frame offset PW blockIdx.y of rows of nfs frames, times
// oscale[i] when given (the back-projection's voxel scales: the sums go straight into the engine's corrections)
template <int PW, bool SLOT>
__global__ __launch_bounds__(256) void k_mf_sparse_spmm(const int64_t* __restrict__ ptr, const int32_t* __restrict__ idx,
                                                        const float* __restrict__ val, int64_t n_valid, int64_t i0,
                                                        int64_t i1, const float* __restrict__ Y, int64_t yplane,
                                                        float* __restrict__ out, const float* __restrict__ oscale,
                                                        int nfs, const int* __restrict__ skip) {
    if (skip && *skip) return;
    constexpr int G = 64 / PW;  // entries in flight per wave
    // eight fp32 chains per row and frame (G groups x CH chains per lane, entries dealt round robin): one chain over
    // a dense row of thousands of entries would exceed an fp32 evaluation's error (tests/test_gpu_sparse.py)
    constexpr int CH = G >= 8 ? 1 : 8 / G;
    const int lane = threadIdx.x & 63, grp = lane / PW, fl = lane % PW;
    const int64_t i = i0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // row (forward) / column (back-projection)
    if (i >= i1) return;
    Y += (int64_t)blockIdx.y * yplane + (SLOT ? mf_bp_slot_s(fl, PW) : fl);
    float acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = 0.f;
    if (i < n_valid) {
        const int64_t k1 = ptr[i + 1];
        int64_t k = ptr[i] + grp;
        for (; k + (CH - 1) * G < k1; k += CH * G)
#pragma unroll
            for (int c = 0; c < CH; ++c) acc[c] = __builtin_fmaf(val[k + c * G], Y[(int64_t)idx[k + c * G] * PW], acc[c]);
        for (int c = 0; k < k1; k += G, ++c) {  // tail: chains 0, 1, ... in turn
            const float y = Y[(int64_t)idx[k] * PW], a = val[k];
#pragma unroll
            for (int cc = 0; cc < CH; ++cc)
                if (cc == c) acc[cc] = __builtin_fmaf(a, y, acc[cc]);
        }
    }
    // chains pairwise, then the groups by a fixed xor tree
#pragma unroll
    for (int w = 1; w < CH; w <<= 1)
#pragma unroll
        for (int c = 0; c + w < CH; c += 2 * w) acc[c] += acc[c + w];
    float tot = acc[0];
#pragma unroll
    for (int o = PW; o < 64; o <<= 1) tot += __shfl_xor(tot, o);
    if (oscale) tot *= oscale[i];
    if (grp == 0) out[i * nfs + PW * blockIdx.y + fl] = tot;  // zero for padded rows / columns
}

template <bool SLOT>
static void spmm(int pw, int nf, dim3 grid, hipStream_t stream, const int64_t* ptr, const int32_t* idx,
                 const float* val, int64_t n_valid, int64_t i0, int64_t i1, const float* Y, int64_t yplane, float* out,
                 const float* oscale, const int* skip, const char* what) {
    if ((nf != 16 && nf != 32 && nf != 64 && nf != 128) || nf % pw != 0)
        throw std::runtime_error(std::string(what) + ": nf must be 16, 32, 64 or 128");
    auto go = [&](auto k) {
        hipLaunchKernelGGL(k, grid, dim3(256), 0, stream, ptr, idx, val, n_valid, i0, i1, Y, yplane, out, oscale, nf,
                           skip);
    };
    switch (pw) {
        case 16: go(k_mf_sparse_spmm<16, SLOT>); break;
        case 32: go(k_mf_sparse_spmm<32, SLOT>); break;
        case 64: go(k_mf_sparse_spmm<64, SLOT>); break;
        default: throw std::runtime_error(std::string(what) + ": plane width must be 16, 32 or 64");
    }
    check_launch(what);
}

void launch_mf_sparse_forward(const SparseRtm& s, int64_t nrows, int64_t nrows_pad, const float* X, int64_t ld,
                              float* Xt, float* Fout, int nf, int pw, hipStream_t stream, const int* skip) {
    check_sparse(s, "mf_sparse_forward");
    check_pw(nf, pw, "mf_sparse_forward");
    if (ld % 64 != 0) throw std::runtime_error("mf_sparse_forward: ld must be a multiple of 64");
    hipLaunchKernelGGL(k_mf_transpose_x, dim3((unsigned)(ld / 64), (unsigned)((nf + 63) / 64)), dim3(256), 0, stream,
                       X, ld, nf, pw, Xt, skip);
    check_launch("k_mf_transpose_x");
    const dim3 grid((unsigned)((nrows_pad + 3) / 4), (unsigned)(nf / pw));
    spmm<false>(pw, nf, grid, stream, s.row_ptr, s.col, s.val, nrows, 0, nrows_pad, Xt, ld * pw, Fout, nullptr, skip,
                "k_mf_sparse_spmm (forward)");
}

void launch_mf_w_planes(const float* W, int64_t rows, int nf, int pw, float* Wt, hipStream_t stream,
                        const int* skip) {
    check_pw(nf, pw, "mf_w_planes");
    hipLaunchKernelGGL(k_mf_w_planes, dim3((unsigned)((rows * nf + 255) / 256)), dim3(256), 0, stream, W, rows, nf,
                       pw, Wt, skip);
    check_launch("k_mf_w_planes");
}

void launch_mf_sparse_backproject(const SparseRtm& s, int64_t nvoxel, const float* W, int64_t wrows, float* part,
                                  const float* scale, int nf, int pw, int64_t v0, int64_t v1, hipStream_t stream,
                                  const int* skip) {
    check_sparse(s, "mf_sparse_backproject");
    check_pw(nf, pw, "mf_sparse_backproject");
    if (v1 <= v0) return;
    const dim3 grid((unsigned)((v1 - v0 + 3) / 4), (unsigned)(nf / pw));
    // W in its slot layout or the frame-order planes of launch_mf_w_planes (mf_sparse_needs_w_planes)
    if (!mf_sparse_needs_w_planes(nf, pw))
        spmm<true>(pw, nf, grid, stream, s.col_ptr, s.row, s.cval, nvoxel, v0, v1, W, 0, part, scale, skip,
                   "k_mf_sparse_spmm (back-projection)");
    else
        spmm<false>(pw, nf, grid, stream, s.col_ptr, s.row, s.cval, nvoxel, v0, v1, W, wrows * pw, part, scale, skip,
                    "k_mf_sparse_spmm (back-projection)");
}

int sparse_lanes(double avg) {
    if (const char* e = std::getenv("SART_SPARSE_LANES"); e && *e) {  // (an A/B knob: a typo must not run the default)
        const int l = std::atoi(e);
        if (l == 4 || l == 8 || l == 16 || l == 32) return l;
        throw std::runtime_error(std::string("SART_SPARSE_LANES must be 4, 8, 16 or 32, not '") + e + "'");
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
