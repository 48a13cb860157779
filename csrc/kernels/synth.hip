// On-device synthetic data for benchmarks and tests (no HDF5, no host copy of the matrix).
//
// Every element is a pure function of (seed, global row, column), so a matrix generated as N row
// shards on N GPUs is bit-identical to the one generated on one GPU: solutions can be compared
// across GPU counts. The reference has no synthetic path (it always reads HDF5, raytransfer.cpp:27).
#include "launchers.hpp"

namespace sart {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ float u01(uint64_t seed, uint64_t idx) {
    const uint64_t z = mix64(seed * 0x9E3779B97F4A7C15ull + idx + 0x632BE59BD9B4E019ull);
    return (float)(z >> 40) * (1.0f / 16777216.0f);  // [0, 1)
}

// A[r][c] = lo + (hi - lo) * U(seed, (row_offset + r) * ncols_total + col_offset + c) on the valid block
// (c < ncols), 0 in the padding: element (R, C) of one global matrix, for row or column shards alike.
__global__ __launch_bounds__(256) void k_synth_matrix(float* __restrict__ A, int64_t ld, int64_t nrows_pad,
                                                      int64_t nrows, int64_t ncols, int64_t row_offset,
                                                      int64_t col_offset, int64_t ncols_total,
                                                      uint64_t seed, float lo, float hi) {
    const int64_t ld4 = ld >> 2;
    const int64_t total4 = nrows_pad * ld4;
    const float span = hi - lo;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / ld4;
        const int64_t c = (i - r * ld4) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < nrows) {
            const uint64_t base = (uint64_t)(row_offset + r) * (uint64_t)ncols_total + (uint64_t)col_offset;
            if (c + 0 < ncols) v.x = lo + span * u01(seed, base + c + 0);
            if (c + 1 < ncols) v.y = lo + span * u01(seed, base + c + 1);
            if (c + 2 < ncols) v.z = lo + span * u01(seed, base + c + 2);
            if (c + 3 < ncols) v.w = lo + span * u01(seed, base + c + 3);
        }
        reinterpret_cast<float4*>(A)[i] = v;
    }
}

__global__ __launch_bounds__(256) void k_synth_vector(double* __restrict__ out, int64_t n, int64_t offset,
                                                      uint64_t seed, double lo, double hi) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    out[i] = lo + (hi - lo) * (double)u01(seed, (uint64_t)(offset + i));
}

void launch_synth_matrix(float* A, int64_t ld, int64_t nrows_pad, int64_t nrows, int64_t ncols, int64_t row_offset,
                         uint64_t seed, float lo, float hi, hipStream_t stream) {
    launch_synth_matrix_block(A, ld, nrows_pad, nrows, ncols, row_offset, 0, ncols, seed, lo, hi, stream);
}

void launch_synth_matrix_block(float* A, int64_t ld, int64_t nrows_pad, int64_t nrows, int64_t ncols,
                               int64_t row_offset, int64_t col_offset, int64_t ncols_total, uint64_t seed, float lo,
                               float hi, hipStream_t stream) {
    const int64_t total4 = nrows_pad * (ld / 4);
    int64_t nblk = (total4 + 255) / 256;
    if (nblk > 65536) nblk = 65536;
    if (nblk < 1) nblk = 1;
    hipLaunchKernelGGL(k_synth_matrix, dim3((unsigned)nblk), dim3(256), 0, stream, A, ld, nrows_pad, nrows, ncols,
                       row_offset, col_offset, ncols_total, seed, lo, hi);
    check_launch("k_synth_matrix");
}

void launch_synth_vector(double* out, int64_t n, int64_t offset, uint64_t seed, double lo, double hi,
                         hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_synth_vector, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, out, n, offset, seed,
                       lo, hi);
    check_launch("k_synth_vector");
}

}  // namespace sart
