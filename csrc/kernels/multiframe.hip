// Multi-frame (batched right-hand side) projections on the fp32 matrix cores of gfx950.
//
// The reference solves frames strictly one after another (reference main.cpp:131-140), streaming
// the whole RTM twice per iteration per frame. Solving NF = 16 frames together turns A.x and A^T.w
// into skinny GEMMs (A.X with X in R^{V x 16}, A^T.W with W in R^{P x 16}) that reuse every byte of
// A 16 times. They run on v_mfma_f32_16x16x4_f32 (exact fp32, 1 fp32 VGPR per operand per lane).
//
// K-permutation trick: each lane loads ONE float4 of A (16 contiguous bytes); component c of that
// float4 is the lane's operand of MFMA k-step c. Any bijection between k-steps and voxels (forward) /
// voxels and output rows (back-projection) is legal as long as both operands and the epilogue agree,
// so no LDS transpose is needed.
//
// MFMA 16x16x4 f32 fragment maps (cdna_hip_programming.md section 3):
//   A operand: lane l holds A[i = l & 15][k = l >> 4]; B operand: B[k = l >> 4][j = l & 15];
//   C/D: col = l & 15, row = (l >> 4) * 4 + reg.
#include "sart_common.hpp"

#include <stdexcept>

namespace sart {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kNF = 16;  // frames per batch (the MFMA N dimension)

__device__ __forceinline__ float comp(const float4& v, int c) {
    return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}

// F[row][f] = sum_v A[row][v] X[f][v]. X is frame-major [16][ldx] (ldx == ld), F is [rows][16].
// One wave: 32 rows (two 16-row tiles sharing the X fragment) x 16 frames, K = all voxels.
// Split-K: blockIdx.y selects the column range [k0, k1) (multiples of 16 columns) and the kernel
// writes Fout + blockIdx.y * nrows_pad * 16; the caller sums the splits.
__global__ __launch_bounds__(256) void k_mf_forward(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                    int64_t nrows_pad, const float* __restrict__ X,
                                                    int64_t ldx, float* __restrict__ Fout, int64_t cols_per_split) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * 32;
    if (row0 >= nrows_pad) return;  // wave-uniform
    const int g = lane >> 4, r = lane & 15;
    const int64_t ld4 = ld >> 2, ldx4 = ldx >> 2;
    const int64_t c0 = (int64_t)blockIdx.y * cols_per_split;
    const int64_t c1 = (c0 + cols_per_split < ld) ? c0 + cols_per_split : ld;
    Fout += (int64_t)blockIdx.y * nrows_pad * kNF;
    const float4* __restrict__ a0p = reinterpret_cast<const float4*>(A) + (row0 + r) * ld4 + g + c0 / 4;
    const float4* __restrict__ a1p = a0p + 16 * ld4;
    const float4* __restrict__ xp = reinterpret_cast<const float4*>(X) + (int64_t)r * ldx4 + g + c0 / 4;

    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    int64_t q = 0;
    const int64_t nq = c1 > c0 ? (c1 - c0) / 4 : 0;  // float4 columns; 4 lane-groups x float4 = 16 voxels/step
    for (; q + 8 <= nq; q += 8) {
        const float4 a00 = a0p[q], a10 = a1p[q], x0 = xp[q];
        const float4 a01 = a0p[q + 4], a11 = a1p[q + 4], x1 = xp[q + 4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a00, c), comp(x0, c), acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a10, c), comp(x0, c), acc1, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a01, c), comp(x1, c), acc2, 0, 0, 0);
            acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a11, c), comp(x1, c), acc3, 0, 0, 0);
        }
    }
    for (; q < nq; q += 4) {
        const float4 a00 = a0p[q], a10 = a1p[q], x0 = xp[q];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a00, c), comp(x0, c), acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a10, c), comp(x0, c), acc1, 0, 0, 0);
        }
    }
    // D: col = frame = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t ra = row0 + g * 4 + i, rb = ra + 16;
        if (ra < nrows) Fout[ra * kNF + r] = acc0[i] + acc2[i];
        if (rb < nrows) Fout[rb * kNF + r] = acc1[i] + acc3[i];
    }
}

// partial[s][v][f] = sum_{rows of split s} A[row][v] W[row][f]. W is [rows][16].
// One wave: 64 voxels x 16 frames; a float4 of A (4 voxels of one row) feeds 4 MFMAs, one per output
// tile c, whose voxel set is {v0 + 4 i + c : i = 0..15}.
__global__ __launch_bounds__(256) void k_mf_backproject(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                        const float* __restrict__ W, int64_t rows_per_split,
                                                        float* __restrict__ partial) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t vb = (int64_t)blockIdx.x * 4 + wave;  // 64-voxel block
    if (vb * 64 >= ld) return;
    const int g = lane >> 4, i16 = lane & 15;
    const int64_t ld4 = ld >> 2;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows) r_end = nrows;

    const float4* __restrict__ ap = reinterpret_cast<const float4*>(A) + vb * 16 + i16;
    floatx4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};

    int64_t r0 = r_begin;
    for (; r0 + 16 <= r_end; r0 += 16) {
        float4 av[4];
        float wv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            av[u] = ap[(r0 + 4 * u + g) * ld4];
            wv[u] = W[(r0 + 4 * u + g) * kNF + i16];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(av[u], c), wv[u], acc[c], 0, 0, 0);
    }
    for (; r0 < r_end; r0 += 4) {
        const int64_t row = r0 + g;
        float4 av = make_float4(0.f, 0.f, 0.f, 0.f);
        float wv = 0.f;
        if (row < r_end) {
            av = ap[row * ld4];
            wv = W[row * kNF + i16];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(av, c), wv, acc[c], 0, 0, 0);
    }
    float* out = partial + (int64_t)blockIdx.y * ld * kNF;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t v = vb * 64 + 4 * (g * 4 + q) + c;
            out[v * kNF + i16] = acc[c][q];
        }
}

int mf_forward_num_splits(int64_t ld, int64_t nrows_pad) {
    const int64_t nblk = (nrows_pad + 127) / 128;
    int64_t s = (1024 + nblk - 1) / nblk;  // >= ~1024 workgroups
    const int64_t smax = ld / 1024;        // >= 1024 columns per split
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    return (int)s;
}

void launch_mf_forward(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* X, int64_t ldx,
                       float* Fout, int nsplit, hipStream_t stream) {
    if (ld % 64 != 0 || ldx != ld) throw std::runtime_error("mf_forward: ld must be a multiple of 64 and ldx == ld");
    if (nrows_pad % 32 != 0) throw std::runtime_error("mf_forward: padded rows must be a multiple of 32");
    if (nsplit < 1) throw std::runtime_error("mf_forward: nsplit must be >= 1");
    const int64_t nblk = (nrows_pad + 127) / 128;
    const int64_t cps = ((ld + nsplit - 1) / nsplit + 15) / 16 * 16;
    hipLaunchKernelGGL(k_mf_forward, dim3((unsigned)nblk, (unsigned)nsplit), dim3(256), 0, stream, A, ld, nrows,
                       nrows_pad, X, ldx, Fout, cps);
    check_launch("k_mf_forward");
}

int mf_backproject_num_splits(int64_t ld, int64_t nrows) {
    const int64_t nblk = (ld / 64 + 3) / 4;
    int64_t s = (2048 + nblk - 1) / nblk;
    const int64_t smax = (nrows + 63) / 64;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    return (int)s;
}

void launch_mf_backproject(const float* A, int64_t ld, int64_t nrows, const float* W, int nsplit, float* partial,
                           hipStream_t stream) {
    if (ld % 64 != 0) throw std::runtime_error("mf_backproject: ld must be a multiple of 64");
    const int64_t rps = ((nrows + nsplit - 1) / nsplit + 15) / 16 * 16;
    const int64_t nblk = (ld / 64 + 3) / 4;
    hipLaunchKernelGGL(k_mf_backproject, dim3((unsigned)nblk, (unsigned)nsplit), dim3(256), 0, stream, A, ld, nrows,
                       W, rps, partial);
    check_launch("k_mf_backproject");
}

}  // namespace sart
