// Multi-frame (batched right-hand side) projections on the fp32 matrix cores of gfx950.
//
// The reference solves frames strictly one after another (reference main.cpp:131-140), streaming
// the whole RTM twice per iteration per frame. Solving nf = 16, 32 or 64 frames together turns A.x and
// A^T.w into skinny GEMMs (A.X with X in R^{V x nf}, A^T.W with W in R^{P x nf}) that reuse every byte
// of A nf times. They run on v_mfma_f32_16x16x4_f32 (exact fp32, 1 fp32 VGPR per operand per lane), one
// MFMA column group per 16 frames (NG = nf / 16 groups).
//
// Rate model (MI355X_MICROARCH.md: 64 fp32 MFMA flop/clk/SIMD, 155 TFLOPS): a column group costs 32 SIMD
// cycles per 1 KiB wave-load of A, so the matrix cores consume A at ~19.6 TB/s with nf = 16, ~9.8 TB/s
// with nf = 32 (both above the ~6 TB/s HBM stream: bandwidth-bound) and ~4.9 TB/s with nf = 64
// (matrix-core-bound, but 4x the frames per byte). Measured per-kernel rates: tools/probe_mf.py.
//
// K-permutation trick: each lane loads ONE float4 of A (16 contiguous bytes); component c of that
// float4 is the lane's operand of MFMA k-step c. Any bijection between k-steps and voxels (forward) /
// voxels and output rows (back-projection) is legal as long as both operands and the epilogue agree,
// so no LDS transpose is needed.
//
// The back-projection streams whole 256-B row segments per instruction with the non-temporal hint
// (load_stream, sart_common.hpp): 8 % faster at nf = 16.
//
// Latency hiding: each wave keeps DEPTH steps of A (and X / W) loads in flight in a register ring of
// DEPTH + 1 slots (step t issues the loads of step t + DEPTH into the slot step t - 1 consumed), so the
// ~2-3 us HBM latency under load is covered by DEPTH steps of matrix-core work instead of one.
//
// MFMA 16x16x4 f32 fragment maps (cdna_hip_programming.md section 3):
//   A operand: lane l holds A[i = l & 15][k = l >> 4]; B operand: B[k = l >> 4][j = l & 15];
//   C/D: col = l & 15, row = (l >> 4) * 4 + reg.
#include "sart_common.hpp"
#include "launchers.hpp"

#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>

namespace sart {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float comp(const float4& v, int c) {
    return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}

// NG contiguous floats (the column groups of one lane's B operand in the back-projection layout).
template <int NG>
__device__ __forceinline__ void load_groups(float (&dst)[NG], const float* __restrict__ p) {
    if constexpr (NG == 4) {
        const float4 v = *reinterpret_cast<const float4*>(p);
        dst[0] = v.x, dst[1] = v.y, dst[2] = v.z, dst[3] = v.w;
    } else if constexpr (NG == 2) {
        const float2 v = *reinterpret_cast<const float2*>(p);
        dst[0] = v.x, dst[1] = v.y;
    } else {
        dst[0] = *p;
    }
}

#ifndef SART_MF_FLUSH
#define SART_MF_FLUSH 2  // (see multiframe_bf16.hip)
#endif
// F[row][f] = sum_v A[row][v] X[f][v]. X is frame-major [nf][ldx] (ldx == ld), F is [rows][nf].
// One wave: 16 * RT rows (RT 16-row tiles sharing each X fragment) x nf frames, K = the columns of its
// split; every float4 of A feeds 4 * NG MFMAs (one per k-component and column group) and every X
// fragment 4 * RT. RT = 4 halves the X operand traffic per byte of A against RT = 2 (X is L2 / MALL
// resident, but at nf = 64 it is twice the A stream with RT = 2).
// Split-K: blockIdx.y selects the column range [k0, k1) (multiples of 16 columns) and the kernel
// writes Fout + blockIdx.y * nrows_pad * nf; the caller sums the splits.
template <int NG, int DEPTH, int RT, bool NT>
__global__ __launch_bounds__(256) void k_mf_forward(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                    int64_t nrows_pad, const float* __restrict__ X,
                                                    int64_t ldx, float* __restrict__ Fout, int64_t cols_per_split,
                                                    const int* __restrict__ skip) {
    if (skip && *skip) return;  // every frame of the batch is done: the sweep is a no-op
    constexpr int NF = 16 * NG;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * (16 * RT);
    if (row0 >= nrows_pad) return;  // wave-uniform; nrows_pad is a multiple of 16 * RT
    const int g = lane >> 4, r = lane & 15;
    const int64_t ld4 = ld >> 2, ldx4 = ldx >> 2;
    const int64_t c0 = (int64_t)blockIdx.y * cols_per_split;
    const int64_t c1 = (c0 + cols_per_split < ld) ? c0 + cols_per_split : ld;
    Fout += (int64_t)blockIdx.y * nrows_pad * NF;
    const float4* __restrict__ a0p = reinterpret_cast<const float4*>(A) + (row0 + r) * ld4 + g + c0 / 4;
    const float4* __restrict__ xp = reinterpret_cast<const float4*>(X) + (int64_t)r * ldx4 + g + c0 / 4;
    const int64_t xg = 16 * ldx4;  // next column group of X

    floatx4 acc[RT][2][NG];  // [row tile][k half][column group]
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < NG; ++j) acc[t][h][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // two-level accumulation (as k_mf_forward_b16_lds, SART_MF_FLUSH): K = 4 per MFMA makes the chains of a
    // 16k-voxel split 4096 fp32 additions long (9.8x the fp32 two-pass kernels' error at 64k x 64k after 20 SART
    // updates). Where the second set fits the register budget (RT NG <= 8: the 16-frame default)
    constexpr bool FL = SART_MF_FLUSH > 0 && RT * NG <= 8;
    floatx4 sum[FL ? RT : 1][FL ? NG : 1];
    if constexpr (FL) {
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int j = 0; j < NG; ++j) sum[t][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    auto flush = [&] {
        if constexpr (FL) {
#pragma unroll
            for (int t = 0; t < RT; ++t)
#pragma unroll
                for (int j = 0; j < NG; ++j) {
                    sum[t][j] += acc[t][0][j] + acc[t][1][j];
                    acc[t][0][j] = acc[t][1][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                }
        }
    };

    const int64_t nq = c1 > c0 ? (c1 - c0) / 4 : 0;  // float4 columns; 4 lane-groups x float4 = 16 voxels
    const int64_t nst = nq / 8;                        // 8-float4 steps
    if (nst > 0) {
        constexpr int RS = DEPTH + 1;
        float4 a[RS][RT][2], x[RS][2][NG];
        auto load = [&](int sl, int64_t t) {
            const int64_t qq = t * 8;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)  // plain loads: a row's two 64-B halves come from two
                    a[sl][rt][h] = NT ? load_stream(a0p + rt * 16 * ld4 + qq + 4 * h)  // SART_MF_NT=1
                                      : a0p[rt * 16 * ld4 + qq + 4 * h];  // instructions; nt measured slower
#pragma unroll
                for (int j = 0; j < NG; ++j) x[sl][h][j] = xp[j * xg + qq + 4 * h];
            }
        };
        // Unconditional loads, clamped to the last step: with path-independent load counts the compiler
        // keeps DEPTH steps in flight (counted vmcnt) instead of draining the ring at every step.
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) load(d, d < nst ? d : nst - 1);
        auto step = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            load((sl + DEPTH) % RS, t + DEPTH < nst ? t + DEPTH : nst - 1);
            if (t >= nst) return;
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int j = 0; j < NG; ++j)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt)
                            acc[rt][h][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(a[sl][rt][h], c),
                                                                                comp(x[sl][h][j], c), acc[rt][h][j],
                                                                                0, 0, 0);
        };
        for (int64_t t0 = 0, it = 0; t0 < nst; t0 += RS, ++it) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (step(std::integral_constant<int, Q>{}, t0 + Q), ...);
            }(std::make_integer_sequence<int, RS>{});
            if constexpr (FL)
                if (it % SART_MF_FLUSH == SART_MF_FLUSH - 1) flush();
        }
    }
    for (int64_t q = nst * 8; q < nq; q += 4) {  // 4-float4 tail of a ragged split
        float4 at[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) at[rt] = a0p[rt * 16 * ld4 + q];
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            const float4 x0 = xp[j * xg + q];
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
                    acc[rt][0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(at[rt], c), comp(x0, c), acc[rt][0][j],
                                                                        0, 0, 0);
        }
    }
    // D: col = frame = 16 j + (lane & 15), row = (lane >> 4) * 4 + reg
#pragma unroll
    for (int j = 0; j < NG; ++j)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t ra = row0 + rt * 16 + g * 4 + i;
                if constexpr (FL) {
                    if (ra < nrows) Fout[ra * NF + 16 * j + r] = sum[rt][j][i] + (acc[rt][0][j][i] + acc[rt][1][j][i]);
                } else {
                    if (ra < nrows) Fout[ra * NF + 16 * j + r] = acc[rt][0][j][i] + acc[rt][1][j][i];
                }
            }
}

// partial[s][v][f] = sum_{rows of split s} A[row][v] W[row][f]. W is in the back-projection layout
// [rows][16][NG] (frame f = 16 j + i at position i * NG + j, mf_bp_slot in multiframe_glue.hip), so a
// lane's NG column-group operands are one contiguous vector load. partial is [splits][ld][nf] in natural
// frame order. One wave: 64 * VT voxels x nf frames; a float4 of A (4 voxels of one row) feeds 4 * NG
// MFMAs, one per output tile c (voxel set {v0 + 4 i + c : i = 0..15}) and column group j, and every W
// operand feeds 4 * VT (VT = 2 halves the W traffic per byte of A; needs ld % 128 == 0).
// Voxel range: the blocks of 64 * VT voxels from vb0 (blockIdx.x = 0) up to voxel vend (the chunks of the
// engine's all-reduce pipeline; the whole row is vb0 = 0, vend = ld).
template <int NG, int DEPTH, int VT>
__global__ __launch_bounds__(256) void k_mf_backproject(const float* __restrict__ A, int64_t ld, int64_t nrows,
                                                        const float* __restrict__ W, int64_t rows_per_split,
                                                        float* __restrict__ partial, int64_t vb0, int64_t vend,
                                                        const int* __restrict__ skip) {
    if (skip && *skip) return;
    constexpr int NF = 16 * NG;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t vb = vb0 + (int64_t)blockIdx.x * 4 + wave;  // block of 64 * VT voxels
    if (vb * 64 * VT >= vend) return;
    const int g = lane >> 4, i16 = lane & 15;
    const int64_t ld4 = ld >> 2;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows) r_end = nrows;

    const float4* __restrict__ ap = reinterpret_cast<const float4*>(A) + vb * 16 * VT + i16;
    const float* __restrict__ wp = W + i16 * NG;
    floatx4 acc[VT][4][NG];
#pragma unroll
    for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < NG; ++j) acc[vt][c][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // two-level accumulation (SART_MF_FLUSH, as k_mf_forward) where the second set fits (VT NG <= 2: 16 frames)
    constexpr bool FL = SART_MF_FLUSH > 0 && VT * NG <= 2;
    floatx4 sum[FL ? VT : 1][4][FL ? NG : 1];
    if constexpr (FL) {
#pragma unroll
        for (int vt = 0; vt < VT; ++vt)
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int j = 0; j < NG; ++j) sum[vt][c][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    auto flush = [&] {
        if constexpr (FL) {
#pragma unroll
            for (int vt = 0; vt < VT; ++vt)
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int j = 0; j < NG; ++j) sum[vt][c][j] += acc[vt][c][j], acc[vt][c][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
    };

    const int64_t nst = r_end > r_begin ? (r_end - r_begin) / 16 : 0;  // 16-row steps
    if (nst > 0) {
        constexpr int RS = DEPTH + 1;
        float4 av[RS][4][VT];
        float wv[RS][4][NG];
        auto load = [&](int sl, int64_t t) {
            const int64_t rr = r_begin + t * 16;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int vt = 0; vt < VT; ++vt) av[sl][u][vt] = load_stream(ap + (rr + 4 * u + g) * ld4 + vt * 16);
                load_groups<NG>(wv[sl][u], wp + (rr + 4 * u + g) * NF);
            }
        };
        // Unconditional loads, clamped to the last step (see k_mf_forward): counted vmcnt in the ring.
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) load(d, d < nst ? d : nst - 1);
        auto step = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            load((sl + DEPTH) % RS, t + DEPTH < nst ? t + DEPTH : nst - 1);
            if (t >= nst) return;
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int j = 0; j < NG; ++j)
#pragma unroll
                        for (int vt = 0; vt < VT; ++vt)
                            acc[vt][c][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(av[sl][u][vt], c), wv[sl][u][j],
                                                                                acc[vt][c][j], 0, 0, 0);
        };
        for (int64_t t0 = 0, it = 0; t0 < nst; t0 += RS, ++it) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (step(std::integral_constant<int, Q>{}, t0 + Q), ...);
            }(std::make_integer_sequence<int, RS>{});
            if constexpr (FL)
                if (it % SART_MF_FLUSH == SART_MF_FLUSH - 1) flush();
        }
    }
    for (int64_t r0 = r_begin + nst * 16; r0 < r_end; r0 += 4) {  // ragged tail, 4 rows per MFMA
        const int64_t row = r0 + g;
        float4 av[VT];
        float wv[NG];
#pragma unroll
        for (int vt = 0; vt < VT; ++vt) av[vt] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < NG; ++j) wv[j] = 0.f;
        if (row < r_end) {
#pragma unroll
            for (int vt = 0; vt < VT; ++vt) av[vt] = load_stream(ap + row * ld4 + vt * 16);
            load_groups<NG>(wv, wp + row * NF);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < NG; ++j)
#pragma unroll
                for (int vt = 0; vt < VT; ++vt)
                    acc[vt][c][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(av[vt], c), wv[j], acc[vt][c][j], 0, 0, 0);
    }
    float* out = partial + (int64_t)blockIdx.y * ld * NF;
#pragma unroll
    for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t v = (vb * VT + vt) * 64 + 4 * (g * 4 + q) + c;
#pragma unroll
                for (int j = 0; j < NG; ++j) {
                    if constexpr (FL) out[v * NF + 16 * j + i16] = sum[vt][c][j][q] + acc[vt][c][j][q];
                    else out[v * NF + 16 * j + i16] = acc[vt][c][j][q];
                }
            }
}

// Split-K of the forward projection: >= ~1024 workgroups, >= 1024 columns per split. (Splitting further
// so that a split's X chunk stays L2-resident measured 0-9 % slower at nf = 16..64, 64k x 64k.)
static int mf_rows(int nf);
int mf_forward_num_splits(int64_t ld, int64_t nrows_pad, int target_blocks) {
    const int64_t rows_per_block = (nrows_pad % 64 == 0 ? mf_rows(0) : 2) * 64;  // 4 waves x 16 * rt rows
    const int64_t nblk = (nrows_pad + rows_per_block - 1) / rows_per_block;
    const char* e = std::getenv("SART_MF_FWD_BLOCKS");  // target workgroups (tuning knob)
    const int64_t target = (e && *e) ? std::atoll(e) : (target_blocks > 0 ? target_blocks : 1024);
    int64_t s = (target + nblk - 1) / nblk;
    const int64_t smax = ld / 1024;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    return (int)s;
}

static int mf_vox(int64_t ld, int nf);
// Split-K of the back-projection: ~512 workgroups. The kernel time is flat from 4 to 32 splits at
// 64k x 64k (profiles/probe_r1_mf_splits.jsonl) while k_mf_collect reads nsplit partial slices.
int mf_backproject_num_splits(int64_t ld, int64_t nrows) {
    const int64_t nblk = (ld / (64 * mf_vox(ld, 64)) + 3) / 4;  // the fp32 kernels' widest batch
    const char* e = std::getenv("SART_MF_BP_BLOCKS");  // target workgroups (tuning knob)
    // 2048 (4 x the 512 of round 1): a split's rows are one fp32 MFMA accumulation chain; 16k-row splits at 64k x 64k
    // were the larger share of the multi-frame engine's error against the fp32 two-pass kernels
    // (profiles/parity_r6_64k_mf_chains.jsonl); the extra partial slices cost k_mf_collect ~1.5 % of a sweep
    const int64_t target = (e && *e) ? std::atoll(e) : 2048;
    int64_t s = (target + nblk - 1) / nblk;
    const int64_t smax = (nrows + 63) / 64;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    return (int)s;
}

static void check_nf(int nf, const char* what) {
    if (nf != 16 && nf != 32 && nf != 64) throw std::runtime_error(std::string(what) + ": nf must be 16, 32 or 64");
}

// Register-ring depth (steps of loads in flight per wave). Defaults per kernel and batch width from
// tools/probe_mf.py on 64k x 64k (profiles/probe_r1_mf_tiles.jsonl, with the default tilings below: forward
// 64 rows per wave, back-projection 64 voxels per wave at nf = 16 and 128 at nf = 32 / 64); SART_MF_DEPTH=1..3
// or mf_set_depth() overrides them.
static int g_mf_depth = -1;
void mf_set_depth(int d) { g_mf_depth = d; }
static int mf_depth(bool forward, int nf) {
    if (g_mf_depth < 0) {
        const char* e = std::getenv("SART_MF_DEPTH");
        g_mf_depth = (e && *e) ? std::atoi(e) : 0;
    }
    if (g_mf_depth >= 1 && g_mf_depth <= 3) return g_mf_depth;
    if (forward) return nf == 64 ? 2 : 3;           // with 64-row waves (profiles/probe_r1_mf_tiles.jsonl)
    return nf == 32 ? 1 : 2;                         // nf 16: 64-voxel waves; nf 32 / 64: 128-voxel waves
}

// 64-voxel tiles per wave of the back-projection: 1 or 2 (ld % 128 == 0); SART_MF_VOX or mf_set_vox().
static int g_mf_vox = -1;
void mf_set_vox(int vt) { g_mf_vox = vt; }
static int mf_vox(int64_t ld, int nf) {
    if (g_mf_vox < 0) {
        const char* e = std::getenv("SART_MF_VOX");
        g_mf_vox = (e && *e) ? std::atoi(e) : 0;
    }
    const int vt = (g_mf_vox == 1 || g_mf_vox == 2) ? g_mf_vox : (nf >= 32 ? 2 : 1);
    return (vt == 2 && ld % 128 == 0) ? 2 : 1;
}

// Row tiles per wave of the forward kernel: 2 (32 rows) or 4 (64 rows); SART_MF_ROWS or mf_set_rows().
static int g_mf_rows = -1;
void mf_set_rows(int rt) { g_mf_rows = rt; }
static int mf_rows(int nf) {
    if (g_mf_rows < 0) {
        const char* e = std::getenv("SART_MF_ROWS");
        g_mf_rows = (e && *e) ? std::atoi(e) : 0;
    }
    if (g_mf_rows == 2 || g_mf_rows == 4) return g_mf_rows;
    (void)nf;
    return 4;
}

template <int NG, int RT, bool NT>
static void fwd_rt_nt(dim3 grid, int depth, hipStream_t stream, const float* A, int64_t ld, int64_t nrows,
                      int64_t nrows_pad, const float* X, int64_t ldx, float* Fout, int64_t cps) {
    if (depth == 1)
        hipLaunchKernelGGL((k_mf_forward<NG, 1, RT, NT>), grid, dim3(256), 0, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, cps, g_mf_skip);
    else if (depth == 3)
        hipLaunchKernelGGL((k_mf_forward<NG, 3, RT, NT>), grid, dim3(256), 0, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, cps, g_mf_skip);
    else
        hipLaunchKernelGGL((k_mf_forward<NG, 2, RT, NT>), grid, dim3(256), 0, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, cps, g_mf_skip);
}

// Non-temporal A loads in the MFMA forward (experiment knob, SART_MF_NT=1; default plain loads).
static int mf_nt() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("SART_MF_NT");
        v = (e && *e) ? std::atoi(e) : 0;
    }
    return v;
}

template <int NG, int RT>
static void fwd_rt(dim3 grid, int depth, hipStream_t stream, const float* A, int64_t ld, int64_t nrows,
                   int64_t nrows_pad, const float* X, int64_t ldx, float* Fout, int64_t cps) {
    if (mf_nt() == 1)
        fwd_rt_nt<NG, RT, true>(grid, depth, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, cps);
    else
        fwd_rt_nt<NG, RT, false>(grid, depth, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, cps);
}

template <int NG>
static void fwd(int rt, int depth, hipStream_t stream, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                const float* X, int64_t ldx, float* Fout, int nsplit, int64_t cps) {
    const dim3 grid((unsigned)((nrows_pad + 64 * rt - 1) / (64 * rt)), (unsigned)nsplit);
    if (rt == 4)
        fwd_rt<NG, 4>(grid, depth, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, cps);
    else
        fwd_rt<NG, 2>(grid, depth, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, cps);
}

void launch_mf_forward(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* X, int64_t ldx,
                       float* Fout, int nsplit, int nf, hipStream_t stream) {
    if (ld % 64 != 0 || ldx != ld) throw std::runtime_error("mf_forward: ld must be a multiple of 64 and ldx == ld");
    if (nrows_pad % 32 != 0) throw std::runtime_error("mf_forward: padded rows must be a multiple of 32");
    if (nsplit < 1) throw std::runtime_error("mf_forward: nsplit must be >= 1");
    check_nf(nf, "mf_forward");
    const int64_t cps = ((ld + nsplit - 1) / nsplit + 15) / 16 * 16;
    const int d = mf_depth(true, nf);
    const int rt = (nrows_pad % 64 == 0) ? mf_rows(nf) : 2;  // a wave's 16 * rt rows lie inside the padding
    if (nf == 16)
        fwd<1>(rt, d, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, nsplit, cps);
    else if (nf == 32)
        fwd<2>(rt, d, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, nsplit, cps);
    else
        fwd<4>(rt, d, stream, A, ld, nrows, nrows_pad, X, ldx, Fout, nsplit, cps);
    check_launch("k_mf_forward");
}

template <int NG, int VT>
static void bwd_vt(dim3 grid, int depth, hipStream_t stream, const float* A, int64_t ld, int64_t nrows, const float* W,
                   int64_t rps, float* partial, int64_t vb0, int64_t vend) {
    if (depth == 1)
        hipLaunchKernelGGL((k_mf_backproject<NG, 1, VT>), grid, dim3(256), 0, stream, A, ld, nrows, W, rps, partial,
                           vb0, vend, g_mf_skip);
    else if (depth == 3)
        hipLaunchKernelGGL((k_mf_backproject<NG, 3, VT>), grid, dim3(256), 0, stream, A, ld, nrows, W, rps, partial,
                           vb0, vend, g_mf_skip);
    else
        hipLaunchKernelGGL((k_mf_backproject<NG, 2, VT>), grid, dim3(256), 0, stream, A, ld, nrows, W, rps, partial,
                           vb0, vend, g_mf_skip);
}

template <int NG>
static void bwd(int vt, int depth, hipStream_t stream, const float* A, int64_t ld, int64_t nrows, const float* W,
                int nsplit, int64_t rps, float* partial, int64_t v0, int64_t v1) {
    const int64_t vb0 = v0 / (64 * vt), nvb = (v1 - v0 + 64 * vt - 1) / (64 * vt);
    const dim3 grid((unsigned)((nvb + 3) / 4), (unsigned)nsplit);
    if (vt == 2)
        bwd_vt<NG, 2>(grid, depth, stream, A, ld, nrows, W, rps, partial, vb0, v1);
    else
        bwd_vt<NG, 1>(grid, depth, stream, A, ld, nrows, W, rps, partial, vb0, v1);
}

int mf_backproject_vox_align(int64_t ld, int nf) { return 64 * mf_vox(ld, nf); }

void launch_mf_backproject(const float* A, int64_t ld, int64_t nrows, const float* W, int nsplit, float* partial,
                           int nf, hipStream_t stream, int64_t v0, int64_t v1) {
    if (ld % 64 != 0) throw std::runtime_error("mf_backproject: ld must be a multiple of 64");
    check_nf(nf, "mf_backproject");
    if (v1 < 0) v1 = ld;
    const int vt = mf_vox(ld, nf);
    if (v0 < 0 || v1 > ld || v0 >= v1 || v0 % (64 * vt) != 0 || (v1 != ld && v1 % (64 * vt) != 0))
        throw std::runtime_error("mf_backproject: voxel range must be aligned to the wave's voxel tile");
    const int64_t rps = ((nrows + nsplit - 1) / nsplit + 15) / 16 * 16;
    const int d = mf_depth(false, nf);
    if (nf == 16)
        bwd<1>(vt, d, stream, A, ld, nrows, W, nsplit, rps, partial, v0, v1);
    else if (nf == 32)
        bwd<2>(vt, d, stream, A, ld, nrows, W, nsplit, rps, partial, v0, v1);
    else
        bwd<4>(vt, d, stream, A, ld, nrows, W, nsplit, rps, partial, v0, v1);
    check_launch("k_mf_backproject");
}

}  // namespace sart
