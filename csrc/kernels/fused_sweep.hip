// Fused single-pass SART sweep for gfx950: one HBM read of the local RTM shard per SART iteration.
//
// The reference streams A twice per iteration: PropagateKernel (A^T.w) and cublasSgemv (A.x)
// (reference sartsolver_cuda.cpp:239-249), i.e. 8*P*V bytes. Here every element of A is loaded into
// registers once and used for both products:
//
//   f_r  = sum_c A[r,c] x[c]              (forward projection, needs the whole row)
//   w_r  = a_r (ghat_r - f_r)   linear    (reference PropagateKernel weight, sart_kernels.cu:79-81)
//        = a_r f_r              log       (fitted half of LogPropagateKernel, sart_kernels.cu:134-146)
//   d_c += sum_r A[r,c] w_r               (back-projection)
//
// Decomposition: a persistent grid of I x J workgroups (<= one per CU, all co-resident).
// Workgroup (i, j) owns column slab j (Wc = 1024*K columns) of row group i and walks the row tiles
// (T = 8/K rows) of its group. Per tile it computes the J-th part of each row dot and publishes it
// as an 8-byte {epoch, value} granule with one write-through (sc1) store -- the data IS the flag,
// no fences (cdna_hip_programming.md Guideline 16, recipe R2). A dedicated exchange wave gathers the
// J granules of the previous tile, sums them in a fixed order (every workgroup of the group obtains
// a bitwise identical f_r), forms w_r and hands it to the four compute waves through LDS; they
// back-project the tile that is still held in registers (ring of 4 tiles: t-2 being back-projected,
// t-1 waiting for its weights, t being reduced, t+1 / t+2 in flight).
//
// Correctness does not depend on workgroup placement or dispatch order: every wait is on data
// tagged with this sweep's epoch, every spin is bounded, and a timeout sets SartState::error so
// the host falls back to the two-pass kernels (no hang, no silent wrong answer).
#include "sart_common.hpp"

#include <stdexcept>
#include <type_traits>

namespace sart {

constexpr int kFusedThreads = 320;  // 4 compute waves + 1 exchange wave
constexpr unsigned kSpinLimit = 1u << 18;

__device__ __forceinline__ uint64_t make_granule(int epoch, float v) {
    return ((uint64_t)(uint32_t)epoch << 32) | (uint64_t)__float_as_uint(v);
}

template <int K, bool LOG>
__global__ __launch_bounds__(kFusedThreads) void k_fused_sweep(
    const float* __restrict__ A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* __restrict__ x,
    const float* __restrict__ ghat, const float* __restrict__ arow, float* __restrict__ partial,
    double* __restrict__ Fpart, uint64_t* __restrict__ gran, int I, int J, SartState* __restrict__ st) {
    constexpr int T = 8 / K;  // rows per tile: T*K float4 = 32 floats per lane per tile
    static_assert(T * K == 8, "tile must hold 8 float4 per lane");

    __shared__ float s_part[4][4][T];  // [tile % 4][compute wave][row]
    __shared__ float s_w[4][T];        // [tile % 4][row]
    __shared__ float s_xch[2048];      // gathered partials of one tile, [j][row]

    if (st->done) return;
    const int epoch = st->epoch;

    const int b = blockIdx.x;
    const int gi = b % I;  // row group (blocks b, b+8, ... share an XCD when I == 8: speed only)
    const int gj = b / I;  // column slab
    const int64_t ntiles = nrows_pad / T;
    const int64_t t_begin = ntiles * gi / I;
    const int64_t nt = ntiles * (gi + 1) / I - t_begin;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t ld4 = ld >> 2;

    if (wave < 4) {
        // ------------------------------ compute waves ------------------------------
        const int64_t col4 = (int64_t)gj * (256 * K) + wave * (64 * K) + lane;
        const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x);
        const float4* __restrict__ a4 = reinterpret_cast<const float4*>(A) + col4;

        float4 xs[K], acc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            xs[k] = x4[col4 + k * 64];
            acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }

        float4 buf[4][T][K];
        auto load_tile = [&](float4(&dst)[T][K], int64_t t) {
            const float4* src = a4 + (t_begin + t) * T * ld4;
#pragma unroll
            for (int r = 0; r < T; ++r)
#pragma unroll
                for (int k = 0; k < K; ++k) dst[r][k] = src[r * ld4 + k * 64];
        };
        if (nt > 0) load_tile(buf[0], 0);
        if (nt > 1) load_tile(buf[1], 1);

        auto step = [&](auto bbc, int64_t t) {
            constexpr int bb = decltype(bbc)::value;
            constexpr int bp = (bb + 2) & 3;  // slot of tile t-2 == slot of tile t+2
            if (t < nt) {
#pragma unroll
                for (int r = 0; r < T; ++r) {
                    float s = 0.f;
#pragma unroll
                    for (int k = 0; k < K; ++k) s += dot4(buf[bb][r][k], xs[k]);
                    s = wave_sum(s);
                    if (lane == 0) s_part[bb][wave][r] = s;
                }
            }
            __syncthreads();
            if (t >= 2 && t - 2 < nt) {
#pragma unroll
                for (int r = 0; r < T; ++r) {
                    const float wr = s_w[bp][r];
#pragma unroll
                    for (int k = 0; k < K; ++k) fma4(acc[k], buf[bp][r][k], wr);
                }
            }
            if (t + 2 < nt) load_tile(buf[bp], t + 2);
        };

        for (int64_t t0 = 0; t0 < nt + 2; t0 += 4) {
            step(std::integral_constant<int, 0>{}, t0 + 0);
            step(std::integral_constant<int, 1>{}, t0 + 1);
            step(std::integral_constant<int, 2>{}, t0 + 2);
            step(std::integral_constant<int, 3>{}, t0 + 3);
        }

        float4* out = reinterpret_cast<float4*>(partial + (int64_t)gi * ld) + col4;
#pragma unroll
        for (int k = 0; k < K; ++k) out[k * 64] = acc[k];
    } else {
        // ------------------------------ exchange wave ------------------------------
        const int n = J * T;
        bool failed = false;
        double F = 0.0;

        auto xstep = [&](auto bbc, int64_t t) {
            constexpr int bb = decltype(bbc)::value;
            constexpr int bw = (bb + 3) & 3;  // slot of tile t-1
            __syncthreads();
            if (t < nt && lane < T) {
                const float s = ((s_part[bb][0][lane] + s_part[bb][1][lane]) + s_part[bb][2][lane]) +
                                s_part[bb][3][lane];
                uint64_t* g = gran + ((t_begin + t) * J + gj) * T + lane;
                __hip_atomic_store(g, make_granule(epoch, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (t >= 1 && t - 1 < nt) {
                const uint64_t* g = gran + (t_begin + t - 1) * J * T;
                if (!failed) {
                    unsigned spins = 0;
                    while (true) {
                        bool ok = true;
                        for (int idx = lane; idx < n; idx += 64) {
                            const uint64_t v = __hip_atomic_load(g + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if ((int)(v >> 32) != epoch) ok = false;
                            s_xch[idx] = __uint_as_float((uint32_t)v);
                        }
                        if (__all(ok)) break;
                        if (++spins > kSpinLimit) {
                            failed = true;
                            if (lane == 0) atomicOr(&st->error, 1);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (lane < T) {
                    float f = 0.f;
                    if (!failed) {
                        for (int jj = 0; jj < J; ++jj) f += s_xch[jj * T + lane];
                    }
                    const int64_t row = (t_begin + t - 1) * T + lane;
                    float w = 0.f;
                    if (row < nrows) {
                        const float a = arow[row];
                        w = LOG ? a * f : a * (ghat[row] - f);
                        if (gj == 0) F += (double)f * (double)f;
                    }
                    s_w[bw][lane] = w;
                }
                __builtin_amdgcn_wave_barrier();
            }
        };

        for (int64_t t0 = 0; t0 < nt + 2; t0 += 4) {
            xstep(std::integral_constant<int, 0>{}, t0 + 0);
            xstep(std::integral_constant<int, 1>{}, t0 + 1);
            xstep(std::integral_constant<int, 2>{}, t0 + 2);
            xstep(std::integral_constant<int, 3>{}, t0 + 3);
        }
        F = wave_sum(F);
        if (lane == 0) Fpart[b] = F;
    }
}

// Geometry chosen by the host for a given padded width: K float4 per lane per row, slab width
// Wc = 1024*K, J = ld / Wc slabs, I = max(1, ncu / J) row groups.
struct FusedGeometry {
    int K, J, I, grid;
};

int fused_pick_k(int64_t ld) {
    // Aim for ~32 slabs (one XCD's CUs share a row group), slabs of 1024..8192 columns.
    for (int K = 1; K <= 8; K *= 2) {
        const int64_t wc = 1024 * (int64_t)K;
        if (ld % wc != 0) return K > 1 ? K / 2 : 0;
        if (ld / wc <= 32) return K;
    }
    return 8;
}

void launch_fused_sweep(bool logmode, int K, const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                        const float* x, const float* ghat, const float* arow, float* partial, double* Fpart,
                        uint64_t* gran, int I, int J, SartState* st, hipStream_t stream) {
    if (K != 1 && K != 2 && K != 4 && K != 8) throw std::runtime_error("fused_sweep: K must be 1, 2, 4 or 8");
    if (ld % (1024 * K) != 0 || ld / (1024 * K) != J)
        throw std::runtime_error("fused_sweep: ld must equal J * 1024 * K");
    if (nrows_pad % (8 / K) != 0) throw std::runtime_error("fused_sweep: padded rows must be a multiple of the tile");
    if (J * (8 / K) > 2048) throw std::runtime_error("fused_sweep: too many slabs for the exchange buffer");
    const dim3 grid((unsigned)(I * J)), block(kFusedThreads);
#define SART_FUSED_CASE(KK)                                                                                        \
    case KK:                                                                                                       \
        if (logmode)                                                                                               \
            hipLaunchKernelGGL((k_fused_sweep<KK, true>), grid, block, 0, stream, A, ld, nrows, nrows_pad, x, ghat, \
                               arow, partial, Fpart, gran, I, J, st);                                              \
        else                                                                                                       \
            hipLaunchKernelGGL((k_fused_sweep<KK, false>), grid, block, 0, stream, A, ld, nrows, nrows_pad, x,      \
                               ghat, arow, partial, Fpart, gran, I, J, st);                                        \
        break;
    switch (K) {
        SART_FUSED_CASE(1)
        SART_FUSED_CASE(2)
        SART_FUSED_CASE(4)
        SART_FUSED_CASE(8)
    }
#undef SART_FUSED_CASE
    check_launch("k_fused_sweep");
}

}  // namespace sart
