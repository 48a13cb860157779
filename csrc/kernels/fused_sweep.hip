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
// (T = TK/K rows, TK float4 per lane) of its group. Per tile it computes the J-th part of each row dot
// and publishes it as an 8-byte {epoch, value} granule with one write-through (sc1) store -- the data
// IS the flag, no fences (cdna_hip_programming.md Guideline 16, recipe R2). A dedicated exchange wave
// gathers the J granules of a tile, sums them in a fixed lane-parallel tree (every workgroup of the
// group obtains a bitwise identical f_r), forms w_r and hands it to the four compute waves through
// LDS; they back-project that tile L steps after reducing it, from a ring of R tiles held in
// registers (tiles t-L .. t in use, t+1 .. t+R-L-1 in flight).
//
// Latency budget per step (one tile): the exchange wave issues the granule loads of tile t-L+2 in
// step t and consumes them in step t+1, so the memory round trip of the gather (2-3 us under full
// streaming load, MI355X_MICROARCH.md price list 'handoff-1to1') overlaps a whole step instead of
// sitting between two barriers.
//
// Correctness does not depend on workgroup placement or dispatch order: every wait is on data
// tagged with this sweep's epoch, every spin is bounded, and a timeout sets SartState::error so
// the host falls back to the two-pass kernels (no hang, no silent wrong answer).
#include "sart_common.hpp"
#include "launchers.hpp"

#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <utility>
#include <vector>

namespace sart {

constexpr int kFusedThreads = 320;  // 4 compute waves + 1 exchange wave
constexpr unsigned kSpinLimit = 1u << 20;
constexpr int kMaxGather = 512;     // J*T granules per tile
constexpr int kGatherRegs = kMaxGather / 64;
constexpr int kRowsGather = 256;    // J*T granules per tile, rows kernel (variant 6)

// diagnostics (dbg & 2): per-workgroup cycle counters, read with fused_debug_stats()
__device__ unsigned long long g_fused_stats[1024 * 8];
// per-tile event trace of the instrumented rows kernel (dbg & 2 with a buffer set by fused_set_trace):
// [block][tile][4] s_memrealtime stamps (100 MHz, one clock for all XCDs): 0 = compute wave 0 published its
// partial, 1 = compute wave 0 got the weight, 2 = exchange stored the granule, 3 = exchange wrote the weight
__device__ unsigned long long* g_fused_trace = nullptr;
__device__ int g_fused_map[1024];  // instrumented builds: gi * 1024 + gj of every block
__device__ long long g_fused_trace_tiles = 0;
__device__ __forceinline__ void trace_stamp(int b, int64_t tile, int ev) {
    if (g_fused_trace != nullptr && tile < g_fused_trace_tiles)
        g_fused_trace[((int64_t)b * g_fused_trace_tiles + tile) * 4 + ev] = __builtin_amdgcn_s_memrealtime();
}

// LDS words polled by other waves of the workgroup (volatile, explicit local address space: ds_read /
// ds_write, counted on lgkmcnt only).
typedef __attribute__((address_space(3))) volatile float lds_vfloat;
typedef __attribute__((address_space(3))) volatile int lds_vint;
typedef int sart_i4v __attribute__((ext_vector_type(4)));
typedef float sart_f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) volatile sart_i4v lds_vi4;
typedef __attribute__((address_space(3))) volatile sart_f4v lds_vf4;

// Row partial of tile u for tile row `lane` (< T) from the compute waves' LDS slot ps: the WPR = 4 / T waves of the
// row, summed in wave order (bitwise the same as reading them one by one). The slot's four flags and four partials are
// each read with ONE 16-byte LDS access: polling four flags in turn put four dependent LDS round trips (queued behind
// the A ring's traffic) into every tile of the publisher and gatherer waves, the per-tile floor of T = 1 sweeps.
// VEC = false: the flags and partials one by one (measured faster for 8-KiB T = 1 slabs, 4.5 %, and chip-wide row
// groups, 7-12 %, whose gatherers then poll the peers' granules later; the 16-byte reads gain 1-5.5 % for XCD-local
// 6 / 7-KiB slabs at T = 1: 150000 voxels 141 -> 148 it/s, profiles/ab_r3_t1_flag4.jsonl)
template <int T, bool VEC>
__device__ __forceinline__ float local_row_partial(lds_vint* s_pflag, lds_vfloat* s_part, int ps, int u, int lane,
                                                   unsigned spin_limit) {
    constexpr int WPR = 4 / T;
    if constexpr (!VEC) {
        float sv = 0.f;
#pragma unroll
        for (int i = 0; i < WPR; ++i) {
            const int wv = lane * WPR + i;
            unsigned spins = 0;
            while (s_pflag[ps * 4 + wv] != u) {
                if (++spins > spin_limit) break;
                __builtin_amdgcn_s_sleep(1);
            }
            asm volatile("" ::: "memory");
            sv += s_part[ps * 4 + wv];
        }
        return sv;
    }
    unsigned spins = 0;
    while (true) {
        const sart_i4v f = *reinterpret_cast<lds_vi4*>(s_pflag + ps * 4);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < WPR; ++i) ok &= f[(lane * WPR + i) & 3] == u;
        if (ok || ++spins > spin_limit) break;  // (the compute waves always publish: the limit cannot trigger)
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    const sart_f4v v = *reinterpret_cast<lds_vf4*>(s_part + ps * 4);
    float sv = 0.f;
#pragma unroll
    for (int i = 0; i < WPR; ++i) sv += v[(lane * WPR + i) & 3];
    return sv;
}

__device__ __forceinline__ uint64_t make_granule(int epoch, float v) {
    return ((uint64_t)(uint32_t)epoch << 32) | (uint64_t)__float_as_uint(v);
}

// ---------------------------------------------------------------------------------------------
// Variant 3 (fallback for widths variant 6 cannot split): in-flight tiles in registers, held tiles in LDS.
//
// Little's law sizing: at ~24.6 GB/s per CU (6.3 TB/s over 256 CUs) and a loaded HBM latency of
// 2-4 us a CU needs ~100 KB of loads in flight. Holding the L tiles that wait for their SART weights
// in registers (variants 0-2) leaves room for only ~2 tiles (64 KB) in flight and caps the sweep at
// ~4 TB/s (the removed variants 0-2). Here each compute wave keeps AH = 4 tiles (4 x 8 KB) of loads in flight in VGPRs; once a
// tile's row partials are reduced it is parked in an LDS ring (NL = L + 1 slots x 32 KB, each wave
// only touches its own 8 KB per slot, so no barrier guards the ring) and read back L steps later for
// the back-projection. 128 KB of loads in flight per CU, 128 KB of LDS.
// ---------------------------------------------------------------------------------------------
template <int K, bool LOG>
__global__ __launch_bounds__(kFusedThreads) void k_fused_sweep_lds(
    const float* __restrict__ A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* __restrict__ x,
    const float* __restrict__ ghat, const float* __restrict__ arow, float* __restrict__ partial,
    double* __restrict__ Fpart, uint64_t* __restrict__ gran, int I, int J, SartState* __restrict__ st, int dbg) {
    constexpr int TK = 8;       // float4 per lane per tile (8 KB per wave, 32 KB per workgroup)
    constexpr int T = TK / K;   // rows per tile
    constexpr int L = 3;        // back-projection lag (steps)
    constexpr int NL = L + 1;   // LDS ring slots
    constexpr int AH = 4;       // tiles in flight
    static_assert(T * K == TK, "tile must be whole rows");

    // all LDS in the one dynamic region (16-B aligned base, cdna_hip_programming.md Guideline 17):
    // [NL][4 waves][TK][64 lanes] float4 ring, then s_part[4][4][8] and s_w[4][8] floats
    extern __shared__ __attribute__((aligned(16))) float4 s_ring[];
    float(*s_part)[4][8] = reinterpret_cast<float(*)[4][8]>(s_ring + NL * 4 * TK * 64);
    float(*s_w)[8] = reinterpret_cast<float(*)[8]>(reinterpret_cast<float*>(s_ring + NL * 4 * TK * 64) + 128);

    if (st->done) return;
    const int epoch = st->epoch;

    const int b = blockIdx.x;
    const int gi = b % I;
    const int gj = b / I;
    const int64_t ntiles = nrows_pad / T;
    const int64_t t_begin = ntiles * gi / I;
    const int64_t nt = ntiles * (gi + 1) / I - t_begin;
    constexpr int UNR = 4;  // == AH (register slots are indexed statically)
    const int64_t nsteps = (nt + L + UNR - 1) / UNR * UNR;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t ld4 = ld >> 2;

    if (wave < 4) {
        const int64_t col4 = (int64_t)gj * (256 * K) + wave * (64 * K) + lane;
        const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x);
        const float4* __restrict__ a4 = reinterpret_cast<const float4*>(A) + col4;
        float4* ring = s_ring + (wave * TK) * 64 + lane;  // + slot * (4 * TK * 64) + q * 64

        // Two-level back-projection sums like variant 6 at T = 1: a lane's chain would otherwise sum all nt * T rows of
        // its group (the chip-wide fallback at 512 x 524288: 1.29x the two-pass error); folded into acc2 every fpass
        // passes of UNR steps, ~sqrt(nt T) rows per chain
        float4 xs[K], acc[K], acc2[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            xs[k] = x4[col4 + k * 64];
            acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            acc2[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        int64_t fpass = (int64_t)__builtin_ceilf(__builtin_sqrtf((float)(nt * T)) / (float)(UNR * T));
        if (fpass < 1) fpass = 1;
        int64_t fcount = 0;
        float4 fl[AH][TK];
        const int64_t tlast = ntiles - 1 - t_begin;  // unconditional clamped loads: see k_fused_sweep_rows
        auto load_tile = [&](float4(&dst)[TK], int64_t t) {
            const float4* src = a4 + (t_begin + (t < tlast ? t : tlast)) * T * ld4;
#pragma unroll
            for (int r = 0; r < T; ++r)
#pragma unroll
                for (int k = 0; k < K; ++k) dst[r * K + k] = load_stream(src + r * ld4 + k * 64);
        };
#pragma unroll
        for (int i = 0; i < AH; ++i) load_tile(fl[i], i);

        auto step = [&](auto bbc, int64_t t) {
            constexpr int bb = decltype(bbc)::value;  // register slot of tile t (t % AH)
            if (t < nt) {
#pragma unroll
                for (int r = 0; r < T; ++r) {
                    float s = 0.f;
#pragma unroll
                    for (int k = 0; k < K; ++k) s += dot4(fl[bb][r * K + k], xs[k]);
                    s = wave_sum(s);
                    if (lane == 0) s_part[t & 3][wave][r] = s;
                }
                float4* slot = ring + (int)(t % NL) * (4 * TK * 64);
#pragma unroll
                for (int q = 0; q < TK; ++q) slot[q * 64] = fl[bb][q];
            }
            load_tile(fl[bb], t + AH);
            __syncthreads();
            if (t >= L && t - L < nt) {
                const int64_t u = t - L;
                const float4* slot = ring + (int)(u % NL) * (4 * TK * 64);
                const int ws = (int)(u & 3);
#pragma unroll
                for (int r = 0; r < T; ++r) {
                    const float wr = s_w[ws][r];
#pragma unroll
                    for (int k = 0; k < K; ++k) fma4(acc[k], slot[(r * K + k) * 64], wr);
                }
            }
        };

        for (int64_t t0 = 0; t0 < nsteps; t0 += UNR) {
            step(std::integral_constant<int, 0>{}, t0 + 0);
            step(std::integral_constant<int, 1>{}, t0 + 1);
            step(std::integral_constant<int, 2>{}, t0 + 2);
            step(std::integral_constant<int, 3>{}, t0 + 3);
            if (++fcount == fpass) {  // registers only
                fcount = 0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    add4(acc2[k], acc[k]);
                    acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
        float4* out = reinterpret_cast<float4*>(partial + (int64_t)gi * ld) + col4;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            add4(acc[k], acc2[k]);
            out[k * 64] = acc[k];
        }
    } else {
        const int n = J * T;
        bool failed = false;
        double F = 0.0;
        uint64_t pv[2][kGatherRegs];

        // Polls are issued unconditionally at clamped addresses (tile in [0, ntiles), granule < n; lanes past
        // n re-read granule n - 1 and are masked when summing), so the compiler counts the polls in flight
        // instead of draining them (see load_tile in k_fused_sweep_rows).
        const int64_t ulast = ntiles - 1 - t_begin;
        auto issue_poll = [&](uint64_t(&dst)[kGatherRegs], int64_t u) {
            const int64_t uc = u < 0 ? 0 : (u < ulast ? u : ulast);
            const uint64_t* g = gran + (t_begin + uc) * (int64_t)n;
#pragma unroll
            for (int m = 0; m < kGatherRegs; ++m) {
                const int idx = lane + 64 * m;
                dst[m] = __hip_atomic_load(g + (idx < n ? idx : n - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        auto finish_tile = [&](uint64_t(&v)[kGatherRegs], int64_t u) {
            if (!failed) {
                unsigned spins = 0;
                while (true) {
                    bool ok = true;
#pragma unroll
                    for (int m = 0; m < kGatherRegs; ++m) ok &= ((int)(v[m] >> 32) == epoch);
                    if (__all(ok)) break;
                    if (++spins > kSpinLimit) {
                        failed = true;
                        if (lane == 0) atomicOr(&st->error, 1);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    issue_poll(v, u);
                }
            }
            float s = 0.f;
            if (!failed) {
#pragma unroll
                for (int m = 0; m < kGatherRegs; ++m)
                    s += (lane + 64 * m < n) ? __uint_as_float((uint32_t)v[m]) : 0.f;
            }
#pragma unroll
            for (int off = T; off < 64; off <<= 1) s += __shfl_xor(s, off, kWave);
            if (lane < T) {
                const int64_t row = (t_begin + u) * T + lane;
                float w = 0.f;
                if (row < nrows) {
                    const float a = arow[row];
                    w = LOG ? a * s : a * (ghat[row] - s);
                    if (gj == 0) F += (double)s * (double)s;
                }
                s_w[u & 3][lane] = w;
            }
        };
        auto xstep = [&](auto pc, int64_t t) {
            constexpr int p = decltype(pc)::value;
            __syncthreads();
            if (dbg & 1) {  // ablation: no inter-workgroup exchange (timing diagnostics only)
                if (lane < T) s_w[(t + 1) & 3][lane] = 0.f;
                return;
            }
            if (t < nt && lane < T) {
                const int ps = (int)(t & 3);
                const float s = ((s_part[ps][0][lane] + s_part[ps][1][lane]) + s_part[ps][2][lane]) +
                                s_part[ps][3][lane];
                uint64_t* g = gran + ((t_begin + t) * J + gj) * T + lane;
                __hip_atomic_store(g, make_granule(epoch, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const int64_t un = t - L + 2;
            issue_poll(pv[p], un);
            const int64_t uc = t - L + 1;
            if (uc >= 0 && uc < nt) finish_tile(pv[p ^ 1], uc);
        };
        for (int64_t t0 = 0; t0 < nsteps; t0 += 2) {
            xstep(std::integral_constant<int, 0>{}, t0);
            xstep(std::integral_constant<int, 1>{}, t0 + 1);
        }
        F = wave_sum(F);
        if (lane == 0) Fpart[b] = F;
    }
}

// ---------------------------------------------------------------------------------------------
// Variant 6 (default): "split rows" + barrier-free LDS hand-offs + XCD-local row groups.
//
// Measured on MI355X (tools/probe.py, exchange disabled): the register/LDS pipeline of variant 3
// streams at the HBM roof (6.2 TB/s) only when each wave performs ONE full-wave reduction per step;
// with T rows per wave per step the T dependent shuffle reductions dominate. Here every compute wave
// owns a different row of the 4-row tile over the same 2048-column slab (8 float4 per lane), so a
// step costs one reduction per wave and no cross-wave partial sum.
// The per-step __syncthreads of variant 3 (and the removed 0-2) coupled the compute waves to every jitter of the
// inter-workgroup exchange; here compute and exchange waves hand off through LDS words tagged with
// the tile index (written data-then-flag by one wave; LDS serves a wave's requests in order), so the
// compute waves block only when the weight they need at step t (tile t - L) is not there yet.
// ---------------------------------------------------------------------------------------------
// XL (variant 6): row groups are formed from workgroups that run on the same XCD, determined at run
// time (HW_REG_XCC_ID + a per-XCD ticket), so granules are plain stores that stay in the XCD's shared
// L2 and polls are L2 round trips instead of memory-side round trips. Correctness still rests only on
// the epoch tags; an unexpected placement (more tickets than slots on an XCD) sets SartState::error and
// the host falls back.
// T (rows per tile) trades row-group width against hand-off volume: the 4 compute waves cover T rows x
// (4 / T) sub-slabs of 2048 columns, so a workgroup's slab is 8192 / T columns and a row's dot is split
// over J = ld * T / 8192 workgroups. T = 1 needs only J granules per tile (8 peers at ld = 65536 instead
// of 32), so a late peer delays fewer workgroups; the waves of one row are summed by the exchange wave.
// SCHED sets the pipeline budget. A hand-off into a CU that streams A costs ~3 us (the poll waits in the
// consumer CU's own vector memory queue: MI355X_MICROARCH.md price list, handoff-1to1 'L->L'), more than
// two 1.3 us steps, so the exchange wave keeps PQ polls in flight (poll tile u - PD in exchange step u,
// finish tile u - PD - PQ + 1); the weights are consumed L >= PD + PQ steps after the reduction:
//   SCHED  L  AH(in flight) x slab  PD PQ
//     0    3  4             VGPR    1  2
//     1    4  4             LDS     1  3     (the newest tile stays in VGPRs one step before parking)
//     2    4  4             LDS     2  2
//     3    3  5             LDS     1  2
//     4    4  4             LDS     2  2     + split exchange: a publisher wave stores, a gatherer wave polls
// Schedule 4 is the default: 6 % faster than 2 at 64k x 64k and 4-5 % at 16k-wide shapes
// (profiles/probe_r1_split_exchange.jsonl); the per-tile trace shows the publication delay of a granule
// falling from 1.7 us to 0.16 us (profiles/fused_trace_r1_split_exchange.jsonl). Schedule 2 was 5-8 %
// faster than 0 (profiles/probe_r1_sched.jsonl). Compute waves storing their own granules measured 8-10 %
// slower than 2: their stores join the vmcnt queue of their streaming loads.
// (LDS x slab: T >= 2 only.) Scalar-memory (s_load glc) polls were measured and are no faster under load:
// an s_load round trip to L2 costs ~1.2 us while the chip streams.
// Register tiles of the v6 compute waves by RTM storage type and lane width. A lane owns CPL consecutive
// columns per k-slot: one 16-byte fp32 load (CPL 4), one 8-byte load of 4 bf16 (CPL 4), or one 16-byte load
// of 8 bf16 (CPL 8, "wide"), widened to H = CPL / 4 float4 where the tile is consumed (row dot and
// back-projection); the LDS ring parks the raw storage type, the x slab and every sum stay fp32.
// Narrow bf16 tiles carry half the bytes of an fp32 tile per instruction and per pipeline step, so at the
// fp32 kernel's step rate they stream half the bytes (487 it/s = 4.2 TB/s at 64k x 64k); wide bf16 tiles
// carry the fp32 tile's 8 KB per wave per step (twice the columns per workgroup: slab 16384 / T).
template <typename AT, int CPL = 4>
struct FusedTile;

template <>
struct FusedTile<float, 4> {
    using R = float4;
    static constexpr int H = 1;
    __device__ __forceinline__ static R load(const R* p) { return load_stream(p); }
    __device__ __forceinline__ static void widen(const R v, float4 (&o)[1]) { o[0] = v; }
};

typedef unsigned sart_u2v __attribute__((ext_vector_type(2)));
template <>
struct FusedTile<bf16_t, 4> {
    using R = uint2;
    static constexpr int H = 1;
    __device__ __forceinline__ static R load(const R* p) {
#if SART_STREAM_NT
        const sart_u2v v = __builtin_nontemporal_load(reinterpret_cast<const sart_u2v*>(p));
        return make_uint2(v.x, v.y);
#else
        return *p;
#endif
    }
    __device__ __forceinline__ static void widen(const R v, float4 (&o)[1]) { o[0] = bf16x4_to_f4(v.x, v.y); }
};

template <>
struct FusedTile<bf16_t, 8> {
    using R = uint4;
    static constexpr int H = 2;
    __device__ __forceinline__ static R load(const R* p) {
#if SART_STREAM_NT
        const sart_u4v v = __builtin_nontemporal_load(reinterpret_cast<const sart_u4v*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
#else
        return *p;
#endif
    }
    __device__ __forceinline__ static void widen(const R v, float4 (&o)[2]) {
        o[0] = bf16x4_to_f4(v.x, v.y);
        o[1] = bf16x4_to_f4(v.z, v.w);
    }
};

// bf16 row dots on v_dot2c_f32_bf16: the x slab is held in LDS as hi = rne(x) and lo ~ x - hi bf16 pairs (the
// fp32 slab's bytes), so a dword of the tile (two bf16) meets its two x columns in two dot2 instructions with no
// conversion: 1 VALU op per element instead of a shift / mask plus half a packed FMA. Products of bf16 are exact
// in fp32 (dot2 measured unbiased, <= 0.75 ulp: tools/dot2_probe.hip).
// hi + lo holds x to 2^-17. With lo rounded to nearest, that representation error is a deterministic function of
// x, so equal or clustered x values (a clamped cold start) bias the row dot coherently: 2^-18 of F, which the
// cancellation in ghat - F amplified to 3x the fp32 self-check error at 512k x 256k. lo is therefore rounded
// stochastically (a hash of the element index picks the rounding point; deterministic, zero mean, independent
// across columns), which makes the dot's x error average out like fp32 rounding.
typedef __bf16 sart_bf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot2_bf16(unsigned a, unsigned b, float c) {
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(sart_bf2, a), __builtin_bit_cast(sart_bf2, b), c, false);
}
__device__ __forceinline__ unsigned sr_bf16_bits(float r, uint32_t key) {  // stochastic rounding of |r| to bf16
    uint32_t h = key * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    return (__float_as_uint(r) + (h & 0xffffu)) >> 16;  // magnitude rounds up with probability = the dropped part
}
__device__ __forceinline__ void split_pair(float a, float b, uint32_t key, unsigned& hi, unsigned& lo) {
    const __bf16 ha = (__bf16)a, hb = (__bf16)b;
    hi = (unsigned)__builtin_bit_cast(unsigned short, ha) | ((unsigned)__builtin_bit_cast(unsigned short, hb) << 16);
    lo = sr_bf16_bits(a - (float)ha, key) | (sr_bf16_bits(b - (float)hb, key + 1) << 16);
}

// Row-dot reductions on DPP instead of ds_bpermute (__shfl_xor): the 6 bpermutes of a full-wave sum are LDS
// round trips that queue behind the ring's LDS traffic, once per tile in every compute wave and in the gatherer.
// Within each 16-lane row: quad_perm xor 1 / xor 2, then row_ror 4 / 8 (rotations keep lane % 4), so every lane
// holds the sum of its row's lanes of the same class lane % T; the four rows are added through v_readlane.
// Fixed order: bitwise reproducible. The result is valid in lanes < T.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int T>
__device__ __forceinline__ float class_sum_dpp(float v, int lane) {
    static_assert(T == 1 || T == 2 || T == 4, "lane classes");
    if constexpr (T == 1) v += dpp_f<0xB1>(v);  // quad_perm [1, 0, 3, 2]
    if constexpr (T <= 2) v += dpp_f<0x4E>(v);  // quad_perm [2, 3, 0, 1]
    v += dpp_f<0x124>(v);                       // row_ror 4
    v += dpp_f<0x128>(v);                       // row_ror 8
    float r = 0.f;
#pragma unroll
    for (int c = 0; c < T; ++c) {
        const float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), c)) +
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), c + 16)) +
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), c + 32)) +
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), c + 48));
        r = lane == c ? t : r;
    }
    return r;
}

// Register tile slots of the fp32 x-slab-in-VGPR schedules (0, 5, 8): >= 32 KiB of A in flight per wave
// (kw 9: 3 slots, the most the 256 VGPRs of a wave hold next to the x slab and the two accumulator sets)
constexpr int t1_reg_slots(int kw) { return kw >= 9 ? 3 : (kw == 8 ? 4 : (kw == 7 ? 5 : (kw == 6 ? 6 : 7))); }
template <typename AT>
constexpr bool BF_T() { return !std::is_same<AT, float>::value; }

// Schedules with a separate publisher wave (the split exchange)
constexpr bool sched_split(int sched) { return sched >= 4 && sched <= 8; }

template <bool LOG, bool XL, bool DIAG, int T, int SCHED, typename AT = float, int CPL = 4, int KW = 8>
__global__ __launch_bounds__(sched_split(SCHED) ? kFusedThreads + 64 : kFusedThreads) void k_fused_sweep_rows(
    const AT* __restrict__ A, int64_t ld, int64_t nrows, int64_t nrows_pad, const float* __restrict__ x,
    const float* __restrict__ ghat, const float* __restrict__ arow, float* __restrict__ partial,
    double* __restrict__ Fpart, uint64_t* __restrict__ gran, int I, int J, SartState* __restrict__ st, int dbg,
    unsigned* __restrict__ xcnt, int64_t chain_tiles) {
    static_assert(T == 1 || T == 2 || T == 4, "rows per tile");
    // KW: lane-vectors per lane per row (8: one wave covers 2048 fp32 columns; 9 / 7 / 6 / 5 give slabs of 9 ... 5 KiB
    // columns, so widths whose 8-KiB slab count does not fit an XCD's 32 CUs still use most of them; 9 and 5 at T = 1)
    static_assert(KW >= 5 && KW <= 9, "lane-vectors per lane");
    static_assert(KW != 9 || (T == 1 && !BF_T<AT>()), "9-KiB slabs: fp32 T = 1 only (register and LDS budget)");
    constexpr int WPR = 4 / T;   // compute waves per row (each on its own 2048-column sub-slab)
    constexpr int D = SCHED == 7 ? 2 : ((SCHED == 1 || SCHED == 2 || SCHED == 4 || SCHED == 6) ? 1 : 0);  // steps a reduced tile stays in VGPRs
    constexpr bool XS_LDS = (SCHED >= 1 && SCHED <= 4) || SCHED == 6 || SCHED == 7;  // x slab in LDS instead of VGPRs
    static_assert(!XS_LDS || T >= 2, "the LDS holds the x slab only for T >= 2");
    // wave 4 publishes granules, wave 5 gathers (no shared vmcnt queue); schedule 5 = the split exchange with
    // the x slab in VGPRs and schedule 0's lag (T = 1, whose x slab does not fit the LDS next to the ring)
    // schedule 6 = the split exchange for wide bf16 tiles at T = 2 (x slab in LDS, 3-slot ring, L = 3: a 4-slot
    // ring and the 32 KB x slab of two sub-slabs would exceed the 160 KB of LDS by the hand-off words)
    // schedule 7 = schedule 6 with the lag of schedule 4 (L = 4, PD = PQ = 2) in the same 3-slot ring: a reduced
    // tile stays in VGPRs two steps before parking (D = 2), so 3 of the 5 register slots are in flight. At
    // 65536 x 262144 bf16 schedule 6 spent 14 % of its sweep on the hand-off (exchange-off ablation, L = 3)
    // and 3 tiles x 8 KB per wave still cover the HBM latency (tools/fused_ablation.py)
    // (the same trade at T = 1, L = 4 in schedule 5's 4-slot ring with D = 1, measured equal to schedule 5 at
    // 70000 ... 262144 columns and was removed: profiles/ablation_r2_t1_sched5_vs_8.jsonl)
    constexpr bool SPLIT = sched_split(SCHED);
    constexpr int NTHR = SPLIT ? kFusedThreads + 64 : kFusedThreads;
    constexpr bool BF = !std::is_same<AT, float>::value;
    constexpr int H = CPL / 4;  // float4 per lane per k-slot (2: wide bf16 tiles)
    constexpr bool DOT2 = BF && XS_LDS;  // bf16 row dots on dot2 with the x slab as hi / lo bf16 pairs in LDS
    static_assert(CPL == 4 || (BF && CPL == 8 && XS_LDS), "wide tiles: bf16 storage, x slab in LDS");
    // bf16 tiles are parked raw in the LDS ring (16 KB per slot), so 8 slots fit in the 128 KB of the fp32
    // ring. With T = 1 (schedule 0) the bf16 sweep keeps 4 polls in flight and lags the back-projection by
    // L = PD + PQ = 5 steps: 12.5 -> 13.2 it/s at 512k x 256k; with T = 4 (schedule 4) the deeper lag
    // measured 3 % slower than the fp32 lag (458 vs 473 it/s at 64k x 64k), so it is kept there.
    constexpr bool DEEP = BF && SCHED == 0;
    constexpr int PD = (SCHED == 2 || SCHED == 4 || SCHED == 7) ? 2 : 1;   // exchange step u polls tile u - PD
    // schedule 8 = schedule 5 with 3 polls in flight and a 4-step lag in a 5-slot ring (chip-wide row groups, whose
    // granules make memory-side round trips; kw 6 / 7 only: five 32-KiB kw 8 slots do not fit the LDS)
    // (the kw 8 analogue, a 4-step lag in the 4-slot ring with a reduced tile held one step in VGPRs, measured 4-5 %
    // slower than schedule 5 at 524288 / 1048576 voxels: profiles/ab_r3_cw_sched9_negative.jsonl)
    constexpr int PQ = DEEP ? 4 : ((SCHED == 1 || SCHED == 8) ? 3 : 2);  // polls in flight (finishes tile u - PD - PQ + 1)
    constexpr int L = DEEP ? PD + PQ : (SCHED == 6 ? 3 : ((SCHED == 7 || SCHED == 8) ? 4 : 3 + D));  // back-projection lag
    static_assert(SCHED != 8 || (KW <= 7 && T == 1 && !BF), "schedule 8: fp32 T = 1 slabs of kw <= 7");
    static_assert(L >= PD + PQ, "the weights must be ready one step before they are used");
    constexpr int NL = (BF && CPL == 4) ? 8 : ((SCHED == 6 || SCHED == 7) ? 3 : (SCHED == 8 ? 5 : 4));  // LDS ring slots (32 KB fp32 or wide bf16 / 16 KB narrow bf16)
    static_assert(L <= NL + D - 1, "a parked tile must be back-projected before its ring slot is reused");
    // register tile slots per wave (8 KB fp32 / 4 KB bf16 each): AH in flight + D held. bf16: 6-7 tiles of
    // 8-byte loads in flight (<= 56 loads, inside the 6-bit vmcnt range); 8 slots with the x slab in LDS
    // measured no faster at 64k x 64k
    // wide bf16 tiles: 8 KB per wave like fp32, 5 slots (4 in flight + 1 held), accumulators 2 x 32 VGPRs
    // fp32 tiles with the x slab in VGPRs (T = 1): AH = RS tiles in flight, sized so that a wave keeps >= 32 KiB of A in
    // flight at every slab width (kw 8: 4, 7: 5, 6: 6, 5: 7 tiles; kw 9: 3, the register limit). Against 4 tiles at every
    // kw this measured +0.5-1.4 % (profiles/ab_r3_t1_ring_depth.jsonl): the narrow slabs' ~0.85 us step floor is the
    // per-step hand-off chain, not loads in flight (see local_row_partial)
    constexpr int RS = XS_LDS ? ((BF && CPL == 4) ? 7 : 5) : (BF ? 7 : t1_reg_slots(KW));
    using FT = FusedTile<AT, CPL>;
    using RT = typename FT::R;
    constexpr int AH = RS - D;   // tiles in flight per wave
    static_assert(L >= PD + 2, "the weights must be ready one step before they are used");
    constexpr int NS = 8;        // LDS hand-off slots
    // Two-level back-projection sums (T = 1): with T = 1 every wave owns its own columns, so a lane's
    // accumulators would sum ALL P / I rows of its group in one fp32 chain (T >= 2 split a group's rows over T
    // waves). Measured at 65536 x 262144 bf16: 2.4x the two-pass kernels' error after one iteration, 26x at
    // 524288 rows. Every ~chain_tiles tiles (host: ~sqrt of the group's tiles) the chain is folded into a second
    // register set acc2 and restarts, so no chain is longer than ~2 sqrt(P / I) terms. (Splitting the group
    // into separately drained segments deadlocks: the exchange wave finishes tile u only after the compute
    // waves published u + PD + PQ - 1.)
    constexpr bool FOLD = (T == 1);
    // Segmented back-projection sums (split schedules, T >= 2): a wave's chain sums one row per tile, P / (T I)
    // rows per group (32768 at 512k x 256k with wide bf16 tiles at T = 2, whose registers have no room for a
    // fold set). With chain_tiles > 0 the group's tiles run in segments of chain_tiles (a multiple of RS): at
    // a segment's end the pipeline drains, every wave stores its sums to its own partial block
    // ((seg * T + row) * I + gi) and the chain restarts. Only split schedules: their gatherer does not need the
    // compute waves' next tiles to finish the current ones (it skips its pacing wait on a segment's first
    // PD + PQ - 1 tiles), so the drain cannot deadlock. chain_tiles = 0: one chain, LDS combine of the T rows.
    constexpr bool SEG = SPLIT && T >= 2;
    constexpr bool FLAG4 = XL && T == 1 && !BF && KW <= 7;  // one 16-byte LDS read of a slot's flags (local_row_partial)
    const bool seg_on = SEG && chain_tiles > 0;

    extern __shared__ __attribute__((aligned(16))) float4 s_ring[];  // [NL][4][KW][64] of RT (128 KB)
    float4* s_xs = s_ring + NL * 4 * KW * 64 * sizeof(RT) / sizeof(float4);  // [WPR][KW][H][64] if XS_LDS
    float* s_small = reinterpret_cast<float*>(s_xs + (XS_LDS ? WPR * KW * H * 64 : 0));
    // Hand-off words: volatile through explicit LDS (address_space(3)) pointers. Through generic pointers
    // the compiler keeps volatile accesses as FLAT instructions, which count on vmcnt too, so every flag
    // poll waited vmcnt(0) and drained the compute waves' in-flight A tiles.
    lds_vfloat* s_part = (lds_vfloat*)s_small;                                // [NS][4]
    lds_vfloat* s_w = (lds_vfloat*)(s_small + NS * 4);                        // [NS][4]
    lds_vint* s_pflag = (lds_vint*)(s_small + 2 * NS * 4);                    // [NS][4]
    lds_vint* s_wflag = s_pflag + NS * 4;                                     // [NS]
    lds_vint* s_tick = s_wflag + NS;                                          // [2]

    if (st->done) return;
    const int epoch = st->epoch;
    const int b = blockIdx.x;
    int gi = b % I;
    int gj = b / I;
    if constexpr (!XL) {
        // Chip-wide groups: the dispatcher deals workgroups to the XCDs round-robin (b % 8), so with gi = b % I a
        // group lived on gcd(I, 8) ... 8 / gcd(I, 8) XCDs: I = 4 put each group of J = 57 ... 61 slabs on 2 XCDs
        // (4.3-4.5 TB/s), I = 6 on 4 (4.9-5.3), odd I on all 8 (5.5-6.2 TB/s, profiles/cw_r4_sweep.jsonl). Number
        // the workgroups XCD by XCD (p = the workgroups of lower XCDs + b / 8) and deal p round-robin to the groups:
        // every group gets ~J / 8 slabs on every XCD whatever I is. (dbg & 8: the old b % I map, A/B runs.)
        if (!(dbg & 8)) {
            const int grid = I * J, x = b & 7;
            const int p = x * (grid >> 3) + (x < (grid & 7) ? x : (grid & 7)) + (b >> 3);
            gi = p % I;
            gj = p / I;
        }
    }
    if constexpr (XL) {
        if (threadIdx.x == 0) {
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
            s_tick[0] = (int)(xcc & 7u);
            s_tick[1] = (int)atomicAdd(&xcnt[xcc & 7u], 1u);
        }
        __syncthreads();
        const int xcc = s_tick[0], ticket = s_tick[1];
        const int per_xcd = I / 8;  // row groups per XCD
        if (ticket >= per_xcd * J) {
            if (threadIdx.x == 0) atomicOr(&st->error, 4);
            return;  // uniform for the workgroup: its peers time out and the host falls back
        }
        if (!(dbg & 4)) {  // (dbg & 4: keep the blockIdx mapping -- timing diagnostics only)
            gi = xcc * per_xcd + ticket / J;
            gj = ticket % J;
        }
    }
    const int64_t ntiles = nrows_pad / T;
    const int64_t t_begin = ntiles * gi / I;
    const int64_t nt = ntiles * (gi + 1) / I - t_begin;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t ld4 = ld >> (CPL == 8 ? 3 : 2);  // row length in tile vectors (RT)
    // Granule row of a tile: J entries (T = 1 for chip-wide groups), padded there to whole 128-byte lines (16
    // granules) so that no line holds granules of two tiles: the J writers of tile u + 1 (other XCDs) then never
    // store into a line the gatherers of tile u are still re-polling through memory (fused_granules sizes the
    // buffer; dbg & 16: unpadded, A/B runs).
    // XCD-local groups keep unpadded rows unless dbg & 32 (A/B runs: SART_FUSED_GPAD=2).
    const int Jg = ((XL && !(dbg & 32)) || (dbg & 16)) ? J : ((J + 15) & ~15);
    if (DIAG && threadIdx.x == 0 && b < 1024) g_fused_map[b] = gi * 1024 + gj;

    for (int i = threadIdx.x; i < NS * 4 + NS; i += NTHR) s_pflag[i] = -1;
    if constexpr (DOT2) {
        // lane-vector lv = (sub * KW + k) * 64 + lane holds CPL columns; LDS: H = 2: [(sub KW + k) 2 + {hi, lo}]
        // [lane] of uint4 (8 bf16 each); H = 1: [(sub KW + k)][lane] of uint4 {hi (4 bf16), lo (4 bf16)}
        const float4* xsrc = reinterpret_cast<const float4*>(x) + (int64_t)gj * (64 * KW * WPR) * H;
        uint4* xd = reinterpret_cast<uint4*>(s_xs);
        for (int lv = threadIdx.x; lv < WPR * KW * 64; lv += NTHR) {
            unsigned hi[2 * H], lo[2 * H];
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const float4 v = xsrc[lv * H + h];
                const uint32_t key = (uint32_t)(((int64_t)gj * (WPR * KW * 64) + lv) * CPL + 4 * h);  // column
                split_pair(v.x, v.y, key, hi[2 * h], lo[2 * h]);
                split_pair(v.z, v.w, key + 2, hi[2 * h + 1], lo[2 * h + 1]);
            }
            if constexpr (H == 2) {
                xd[((lv >> 6) * 2 + 0) * 64 + (lv & 63)] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
                xd[((lv >> 6) * 2 + 1) * 64 + (lv & 63)] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
            } else {
                xd[lv] = make_uint4(hi[0], hi[1], lo[0], lo[1]);
            }
        }
    } else if constexpr (XS_LDS) {
        // global float4 i of the slab = lane-vector i / H, half i % H; LDS [(sub * KW + k) * H + h][lane] so a
        // wave reads 64 consecutive float4 per (k, h)
        const float4* xsrc = reinterpret_cast<const float4*>(x) + (int64_t)gj * (64 * KW * WPR) * H;
        if constexpr (H == 1) {
            for (int i = threadIdx.x; i < WPR * KW * 64; i += NTHR) s_xs[i] = xsrc[i];
        } else {
            for (int i = threadIdx.x; i < WPR * KW * 64 * H; i += NTHR) {
                const int lv = i / H, h = i % H;  // lv = (sub * KW + k) * 64 + lane
                s_xs[((lv >> 6) * H + h) * 64 + (lv & 63)] = xsrc[i];
            }
        }
    }
    __syncthreads();

    if (wave < 4) {
        const int wrow = wave / WPR, wsub = wave % WPR;
        const int64_t slab4 = (int64_t)gj * (64 * KW * WPR);                // first lane-vector of the slab
        const int64_t col4 = slab4 + wsub * (64 * KW) + lane;              // + k * 64 (CPL columns each)
        const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x);
        const RT* __restrict__ a4 = reinterpret_cast<const RT*>(A) + col4 + (int64_t)wrow * ld4;
        RT* ring = reinterpret_cast<RT*>(s_ring) + (wave * KW) * 64 + lane;  // tiles parked in storage type
        float4 xs[XS_LDS ? 1 : KW], acc[KW][H], acc2[FOLD ? KW : 1];
        const float4* xl = s_xs + wsub * (KW * H * 64) + lane;             // + (k * H + h) * 64
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            if constexpr (!XS_LDS) xs[k] = x4[col4 + k * 64];
#pragma unroll
            for (int h = 0; h < H; ++h) acc[k][h] = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (FOLD) acc2[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        RT fl[RS][KW];
        // Tile loads are issued unconditionally, clamped to the last tile of the matrix (past the group's
        // end they re-read valid rows that nobody uses). A guarded load makes the vmcnt bookkeeping depend
        // on the path, and the compiler then waits for EVERY load in flight wherever a tile is consumed,
        // which collapses the AH-tile pipeline to one tile.
        const int64_t tlast = ntiles - 1 - t_begin;
        int64_t lo = 0, hi = nt;  // tiles of the current segment (SEG) or of the whole group
        auto load_tile = [&](RT(&dst)[KW], int64_t t) {
            const int64_t tc = t < tlast ? t : tlast;
            const RT* src = a4 + (t_begin + tc) * T * ld4;
#pragma unroll
            for (int k = 0; k < KW; ++k) dst[k] = FT::load(src + k * 64);
        };
#pragma unroll
        for (int i = 0; i < AH; ++i) load_tile(fl[i], i);
        bool stuck = false;
        unsigned long long stall = 0, nstall = 0;

        auto park = [&](RT(&src)[KW], int64_t t) {
            RT* slot = ring + (int)(t % NL) * (4 * KW * 64);
#pragma unroll
            for (int k = 0; k < KW; ++k) slot[k * 64] = src[k];
        };
        auto step = [&](auto bbc, int64_t t) {
            constexpr int bb = decltype(bbc)::value;        // register slot of tile t (t % RS)
            constexpr int bp = (bb + RS - D) % RS;          // register slot of tile t - D
            if (t < hi) {
                float s = 0.f;
                if constexpr (DOT2) {
                    const uint4* xb = reinterpret_cast<const uint4*>(xl);
                    float sh = 0.f, sl = 0.f;  // hi and lo chains
#pragma unroll
                    for (int k = 0; k < KW; ++k) {
                        const RT a = fl[bb][k];
                        if constexpr (H == 2) {
                            const uint4 xh = xb[(k * 2 + 0) * 64], xo = xb[(k * 2 + 1) * 64];
                            sh = dot2_bf16(a.x, xh.x, sh), sl = dot2_bf16(a.x, xo.x, sl);
                            sh = dot2_bf16(a.y, xh.y, sh), sl = dot2_bf16(a.y, xo.y, sl);
                            sh = dot2_bf16(a.z, xh.z, sh), sl = dot2_bf16(a.z, xo.z, sl);
                            sh = dot2_bf16(a.w, xh.w, sh), sl = dot2_bf16(a.w, xo.w, sl);
                        } else {
                            const uint4 v = xb[k * 64];  // {hi pair 0, hi pair 1, lo pair 0, lo pair 1}
                            sh = dot2_bf16(a.x, v.x, sh), sl = dot2_bf16(a.x, v.z, sl);
                            sh = dot2_bf16(a.y, v.y, sh), sl = dot2_bf16(a.y, v.w, sl);
                        }
                    }
                    s = sh + sl;
                } else {
#pragma unroll
                    for (int k = 0; k < KW; ++k) {
                        float4 w[H];
                        FT::widen(fl[bb][k], w);
#pragma unroll
                        for (int h = 0; h < H; ++h) {
                            if constexpr (XS_LDS)
                                s += dot4(w[h], xl[(k * H + h) * 64]);
                            else
                                s += dot4(w[h], xs[k]);
                        }
                    }
                }
                // lane 0 publishes. DPP for bf16 tiles at T = 4 (bench A/B at 64k x 64k: 772 vs 756 it/s); bf16 at
                // T = 2 (512k x 256k: 20.9 vs 21.3 it/s) and fp32 tiles keep the LDS bpermutes
                // (profiles/ab_r2_bf16_dpp_bench.jsonl, profiles/ab_r2_dpp_reductions.jsonl)
                if constexpr (BF && T == 4)
                    s = class_sum_dpp<1>(s, lane);
                else
                    s = wave_sum(s);
                if (lane == 0) {
                    s_part[(t & (NS - 1)) * 4 + wave] = s;
                    asm volatile("" ::: "memory");
                    s_pflag[(t & (NS - 1)) * 4 + wave] = (int)t;
                    if (DIAG && wave == 0) trace_stamp(b, t, 0);
                }
            }
            // park tile t - D (its LDS slot held tile t - D - NL, back-projected in step t - 1)
            if (t - D >= lo && t - D < hi) park(fl[bp], t - D);
            load_tile(fl[bp], t + AH);  // slot bp is free again
            if (t - L >= lo && t - L < hi) {
                const int64_t u = t - L;
                const int ws = (int)(u & (NS - 1));
                unsigned spins = 0;
                const unsigned long long w0 = DIAG ? __builtin_amdgcn_s_memtime() : 0;
                while (s_wflag[ws] != (int)u && !stuck) {
                    if (++spins > kSpinLimit) {
                        stuck = true;
                        if (lane == 0) atomicOr(&st->error, 2);
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if constexpr (DIAG) {
                    stall += __builtin_amdgcn_s_memtime() - w0;
                    nstall += spins > 0;
                    if (wave == 0 && lane == 0) trace_stamp(b, u, 1);
                }
                asm volatile("" ::: "memory");
                const float wr = s_w[ws * 4 + wrow];
                const RT* slot = ring + (int)(u % NL) * (4 * KW * 64);
#pragma unroll
                for (int k = 0; k < KW; ++k) {
                    float4 w[H];
                    FT::widen(slot[k * 64], w);
#pragma unroll
                    for (int h = 0; h < H; ++h) fma4(acc[k][h], w[h], wr);
                }
            }
        };
        const unsigned long long tstart = DIAG ? __builtin_amdgcn_s_memtime() : 0;
        // One pipeline loop for every mode: segments of chain_tiles tiles (SEG with chain_tiles > 0) or a single
        // segment of the whole group; FOLD folds the T = 1 chain every fpass passes.
        const int64_t F = seg_on ? chain_tiles : nt;
        const int64_t fpass = FOLD && chain_tiles > 0 ? (chain_tiles + RS - 1) / RS : (int64_t)1 << 62;
        int64_t fcount = 0, seg = 0;
        for (lo = 0; lo < nt; lo += F, ++seg) {
            hi = lo + F < nt ? lo + F : nt;
            if (SEG && lo > 0) {  // refill the pipeline (segment 0's prologue ran above)
#pragma unroll
                for (int i = 0; i < AH; ++i) load_tile(fl[i], lo + i);
            }
            for (int64_t t0 = lo; t0 < hi + L; t0 += RS) {  // RS steps per pass: register slots are static
                [&]<int... Q>(std::integer_sequence<int, Q...>) {
                    (step(std::integral_constant<int, Q>{}, t0 + Q), ...);
                }(std::make_integer_sequence<int, RS>{});
                if constexpr (FOLD) {
                    if (++fcount == fpass) {  // registers only: no memory operation joins the vmcnt pipeline
                        fcount = 0;
#pragma unroll
                        for (int k = 0; k < KW; ++k) {
                            add4(acc2[k], acc[k][0]);
                            acc[k][0] = make_float4(0.f, 0.f, 0.f, 0.f);
                        }
                    }
                }
            }
            if (SEG && seg_on) {  // this wave's sums of the segment: own partial block, then restart the chain
                float4* out = reinterpret_cast<float4*>(partial + (((int64_t)seg * T + wrow) * I + gi) * ld);
#pragma unroll
                for (int k = 0; k < KW; ++k)
#pragma unroll
                    for (int h = 0; h < H; ++h) {
                        out[(col4 + k * 64) * H + h] = acc[k][h];
                        acc[k][h] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
            }
        }
        if (SEG && seg_on) {
            __syncthreads();  // the exchange waves' two end barriers
            __syncthreads();
            return;
        }
        if constexpr (FOLD) {
#pragma unroll
            for (int k = 0; k < KW; ++k) add4(acc[k][0], acc2[k]);
        }
        if (DIAG && lane == 0) {
            g_fused_stats[b * 8 + wave] = stall;                       // [0..3] stall cycles per wave
            if (wave == 0) g_fused_stats[b * 8 + 4] = __builtin_amdgcn_s_memtime() - tstart;  // loop cycles
            if (wave == 1) g_fused_stats[b * 8 + 5] = nstall;          // steps that waited
        }
        // the T waves of a sub-slab hold partial sums of the same columns: combine through LDS
        __syncthreads();
        float4* red = s_ring + (wave * KW * H) * 64 + lane;
#pragma unroll
        for (int k = 0; k < KW; ++k)
#pragma unroll
            for (int h = 0; h < H; ++h) red[(k * H + h) * 64] = acc[k][h];
        __syncthreads();
        float4* out = reinterpret_cast<float4*>(partial + (int64_t)gi * ld);
        if constexpr (H == 1) out += slab4 + lane;  // (fp32 / narrow bf16: the original addressing)
#pragma unroll
        for (int i = 0; i < (WPR * KW * H + 3) / 4; ++i) {  // q = (sub * KW + k) * H + h over the four waves
            const int q = wave + 4 * i;
            if (q >= WPR * KW * H) break;
            const int sub = q / (KW * H), k = (q / H) % KW, h = q % H;
            float4 v = s_ring[q * 64 + lane];  // wave (row 0, sub)
#pragma unroll
            for (int rr = 1; rr < T; ++rr) {
                const float4 o = s_ring[(((rr * WPR + sub) * KW + k) * H + h) * 64 + lane];
                v.x += o.x;
                v.y += o.y;
                v.z += o.z;
                v.w += o.w;
            }
            if constexpr (H == 1)
                out[q * 64] = v;
            else
                out[(slab4 + (sub * KW + k) * 64 + lane) * H + h] = v;
        }
    } else if (SPLIT && wave == 4) {
        // Publisher wave (schedule 4): stores this workgroup's row partials as soon as the compute waves
        // have reduced them. It issues no loads, so no poll ever waits behind a granule store's
        // acknowledgement in the same wave's vmcnt queue (the coupling that delays publication when one
        // exchange wave both stores and polls).
        for (int64_t u = 0; u < nt; ++u) {
            const int ps = (int)(u & (NS - 1));
            if (lane < T) {
                const float sv = local_row_partial<T, FLAG4>(s_pflag, s_part, ps, (int)u, lane, kSpinLimit);
                if (!(dbg & 1)) {
                    uint64_t* g = gran + ((t_begin + u) * Jg + gj) * T + lane;
                    if constexpr (XL)
                        __hip_atomic_store(g, make_granule(epoch, sv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    else
                        __hip_atomic_store(g, make_granule(epoch, sv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (DIAG && lane == 0) trace_stamp(b, u, 2);
            }
        }
        __syncthreads();  // matches the compute waves' first combine barrier
        __syncthreads();  // and the second
    } else {
        const int n = J * T;
        bool failed = false;
        double F = 0.0;
        constexpr int GR = kRowsGather / 64;  // poll registers per lane (J * T <= kRowsGather)
        uint64_t pv[PQ][GR];
        // arow / ghat of the tile polled into pv[p], loaded together with its poll: a load issued only when the
        // tile is finished put a dependent L2 round trip (~1 us under streaming load) into every tile's hand-off
        float pa[PQ], pg[PQ];
        // unconditional clamped polls (see issue_poll in k_fused_sweep_lds): counted vmcnt, PQ polls in flight
        const int64_t ulast = ntiles - 1 - t_begin;
        auto issue_rows = [&](float& a, float& gh, int64_t u) {  // every lane (unconditional): row of lane % T
            const int64_t uc = u < 0 ? 0 : (u < ulast ? u : ulast);
            const int64_t row = (t_begin + uc) * T + (lane & (T - 1));
            a = arow[row];
            gh = LOG ? 0.f : ghat[row];
        };
        auto issue_poll = [&](uint64_t(&dst)[GR], int64_t u) {
            const int64_t uc = u < 0 ? 0 : (u < ulast ? u : ulast);
            const uint64_t* g = gran + (t_begin + uc) * (int64_t)Jg * T;
#pragma unroll
            for (int m = 0; m < GR; ++m) {
                const int idx = lane + 64 * m;
                dst[m] = __hip_atomic_load(g + (idx < n ? idx : n - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        unsigned long long xwait = 0, xrepoll = 0;
        auto finish_tile = [&](uint64_t(&v)[GR], float a, float gh, int64_t u) {
            const unsigned long long f0 = DIAG ? __builtin_amdgcn_s_memtime() : 0;
            if (!failed && !(dbg & 1)) {
                unsigned spins = 0;
                while (true) {
                    bool ok = true;
#pragma unroll
                    for (int m = 0; m < GR; ++m) ok &= ((int)(v[m] >> 32) == epoch);
                    if (__all(ok)) break;
                    if (++spins > kSpinLimit) {
                        failed = true;
                        if (lane == 0) atomicOr(&st->error, 1);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    issue_poll(v, u);
                    ++xrepoll;
                }
            }
            if constexpr (DIAG) {
                volatile uint64_t sink = v[0];  // make the wait for the poll registers part of the window
                (void)sink;
                xwait += __builtin_amdgcn_s_memtime() - f0;
            }
            float s = 0.f;
            if (!failed && !(dbg & 1)) {
#pragma unroll
                for (int m = 0; m < GR; ++m) s += (lane + 64 * m < n) ? __uint_as_float((uint32_t)v[m]) : 0.f;
            }
            // 8-KiB fp32 slabs keep the bpermutes: same-box A/B, 512kx256k preset shard (T = 1) 93.8 -> 102.1 it/s,
            // 64k x 64k (T = 4) +0.2 % (profiles/ab_r2_kw8_t1_gatherer.jsonl, ab_r2_kw8_t4_gatherer.jsonl)
            // (and bf16 at T = 2 like its compute waves; bf16 T = 4 and 6 / 7-KiB fp32 slabs use DPP)
            if constexpr (KW == 8 && !(BF && T == 4)) {
                for (int off = T; off < 64; off <<= 1) s += __shfl_xor(s, off, kWave);
            } else {
                s = class_sum_dpp<T>(s, lane);  // lane r < T: row r of the tile (fp32 200000 columns: -6 %)
            }
            const int ws = (int)(u & (NS - 1));
            if (lane < T) {
                const int64_t row = (t_begin + u) * T + lane;
                float w = 0.f;
                if (row < nrows) {
                    w = LOG ? a * s : a * (gh - s);
                    if (gj == 0) F += (double)s * (double)s;
                }
                s_w[ws * 4 + lane] = w;
            }
            asm volatile("" ::: "memory");
            if (lane == 0) s_wflag[ws] = (int)u;
            if (DIAG && lane == 0) trace_stamp(b, u, 3);
        };
        auto xiter = [&](auto pc, int64_t u) {
            constexpr int p = decltype(pc)::value;  // pv[p] receives tile u - PD
            // pacing: wait for the local row partials of tile u, except on a segment's first PD + PQ - 1 tiles,
            // while the compute waves drain the previous segment (split schedules only use the wait to pace)
            const bool pace = !(SEG && seg_on && u % chain_tiles < PD + PQ - 1);
            if (u < nt && pace) {
                const int ps = (int)(u & (NS - 1));
                if (lane < T) {
                    const float sv = local_row_partial<T, FLAG4>(s_pflag, s_part, ps, (int)u, lane, kSpinLimit);  // fixed order
                    if (!(dbg & 1) && !SPLIT) {
                        uint64_t* g = gran + ((t_begin + u) * Jg + gj) * T + lane;
                        if constexpr (XL)  // plain 8-byte store: the line stays in this XCD's L2
                            __hip_atomic_store(g, make_granule(epoch, sv), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                        else
                            __hip_atomic_store(g, make_granule(epoch, sv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (DIAG && lane == 0 && !SPLIT) trace_stamp(b, u, 2);
                }
            }
            issue_poll(pv[p], u - PD);  // (also with dbg & 1: the results are then ignored)
            issue_rows(pa[p], pg[p], u - PD);
            const int64_t f = u - PD - PQ + 1;  // polled PQ - 1 steps ago into pv[(p + 1) % PQ]
            if (f >= 0 && f < nt) finish_tile(pv[(p + 1) % PQ], pa[(p + 1) % PQ], pg[(p + 1) % PQ], f);
        };
        for (int64_t u0 = 0; u0 < nt + PD + PQ - 1; u0 += PQ) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (xiter(std::integral_constant<int, Q>{}, u0 + Q), ...);
            }(std::make_integer_sequence<int, PQ>{});
        }
        F = wave_sum(F);
        if (lane == 0) Fpart[b] = F;
        if (DIAG && lane == 0) {
            g_fused_stats[b * 8 + 6] = xwait;
            g_fused_stats[b * 8 + 7] = xrepoll;
        }
        __syncthreads();  // matches the compute waves' first combine barrier
        __syncthreads();  // and the second
    }
}

constexpr size_t rows_lds_bytes(int T, int sched, int H = 1, int KW = 8) {
    return (sched == 6 || sched == 7 ? 3 : (sched == 8 ? 5 : 4)) /*NL x 4 waves x KW x 64 lanes x 16 B*/ * 4 * KW * 64 * sizeof(float4) +
           (((sched >= 1 && sched <= 4) || sched == 6 || sched == 7) ? (4 / T) * KW * 64 * H * sizeof(float4) : 0) +  // x slab
           (8 * 4 * 3 + 8 + 4) * sizeof(float);
}
static_assert(rows_lds_bytes(4, 4, 2) <= 160 * 1024, "wide bf16 tiles: T = 4 fits the LDS");
static_assert(rows_lds_bytes(2, 6, 2) <= 160 * 1024, "wide bf16 tiles: T = 2 (schedule 6) fits the LDS");
static_assert(rows_lds_bytes(2, 7, 2) <= 160 * 1024, "wide bf16 tiles: T = 2 (schedule 7) fits the LDS");
static_assert(rows_lds_bytes(2, 4, 2) > 160 * 1024, "schedule 6 exists because the 4-slot ring does not fit");
static_assert(rows_lds_bytes(1, 5, 1, 9) <= 160 * 1024, "9-KiB slabs: T = 1 (schedule 5) fits the LDS");
static_assert(rows_lds_bytes(1, 8, 1, 7) <= 160 * 1024 && rows_lds_bytes(1, 8, 1, 8) > 160 * 1024,
              "schedule 8: a 5-slot ring of kw 7 slabs fits, of kw 8 slabs not");

static int g_fused_dbg = 0;    // diagnostics only (set through fused_set_debug)
static int g_fused_sched = 4;  // variant 6 pipeline schedule (k_fused_sweep_rows SCHED)
void fused_set_debug(int flags) { g_fused_dbg = flags; }
void fused_set_schedule(int sched) {
    if (sched < 0 || sched > 5) throw std::runtime_error("fused_set_schedule: 0 .. 5");
    g_fused_sched = sched;
}
int fused_get_schedule() { return g_fused_sched; }
static int g_fused_last_sched = -1;  // SCHED of the last k_fused_sweep_rows launch (variant 3: -1)
int fused_last_schedule() { return g_fused_last_sched; }

int64_t fused_granules(int64_t nrows_pad, int J, bool xl) {
    (void)xl;  // (XCD-local rows are padded too under SART_FUSED_GPAD=2)
    return nrows_pad * ((J + 15) & ~15);
}
bool fused_split_schedule(int T, bool bf16) {  // mirrors the schedule choice of launch_rows / launch_fused_sweep_bf16
    if (bf16) return T >= 2 || g_fused_sched == 5;
    return g_fused_sched >= 4;  // T = 1: 4 and 5 both run schedule 5; T >= 2: 5 runs 4
}
std::vector<int> fused_debug_map(int nblocks) {
    std::vector<int> out((size_t)nblocks);
    hip_call(hipMemcpyFromSymbol(out.data(), HIP_SYMBOL(g_fused_map), out.size() * sizeof(int), 0, hipMemcpyDeviceToHost), "hipMemcpyFromSymbol");
    return out;
}
void fused_set_trace(unsigned long long* buf, long long tiles) {
    hip_call(hipMemcpyToSymbol(HIP_SYMBOL(g_fused_trace), &buf, sizeof(buf), 0, hipMemcpyHostToDevice), "hipMemcpyToSymbol");
    hip_call(hipMemcpyToSymbol(HIP_SYMBOL(g_fused_trace_tiles), &tiles, sizeof(tiles), 0, hipMemcpyHostToDevice), "hipMemcpyToSymbol");
}
std::vector<unsigned long long> fused_debug_stats(int nblocks) {
    std::vector<unsigned long long> out((size_t)nblocks * 8);
    hip_call(hipMemcpyFromSymbol(out.data(), HIP_SYMBOL(g_fused_stats), out.size() * sizeof(unsigned long long), 0,
                        hipMemcpyDeviceToHost), "hipMemcpyFromSymbol");
    return out;
}


constexpr size_t kLdsRingBytes = 4 /*NL*/ * 4 /*waves*/ * 8 /*TK*/ * 64 * sizeof(float4) + 160 * sizeof(float);

template <int K>
static void launch_lds(bool logmode, dim3 grid, hipStream_t stream, const float* A, int64_t ld, int64_t nrows,
                       int64_t nrows_pad, const float* x, const float* ghat, const float* arow, float* partial,
                       double* Fpart, uint64_t* gran, int I, int J, SartState* st) {
    static bool configured = false;
    if (!configured) {  // opt in to > 64 KiB of dynamic LDS once per instantiation
        hip_call(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused_sweep_lds<K, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsRingBytes), "hipFuncSetAttribute");
        hip_call(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused_sweep_lds<K, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsRingBytes), "hipFuncSetAttribute");
        configured = true;
    }
    if (logmode)
        hipLaunchKernelGGL((k_fused_sweep_lds<K, true>), grid, dim3(kFusedThreads), kLdsRingBytes, stream, A, ld,
                           nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st, g_fused_dbg);
    else
        hipLaunchKernelGGL((k_fused_sweep_lds<K, false>), grid, dim3(kFusedThreads), kLdsRingBytes, stream, A, ld,
                           nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st, g_fused_dbg);
}

template <bool LG, bool X, bool D, int T, int SC, typename AT = float, int CPL = 4, int KW = 8>
static void launch_rows_t(dim3 grid, hipStream_t stream, const AT* A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                          const float* x, const float* ghat, const float* arow, float* partial, double* Fpart,
                          uint64_t* gran, int I, int J, SartState* st, unsigned* xcnt, int64_t chain_tiles) {
    constexpr size_t lds = rows_lds_bytes(T, SC, CPL / 4, KW);
    g_fused_last_sched = SC;
    static bool configured = false;
    if (!configured) {
        hip_call(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused_sweep_rows<LG, X, D, T, SC, AT, CPL, KW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "hipFuncSetAttribute");
        configured = true;
    }
    int dbg = g_fused_dbg;
    if constexpr (X) {
        const char* gp = std::getenv("SART_FUSED_GPAD");
        if (gp && *gp && std::atoi(gp) == 2) dbg |= 32;
    } else {
        // group map (SART_FUSED_CW_MAP: 0 = b % I, 1 = XCD-balanced, default: balanced for even I only) and granule
        // padding (SART_FUSED_GPAD=0: unpadded), read per launch (A/B runs)
        const char* e = std::getenv("SART_FUSED_CW_MAP");
        const int map = (e && *e) ? std::atoi(e) : 2;
        if (map == 0 || (map == 2 && I % 2 == 1)) dbg |= 8;
        const char* gp = std::getenv("SART_FUSED_GPAD");
        if (gp && *gp && std::atoi(gp) == 0) dbg |= 16;
    }
    hipLaunchKernelGGL((k_fused_sweep_rows<LG, X, D, T, SC, AT, CPL, KW>), grid,
                       dim3(sched_split(SC) ? kFusedThreads + 64 : kFusedThreads), lds, stream, A, ld, nrows,
                       nrows_pad, x,
                       ghat, arow, partial, Fpart, gran, I, J, st, dbg, xcnt, chain_tiles);
}

template <int T>
static void launch_rows(bool logmode, dim3 grid, hipStream_t stream, const float* A, int64_t ld, int64_t nrows,
                        int64_t nrows_pad, const float* x_, const float* ghat, const float* arow, float* partial,
                        double* Fpart, uint64_t* gran, int I, int J, SartState* st, unsigned* xcnt,
                        int64_t chain_tiles, int kw, bool xl) {
    if (!xl) {
        // chip-wide row groups (T = 1, schedule 5): workgroup b is (b % I, b / I), granules written through to
        // memory (agent scope), so a group may span XCDs: J up to the CU count, I = CUs / J of any value
        if constexpr (T == 1) {
            auto go_cw = [&](auto lg, auto k, auto sc) {
                launch_rows_t<decltype(lg)::value, false, false, 1, decltype(sc)::value, float, 4, decltype(k)::value>(
                    grid, stream, A, ld, nrows, nrows_pad, x_, ghat, arow, partial, Fpart, gran, I, J, st, xcnt,
                    chain_tiles);
            };
            // kw 6 / 7: schedule 8, the deeper exchange pipeline (+5.3 % at 300000 voxels, +2.8 % at 530432,
            // profiles/ab_r3_cw_sched8.jsonl); SART_FUSED_CW_SCHED=5 keeps schedule 5 (read per launch: A/B runs)
            const char* cws = std::getenv("SART_FUSED_CW_SCHED");
            const bool deep = !(cws && std::atoi(cws) == 5);
            using S5 = std::integral_constant<int, 5>;
            using S8 = std::integral_constant<int, 8>;
            auto by_kw = [&](auto lg) {
                if (kw == 8) go_cw(lg, std::integral_constant<int, 8>{}, S5{});
                else if (kw == 9) go_cw(lg, std::integral_constant<int, 9>{}, S5{});
                else if (kw == 7 && deep) go_cw(lg, std::integral_constant<int, 7>{}, S8{});
                else if (kw == 7) go_cw(lg, std::integral_constant<int, 7>{}, S5{});
                else if (kw == 6 && deep) go_cw(lg, std::integral_constant<int, 6>{}, S8{});
                else if (kw == 6) go_cw(lg, std::integral_constant<int, 6>{}, S5{});
                else go_cw(lg, std::integral_constant<int, 5>{}, S5{});
            };
            if (logmode) by_kw(std::true_type{}); else by_kw(std::false_type{});
            return;
        } else {
            // T = 2 / 4 (schedule 4, x slab in LDS): rows of more than an XCD's 32 slabs of 2048 / 4096 columns
            auto go_cw = [&](auto lg, auto k) {
                launch_rows_t<decltype(lg)::value, false, false, T, 4, float, 4, decltype(k)::value>(
                    grid, stream, A, ld, nrows, nrows_pad, x_, ghat, arow, partial, Fpart, gran, I, J, st, xcnt,
                    chain_tiles);
            };
            auto by_kw = [&](auto lg) {
                if (kw == 8) go_cw(lg, std::integral_constant<int, 8>{});
                else if (kw == 7) go_cw(lg, std::integral_constant<int, 7>{});
                else if (kw == 6) go_cw(lg, std::integral_constant<int, 6>{});
                else throw std::runtime_error("fused_sweep v6: chip-wide T >= 2 needs kw 6 ... 8");
            };
            if (logmode) by_kw(std::true_type{}); else by_kw(std::false_type{});
            return;
        }
    }
    const bool diag = (g_fused_dbg & 2) != 0;  // instrumented build only when asked (timing diagnostics)
    // g_fused_sched: pipeline schedule (k_fused_sweep_rows SCHED); schedules 1-4 hold the x slab in LDS,
    // which has room for it only when T >= 2. T = 1 runs schedule 5 (the split exchange with the x slab in
    // VGPRs) under the default schedule 4 (or 5): +10-14 % over schedule 0 at 73k-262k columns, with and
    // without idle CUs (profiles/probe_r2_t1_sched5.jsonl); schedules 0-3 select schedule 0 for T = 1.
    // Instrumented builds: schedules 0, 2 and 4.
    int sched = T >= 2 ? (g_fused_sched == 5 ? 4 : g_fused_sched) : (g_fused_sched >= 4 ? 5 : 0);
    if (diag && sched != 2 && sched != 4) sched = 0;
    auto go = [&](auto lg, auto d, auto sc) {
        launch_rows_t<decltype(lg)::value, true, decltype(d)::value, T, decltype(sc)::value>(
            grid, stream, A, ld, nrows, nrows_pad, x_, ghat, arow, partial, Fpart, gran, I, J, st, xcnt, chain_tiles);
    };
    using TT = std::true_type;
    using FF = std::false_type;
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, (T >= 2 ? 1 : 0)>;
    using S2 = std::integral_constant<int, (T >= 2 ? 2 : 0)>;
    using S3 = std::integral_constant<int, (T >= 2 ? 3 : 0)>;
    using S4 = std::integral_constant<int, (T >= 2 ? 4 : 0)>;
    using S5 = std::integral_constant<int, (T == 1 ? 5 : 4)>;
    auto by_log = [&](auto d, auto sc) {
        if (logmode) go(TT{}, d, sc); else go(FF{}, d, sc);
    };
    if (kw != 8) {  // narrower slabs: the default schedules only (4 at T >= 2, 5 at T = 1), no diagnostics
        auto go_kw = [&](auto lg, auto k) {
            using SD = std::integral_constant<int, (T >= 2 ? 4 : 5)>;
            launch_rows_t<decltype(lg)::value, true, false, T, SD::value, float, 4, decltype(k)::value>(
                grid, stream, A, ld, nrows, nrows_pad, x_, ghat, arow, partial, Fpart, gran, I, J, st, xcnt,
                chain_tiles);
        };
        auto by_kw = [&](auto lg) {
            if (kw == 7) go_kw(lg, std::integral_constant<int, 7>{});
            else if (kw == 6) go_kw(lg, std::integral_constant<int, 6>{});
            else if constexpr (T == 1) {
                if (kw == 9) go_kw(lg, std::integral_constant<int, 9>{});
                else go_kw(lg, std::integral_constant<int, 5>{});
            }
        };
        if (logmode) by_kw(TT{}); else by_kw(FF{});
        return;
    }
    if (diag) {
        if (sched == 2) by_log(TT{}, S2{});
        else if (sched == 4) by_log(TT{}, S4{});
        else by_log(TT{}, S0{});
        return;
    }
    switch (sched) {
        case 1: by_log(FF{}, S1{}); break;
        case 2: by_log(FF{}, S2{}); break;
        case 3: by_log(FF{}, S3{}); break;
        case 4: by_log(FF{}, S4{}); break;
        case 5: by_log(FF{}, S5{}); break;
        default: by_log(FF{}, S0{}); break;
    }
}

// Variant 3 slab width: 1024 * K columns, K the smallest power of two <= 8 giving at most 32 slabs.
int fused_pick_k(int64_t ld) {
    for (int K = 1; K <= 8; K *= 2) {
        const int64_t wc = 1024 * (int64_t)K;
        if (ld % wc != 0) return K > 1 ? K / 2 : 0;
        if (ld / wc <= 32) return K;
    }
    return 8;
}

int fused_fpart_per_block(int variant) {
    (void)variant;
    return 1;
}

int fused_tile_rows(int K, int variant) {
    return variant == 6 ? K : 8 / K;  // variant 6: K carries the rows per tile; variant 3: 8 float4 per lane
}

void launch_fused_sweep(bool logmode, int K, int variant, const float* A, int64_t ld, int64_t nrows,
                        int64_t nrows_pad, const float* x, const float* ghat, const float* arow, float* partial,
                        double* Fpart, uint64_t* gran, int I, int J, SartState* st, unsigned* xcnt,
                        hipStream_t stream, int64_t chain_tiles, int kw, bool xl) {
    if (variant != 3 && variant != 6) throw std::runtime_error("fused_sweep: variant must be 6 or 3");
    const dim3 grid((unsigned)(I * J));
    if (variant == 6) {
        const int T = K;
        if (T >= 2 && chain_tiles % kChainAlign != 0)
            throw std::runtime_error("fused_sweep v6: segment length must be a multiple of 140 tiles");
        if (T != 1 && T != 2 && T != 4) throw std::runtime_error("fused_sweep v6: rows per tile (K) must be 1, 2 or 4");
        if (kw < 5 || kw > 9) throw std::runtime_error("fused_sweep v6: lane-vectors per lane (kw) must be 5 ... 9");
        if ((kw == 5 || kw == 9) && T != 1) throw std::runtime_error("fused_sweep v6: 5- and 9-KiB slabs need T = 1");
        const int64_t slab = 1024 * kw / T;  // columns per workgroup
        if (ld % slab != 0 || ld / slab != J) throw std::runtime_error("fused_sweep v6: ld must equal J * slab");
        if (nrows_pad % 4 != 0) throw std::runtime_error("fused_sweep v6: padded rows must be a multiple of 4");
        if (J * T > kRowsGather) throw std::runtime_error("fused_sweep v6: J * T > 256");
        if (xl && (xcnt == nullptr || I % 8 != 0))
            throw std::runtime_error("fused_sweep v6: XCD-local groups need the per-XCD ticket counters and I % 8 == 0");
        if (!xl && T != 1 && (kw < 6 || kw > 8))
            throw std::runtime_error("fused_sweep v6: chip-wide row groups at T >= 2 need kw 6 ... 8");
        if (I < 1) throw std::runtime_error("fused_sweep v6: no row groups");
        if (T == 1) launch_rows<1>(logmode, grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st, xcnt,
                        chain_tiles, kw, xl);
        else if (T == 2) launch_rows<2>(logmode, grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st, xcnt,
                        chain_tiles, kw, xl);
        else launch_rows<4>(logmode, grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st, xcnt,
                        chain_tiles, kw, xl);
        check_launch("k_fused_sweep_rows");
        return;
    }
    if (K != 1 && K != 2 && K != 4 && K != 8) throw std::runtime_error("fused_sweep v3: K must be 1, 2, 4 or 8");
    if (ld % (1024 * K) != 0 || ld / (1024 * K) != J) throw std::runtime_error("fused_sweep v3: ld must equal J * 1024 * K");
    const int T = 8 / K;
    if (nrows_pad % T != 0) throw std::runtime_error("fused_sweep v3: padded rows must be a multiple of the tile");
    if (J * T > kMaxGather) throw std::runtime_error("fused_sweep v3: too many slabs for the gather registers");
    g_fused_last_sched = -1;
    switch (K) {
        case 1: launch_lds<1>(logmode, grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st); break;
        case 2: launch_lds<2>(logmode, grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st); break;
        case 4: launch_lds<4>(logmode, grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st); break;
        default: launch_lds<8>(logmode, grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st); break;
    }
    check_launch("k_fused_sweep_lds");
}

// bf16-stored RTM: variant 6 only (XCD-local row groups, same exchange as fp32). cpl 8 ("wide": 16-byte loads of
// 8 bf16 per lane, slab 16384 / T columns) needs T = 4 (schedule 4, x slab in LDS) or T = 2 (schedule 6: a
// 3-slot ring next to the two sub-slabs' x slab); cpl 4 ("narrow": 8-byte
// loads, slab 8192 / T) runs schedule 4 for T >= 2 and for T = 1 schedule 0 with the deep bf16 lag (or 5 when
// selected). A protocol timeout falls back to the bf16 two-pass kernels.
void launch_fused_sweep_bf16(bool logmode, int T, const bf16_t* A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                             const float* x, const float* ghat, const float* arow, float* partial, double* Fpart,
                             uint64_t* gran, int I, int J, SartState* st, unsigned* xcnt, hipStream_t stream, int cpl,
                             int64_t chain_tiles, int kw, bool xl) {
    if (T != 1 && T != 2 && T != 4) throw std::runtime_error("fused_sweep bf16: rows per tile must be 1, 2 or 4");
    if (cpl != 4 && !(cpl == 8 && (T == 4 || T == 2)))
        throw std::runtime_error("fused_sweep bf16: wide tiles need T = 4 or 2");
    if (kw != 8 && !(cpl == 8 && kw >= 5 && kw <= 7))
        throw std::runtime_error("fused_sweep bf16: kw 5 ... 7 only with wide tiles (narrow tiles: kw 8)");
    if (nrows_pad % 4 != 0) throw std::runtime_error("fused_sweep bf16: padded rows must be a multiple of 4");
    if (T >= 2 && chain_tiles % kChainAlign != 0)
        throw std::runtime_error("fused_sweep bf16: segment length must be a multiple of 140 tiles");
    const int64_t slab = 256 * (int64_t)cpl * kw / T;  // 4 / T sub-slabs of 64 lanes x kw lane-vectors x cpl columns
    if (ld % slab != 0 || ld / slab != J) throw std::runtime_error("fused_sweep bf16: ld must equal J * slab");
    if (J * 4 > kMaxGather || J * T > kRowsGather) throw std::runtime_error("fused_sweep bf16: too many slabs");
    if (xl && (xcnt == nullptr || I % 8 != 0))
        throw std::runtime_error("fused_sweep bf16: XCD-local groups need ticket counters and I % 8 == 0");
    if (!xl && cpl != 8) throw std::runtime_error("fused_sweep bf16: chip-wide row groups take the wide tiles only");
    if (I < 1) throw std::runtime_error("fused_sweep bf16: no row groups");
    const dim3 grid((unsigned)(I * J));
    // chip-wide row groups (xl false, wide tiles only): the fp32 chip-wide protocol (granules through memory in
    // padded rows, the XCD-balanced map) at T = 4 / 2, where a row of 32 wide slabs does not fit one XCD
    auto go = [&](auto lg, auto tt, auto sc, auto cp) {
        constexpr int TT = decltype(tt)::value, SC = decltype(sc)::value, CP = decltype(cp)::value;
        auto run = [&](auto k) {
            if constexpr (CP == 8) {
                if (!xl) {
                    launch_rows_t<decltype(lg)::value, false, false, TT, SC, bf16_t, CP, decltype(k)::value>(
                        grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st, xcnt,
                        chain_tiles);
                    return;
                }
            }
            launch_rows_t<decltype(lg)::value, true, false, TT, SC, bf16_t, CP, decltype(k)::value>(
                grid, stream, A, ld, nrows, nrows_pad, x, ghat, arow, partial, Fpart, gran, I, J, st, xcnt, chain_tiles);
        };
        if constexpr (CP == 8) {  // wide tiles: narrower slabs so that J fills an XCD's 32 CUs at more widths
            if (kw == 7) return run(std::integral_constant<int, 7>{});
            if (kw == 6) return run(std::integral_constant<int, 6>{});
            if (kw == 5) return run(std::integral_constant<int, 5>{});
        }
        run(std::integral_constant<int, 8>{});
    };
    using S0 = std::integral_constant<int, 0>;
    using S4 = std::integral_constant<int, 4>;
    using S5 = std::integral_constant<int, 5>;
    using S6 = std::integral_constant<int, 6>;
    using S7 = std::integral_constant<int, 7>;
    // wide tiles at T = 2: schedule 7 (L = 4) unless SART_BF16_T2_SCHED=6 (read per launch: tests switch it)
    const char* t2e = std::getenv("SART_BF16_T2_SCHED");
    const bool t2_sched6 = t2e && std::atoi(t2e) == 6;
    using C4 = std::integral_constant<int, 4>;
    using C8 = std::integral_constant<int, 8>;
    auto by_t = [&](auto lg) {
        if (cpl == 8 && T == 2 && t2_sched6) go(lg, std::integral_constant<int, 2>{}, S6{}, C8{});
        else if (cpl == 8 && T == 2) go(lg, std::integral_constant<int, 2>{}, S7{}, C8{});
        else if (cpl == 8) go(lg, std::integral_constant<int, 4>{}, S4{}, C8{});
        else if (T == 1 && g_fused_sched == 5) go(lg, std::integral_constant<int, 1>{}, S5{}, C4{});
        else if (T == 1) go(lg, std::integral_constant<int, 1>{}, S0{}, C4{});
        else if (T == 2) go(lg, std::integral_constant<int, 2>{}, S4{}, C4{});
        else go(lg, std::integral_constant<int, 4>{}, S4{}, C4{});
    };
    if (logmode) by_t(std::true_type{}); else by_t(std::false_type{});
    check_launch("k_fused_sweep_rows<bf16>");
}

}  // namespace sart
