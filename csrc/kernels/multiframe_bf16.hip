// Multi-frame projections of a bf16-stored RTM on the bf16 matrix cores of gfx950 (v_mfma_f32_16x16x32_bf16:
// 16x the fp32 MFMA rate, so the skinny GEMMs of the multi-frame solver stay HBM-bound at 64 frames, where the
// fp32 engine is matrix-core-bound; multiframe.hip).
//
// Numerics. The matrix is bf16 by choice of storage (--rtm_bf16: every element is exact in the operand).
// The other operand (the solutions X of the forward projection, the SART weights W of the back-projection) is
// fp32 state; it enters as two bf16 planes, hi = rne(x) and lo = rne(x - hi), and every product runs twice
// (A hi + A lo) into the same fp32 accumulator: |x - hi - lo| <= 2^-17 |x|, below the storage rounding of
// A itself (2^-9) by a factor 256, with fp32 accumulation as in the fp32 engine. The planes are written once
// per sweep by k_mf_split_x / k_mf_split_w (multiframe_glue.hip).
//
// Fragment maps (cdna_hip_programming.md section 3, 16x16x32 bf16): lane l holds A[i = l & 15][k = 8 (l >> 4) + j]
// and B[k = 8 (l >> 4) + j][n = l & 15] in element j = 0..7; C/D: n = l & 15, i = (l >> 4) * 4 + reg.
//
// Forward F[row][f] = sum_v A[row][v] X[f][v]: M = 16 rows, N = 16 frames, K = 32 voxels. A lane's eight k
// are eight consecutive voxels of one row, so one 16-byte load of A and one of each X plane per 32 voxels;
// a wave owns 16 * RT rows and reuses each X fragment RT times.
//
// Back-projection D[v][f] = sum_row A[row][v] W[row][f]: M = 16 voxels, N = 16 frames, K = 32 rows. A lane's
// eight k must be eight ROWS of one voxel, while a row of A is contiguous: each lane loads 8 bytes (4 voxels)
// of 8 rows (16 lanes x 8 B = one 128-B line per row and instruction) and regroups them with v_perm_b32 into
// four fragments, one per voxel phase p (voxels 4 i + p of the 64-voxel block), no LDS round trip. The W
// planes are stored frame-major [nf][rows] so a lane's eight rows are one 16-byte load.
//
// Ring loads are unconditional (clamped to the last step) like the fp32 kernels: the compiler then keeps
// DEPTH steps of loads in flight with counted vmcnt waits.
//
// Split-A mode (AT = float: an fp32-stored RTM on the bf16 matrix cores). The fp32 engine (multiframe.hip) is
// matrix-core bound at 32 / 64 frames: fp32 MFMA runs at 1/16 of the bf16 rate. The LDS kernels below also take
// an fp32 A, split each element in registers as it is consumed, hi = rne(a), lo = rne(a - hi)
// (|a - hi - lo| <= 2^-18 |a|, below the fp32 accumulation error of a 64k-long dot), and run three products
// A_hi X_hi + A_hi X_lo + A_lo X_hi into the fp32 accumulator (the dropped A_lo X_lo is ~2^-17 of the product;
// A and X are non-negative, so the forward sums do not cancel and these errors stay at 2^-17 / sqrt(K) of F:
// fp32 level, tools/x3_accuracy.py). The back-projection's weights are residuals of both signs whose sum cancels:
// there a representation error of 2^-18 of each term shows at full size in A^T W (measured 4e-6 against fp32's
// 1.4e-7), so A and W enter as three pieces each (hi + mid + lo to 2^-27) and six products (every pair of
// combined weight >= 2^-16). Three / six bf16 MFMAs cost 3/16 / 6/16 of one fp32 MFMA of the same K; the splits
// are 3 / 5 VALU operations per element of A, which overlap the stream. The stored matrix, the fp32 state and the
// fp32 sums are those of the fp32 engine.
#include "sart_common.hpp"
#include "launchers.hpp"

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>

namespace sart {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // a first-class 16-byte value (no struct memcpy)

__device__ __forceinline__ floatx4 mfma_b16(const uint4 a, const uint4 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}
__device__ __forceinline__ floatx4 mfma_b16(const uint4 a, const u32x4 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

typedef unsigned u32x8 __attribute__((ext_vector_type(8)));  // eight fp32 of A (a split-A forward fragment)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ floatx4 mfma_b16(const u32x4 a, const u32x4 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

// Split two fp32 (bit patterns x = element 2m, y = element 2m + 1) into packed bf16 hi = rne and lo = rne of
// the remainder.
__device__ __forceinline__ void split_a2(unsigned x, unsigned y, unsigned& hi, unsigned& lo) {
    const float a = __uint_as_float(x), b = __uint_as_float(y);
    const bf16x2_t h = bf16x2_t{(__bf16)a, (__bf16)b};
    hi = __builtin_bit_cast(unsigned, h);
    const float ra = a - __uint_as_float(hi << 16), rb = b - __uint_as_float(hi & 0xffff0000u);
    lo = __builtin_bit_cast(unsigned, bf16x2_t{(__bf16)ra, (__bf16)rb});
}

// Forward fragment of a split-A wave: eight consecutive fp32 of one row -> hi / lo bf16 fragments.
__device__ __forceinline__ void split_a8(const u32x8 v, u32x4& hi, u32x4& lo) {
    unsigned h0, h1, h2, h3, l0, l1, l2, l3;
    split_a2(v[0], v[1], h0, l0);
    split_a2(v[2], v[3], h1, l1);
    split_a2(v[4], v[5], h2, l2);
    split_a2(v[6], v[7], h3, l3);
    hi = u32x4{h0, h1, h2, h3};
    lo = u32x4{l0, l1, l2, l3};
}

typedef _Float16 halfx8_t __attribute__((ext_vector_type(8)));
typedef _Float16 halfx2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ floatx4 mfma_h16(const u32x4 a, const u32x4 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8_t, a), __builtin_bit_cast(halfx8_t, b),
                                                  c, 0, 0, 0);
}
// Two VALU operations per element: p1 = rne16(a s) and p2 = rne16(a s - p1) are each one v_fma_mix{lo,hi}_f16 (fp32
// a and s, for p2 an f16 half of p1 as the negated addend; the f16 result goes into one half of the packed register).
// a s is exact (s is a power of two inside the clamped range) and so is a s - p1 in fp32, so each single rounding to
// f16 gives the bits of scaling, converting and subtracting separately. Written in C++ the compiler emitted the
// scale, a v_cvt_pk_f16_f32 and the products again for the residual (7 operations per pair instead of 4), or packed
// fp32 FMAs and conversions back, which cost more beside MFMAs (MI355X_MICROARCH.md, filler prices).
__device__ __forceinline__ void split_h2(unsigned x, unsigned y, float s, unsigned& p1, unsigned& p2) {
    asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
        "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
        "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(p1), "=&v"(p2)
        : "v"(__uint_as_float(x)), "v"(__uint_as_float(y)), "v"(s));
}
// Forward fragment of an f16-pair split-A wave: eight consecutive fp32 of one row, scaled by the row's s_p
__device__ __forceinline__ void split_h8(const u32x8 v, float s, u32x4& p1, u32x4& p2) {
    unsigned a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) split_h2(v[2 * q], v[2 * q + 1], s, a[q], b[q]);
    p1 = u32x4{a[0], a[1], a[2], a[3]};
    p2 = u32x4{b[0], b[1], b[2], b[3]};
}

// Three pieces, exact: hi + mid + lo = a (the back-projection, whose signed weights cancel in the sum). Truncation
// splits: hi = the top 16 bits of a, r = a - hi is exact (same sign and exponent, <= 16 significant bits), mid = the
// top 16 bits of r, lo = r - mid exact with <= 8 significant bits, i.e. a bf16 value. Per pair of elements: 4 v_and,
// 4 subtractions and 3 v_perm (upper halves), as many operations as the round-to-nearest split (3 cvt_pk, 4
// widenings, 4 subtractions) but cheaper ones beside the MFMAs (+1.5-3 % at 32 / 64 frames,
// profiles/ab_r2_mf_trunc_split.jsonl), and no representation error left at all.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split_a2_3(unsigned x, unsigned y, unsigned& hi, unsigned& mid, unsigned& lo) {
    const f32x2 a = {__uint_as_float(x), __uint_as_float(y)};
    const f32x2 h = {__uint_as_float(x & 0xffff0000u), __uint_as_float(y & 0xffff0000u)};
    // one subtraction and one fma per pair, not two isomorphic subtractions: the compiler would pack those into
    // v_pk_add_f32, which costs more than two plain operations beside MFMAs (MI355X_MICROARCH.md, filler prices)
    const f32x2 r = {a.x - h.x, __builtin_fmaf(h.y, -1.0f, a.y)};
    const unsigned rx = __float_as_uint(r.x), ry = __float_as_uint(r.y);
    const f32x2 m = {__uint_as_float(rx & 0xffff0000u), __uint_as_float(ry & 0xffff0000u)};
    const f32x2 l = {r.x - m.x, __builtin_fmaf(m.y, -1.0f, r.y)};
    constexpr unsigned kUpper = 0x07060302u;  // bytes 2-3 of S1 (x: element 2m), then bytes 2-3 of S0 (y)
    hi = __builtin_amdgcn_perm(y, x, kUpper);
    mid = __builtin_amdgcn_perm(ry, rx, kUpper);
    lo = __builtin_amdgcn_perm(__float_as_uint(l.y), __float_as_uint(l.x), kUpper);
}

// Back-projection fragment of voxel phase P from eight 16-byte fp32 row loads (4 voxels each): element j = the
// fp32 of voxel P in row load j, split into hi / mid / lo.
template <int P>
__device__ __forceinline__ void split_phase3(const u32x4 (&v)[8], u32x4& hi, u32x4& mid, u32x4& lo) {
    unsigned h[4], m[4], l[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) split_a2_3(v[2 * q][P], v[2 * q + 1][P], h[q], m[q], l[q]);
    hi = u32x4{h[0], h[1], h[2], h[3]};
    mid = u32x4{m[0], m[1], m[2], m[3]};
    lo = u32x4{l[0], l[1], l[2], l[3]};
}

// Raw A storage of one fragment: 16 bytes of bf16 or 32 bytes of fp32 (forward); 8 or 16 bytes of one row's
// four voxels (back-projection).
template <typename AT> struct ARaw;
template <> struct ARaw<bf16_t> { typedef uint4 fwd; typedef uint2 bwd; };
template <> struct ARaw<float> { typedef u32x8 fwd; typedef u32x4 bwd; };

// Fragment of voxel phase P from the eight 8-byte row loads: element j = bf16 P of row load j.
template <int P>
__device__ __forceinline__ uint4 phase_frag(const uint2 (&v)[8]) {
    constexpr unsigned sel = (P & 1) ? 0x07060302u : 0x05040100u;  // high / low halves of (S1, S0)
    auto d = [&](int m) {
        const unsigned a = (P >> 1) ? v[2 * m].y : v[2 * m].x;
        const unsigned b = (P >> 1) ? v[2 * m + 1].y : v[2 * m + 1].x;
        return __builtin_amdgcn_perm(b, a, sel);  // bytes 0-3 select from a (S1), 4-7 from b (S0)
    };
    return make_uint4(d(0), d(1), d(2), d(3));
}

}  // namespace

// Column range and X plane layout of a forward launch: element (frame f, voxel c) of a plane sits at
// f * xfs + (c / 32) * xbs + c % 32. Frame-major planes [nf][ld]: xfs = ld, xbs = 32. Blocked planes
// [ld / 32][nf][32] (launch_mf_split_x with ld > 0): xfs = 32, xbs = 32 nf, so the X tile of a step (nf frames of
// 32 voxels) is one contiguous 2 nf * 32 bytes per plane instead of nf 64-byte pieces ld * 2 bytes apart.
struct FwdCols {
    int64_t cps, xfs, xbs;
    // f16-pair split-A forward (H16): per-row scales of A ([nrows_pad] scales, then their inverses) and the
    // per-frame inverse scales of the X pieces (launch_mf_split_x16)
    const float* rsc = nullptr;
    const float* xinv = nullptr;
};

// Split-K over columns: blockIdx.y selects [c0, c1) (multiples of 64); Fout + blockIdx.y * nrows_pad * nf.
// A step covers KB blocks of 32 voxels; with KB = 2 the two loads of a row are the two halves of one 128-byte
// line, issued back to back.
template <int NG, int DEPTH, int RT, int KB>
__global__ __launch_bounds__(256) void k_mf_forward_b16(const bf16_t* __restrict__ A, int64_t ld, int64_t nrows,
                                                        int64_t nrows_pad, const bf16_t* __restrict__ Xh,
                                                        const bf16_t* __restrict__ Xl, float* __restrict__ Fout,
                                                        FwdCols fc, const int* __restrict__ skip) {
    const int64_t cols_per_split = fc.cps, xfs = fc.xfs, xbs = fc.xbs;
    if (skip && *skip) return;  // every frame of the batch is done: the sweep is a no-op
    constexpr int NF = 16 * NG;
    constexpr int RS = DEPTH + 1;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * (16 * RT);
    if (row0 >= nrows_pad) return;  // wave-uniform; nrows_pad is a multiple of 16 * RT
    const int g = lane >> 4, r = lane & 15;
    const int64_t c0 = (int64_t)blockIdx.y * cols_per_split;
    const int64_t c1 = (c0 + cols_per_split < ld) ? c0 + cols_per_split : ld;
    Fout += (int64_t)blockIdx.y * nrows_pad * NF;
    const bf16_t* __restrict__ ap = A + (row0 + r) * ld + c0 + 8 * g;
    const int64_t xo = (int64_t)r * xfs + (c0 >> 5) * xbs + 8 * g;  // frame r of column group 0; group j: + 16 j xfs

    floatx4 acc[RT][NG];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < NG; ++j) acc[t][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int64_t nst = c1 > c0 ? (c1 - c0) / (32 * KB) : 0;
    if (nst > 0) {
        uint4 a[RS][RT][KB], xh[RS][NG][KB], xl[RS][NG][KB];
        auto load = [&](int sl, int64_t t) {
            const int64_t q = t * 32 * KB;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int kb = 0; kb < KB; ++kb)
                    a[sl][rt][kb] = *reinterpret_cast<const uint4*>(ap + rt * 16 * ld + q + 32 * kb);
#pragma unroll
            for (int j = 0; j < NG; ++j)
#pragma unroll
                for (int kb = 0; kb < KB; ++kb) {
                    xh[sl][j][kb] = *reinterpret_cast<const uint4*>(Xh + xo + (int64_t)j * 16 * xfs + (t * KB + kb) * xbs);
                    xl[sl][j][kb] = *reinterpret_cast<const uint4*>(Xl + xo + (int64_t)j * 16 * xfs + (t * KB + kb) * xbs);
                }
        };
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) load(d, d < nst ? d : nst - 1);
        auto step = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            load((sl + DEPTH) % RS, t + DEPTH < nst ? t + DEPTH : nst - 1);
            if (t >= nst) return;
#pragma unroll
            for (int kb = 0; kb < KB; ++kb)
#pragma unroll
                for (int j = 0; j < NG; ++j)
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) {
                        acc[rt][j] = mfma_b16(a[sl][rt][kb], xh[sl][j][kb], acc[rt][j]);
                        acc[rt][j] = mfma_b16(a[sl][rt][kb], xl[sl][j][kb], acc[rt][j]);
                    }
        };
        for (int64_t t0 = 0; t0 < nst; t0 += RS) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (step(std::integral_constant<int, Q>{}, t0 + Q), ...);
            }(std::make_integer_sequence<int, RS>{});
        }
    }
    // D: n = frame 16 j + (lane & 15), i = (lane >> 4) * 4 + reg = row within the 16-row tile
#pragma unroll
    for (int j = 0; j < NG; ++j)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t ra = row0 + rt * 16 + g * 4 + i;
                if (ra < nrows) Fout[ra * NF + 16 * j + r] = acc[rt][j][i];
            }
}

// The forward with X shared through LDS: the four waves of a workgroup own different rows of the same column
// range, so they need the same X fragments. Per step the X tile ([KB][hi, lo][NG][16 frames][32 voxels], 1 KiB
// per (kb, plane, group)) is loaded once per workgroup, each wave loading a quarter into registers and writing
// it to one of two LDS stages; every wave then reads its fragments from LDS (contiguous 1 KiB per fragment
// instruction: conflict-free). X bytes through the vector memory path per byte of A drop 4x (2 N / R with
// R = 64 RT rows per wave -> per workgroup), which is what bounds the register-operand forward at 32 / 64
// frames (profiles/probe_r2_mf_b16.jsonl). One barrier per step; waves past the padded rows clamp to the last
// row tile (they take part in the X staging and barriers, and store nothing).
//
// AS (A staged): a fragment-shaped load (lane (r, g) = 16 B of row r) touches 16 rows x 64 B per instruction,
// half lines, twice the address-path work per byte of the back-projection's row loads. With AS each wave loads
// its A tile in full 128-B row segments (R16 lanes per row, 64 / R16 rows per instruction), writes it to a
// wave-private LDS image with the 16-B slot XOR-swizzled by (row & 7) (slot row * R16 + (seg ^ (row & 7)): the
// 16 lanes that read one fragment column hit 8 different bank groups), and reads the fragments back with
// ds_read_b128. Same in-order LDS queue for the write and the read of one wave: no barrier.
// Waves per SIMD the register budget is cut for (the second __launch_bounds__ argument): SART_MF_MINW_FWD /
// SART_MF_MINW_BWD at compile time (A/B builds); 1 lets the 64-frame bf16 kernels take 284 / 332 VGPRs (one wave per
// SIMD, no latency hiding across waves).
#ifndef SART_MF_MINW_FWD
#define SART_MF_MINW_FWD 1
#endif
#ifndef SART_MF_MINW_BWD
#define SART_MF_MINW_BWD 1
#endif
// A-staged forwards (AS): non-temporal loads of the A tile (A/B builds: -DSART_MF_AS_NT=0)
#ifndef SART_MF_AS_NT
#define SART_MF_AS_NT 1
#endif
// split-A: X / W of the next step staged into LDS after the step's MFMAs (A/B builds: -DSART_MF_STAGE_LATE=0)
#ifndef SART_MF_STAGE_LATE
#define SART_MF_STAGE_LATE 1
#endif
// Two-level accumulation of the split-K sums: every SART_MF_FLUSH outer iterations (of DEPTH + 1 steps) the MFMA
// accumulators are added into a second fp32 sum and restarted, so no fp32 chain runs over a whole split. One chain
// per split (16384 terms at 64k x 64k) measured 3.5x the fp32 two-pass kernels' error at 64 frames after 20 SART
// updates on the ray-traced RTM (profiles/parity_r6_64k_raytraced.jsonl); every 4 trips: 0.76-1.01x, every 2:
// 0.75-1.07x, 4 is +0.3 / +0.7 % faster at 64 / 128 frames (profiles/ab_r6_mf_flush.txt); 0 disables (A/B).
#ifndef SART_MF_FLUSH
#define SART_MF_FLUSH 4
#endif
// the forward's second-level sum in LDS (1) or registers (0, default: 13930 against 13300 frame-it/s at 128 frames,
// equal at 64; profiles/ab_r6_mf_flush.txt)
#ifndef SART_MF_FLUSH_LDS
#define SART_MF_FLUSH_LDS 0
#endif
// bf16 X / W fragments read from LDS all at once at the top of a step (A/B builds: -DSART_MF_XF_EARLY=0)
#ifndef SART_MF_XF_EARLY
#define SART_MF_XF_EARLY 1
#endif
template <typename AT, int NG>
constexpr int mf_fwd_min_waves() { return std::is_same<AT, float>::value ? 1 : (NG == 4 ? SART_MF_MINW_FWD : 1); }

// ABL: diagnostic ablations as in k_mf_backproject_b16_lds (bit 0 no MFMAs, bit 1 no split of A, bit 2 no X staging
// and no barrier); 0 in every production launch.
// EX (early X): X of step u is loaded at step u - DEPTH - 1, ahead of A's batch (see EW of k_mf_backproject_b16_lds).
// H16 (split-A only): A enters as two f16 pieces of A s_p (s_p per row, FwdCols::rsc) and X as two f16 pieces of
// X s_f (launch_mf_split_x16), three v_mfma_f32_16x16x32_f16 products (a2 x1, a1 x2, a1 x1), the epilogue multiplies
// by 1 / (s_p s_f): 2^-22 per product instead of the 2^-17 of the bf16 hi + lo pieces, at the same cost.
template <int NG, int DEPTH, int RT, int KB, typename AT = bf16_t, bool AS = false, int ABL = 0, bool EX = false,
          bool H16 = false>
__global__ __launch_bounds__(256, (mf_fwd_min_waves<AT, NG>())) void k_mf_forward_b16_lds(const AT* __restrict__ A, int64_t ld, int64_t nrows,
                                                            int64_t nrows_pad, const bf16_t* __restrict__ Xh,
                                                            const bf16_t* __restrict__ Xl, float* __restrict__ Fout,
                                                            FwdCols fc, const int* __restrict__ skip) {
    const int64_t cols_per_split = fc.cps, xfs = fc.xfs, xbs = fc.xbs;
    if (skip && *skip) return;
    constexpr int NF = 16 * NG;
    constexpr int RS = DEPTH + 1;
    constexpr int C = KB * 2 * NG;             // 1 KiB X pieces per step
    constexpr int XQ = C >= 4 ? C / 4 : 1;     // pieces per wave (C = 2: two waves load each piece)
    __shared__ __attribute__((aligned(16))) u32x4 s_x[2][C][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * (16 * RT);
    const bool live = row0 < nrows_pad;
    if (!live) row0 = nrows_pad - 16 * RT;  // nrows_pad is a multiple of 16 * RT
    const int g = lane >> 4, r = lane & 15;
    const int64_t c0 = (int64_t)blockIdx.y * cols_per_split;
    const int64_t c1 = (c0 + cols_per_split < ld) ? c0 + cols_per_split : ld;
    Fout += (int64_t)blockIdx.y * nrows_pad * NF;
    constexpr bool A32 = std::is_same<AT, float>::value;
    constexpr bool LATE = SART_MF_STAGE_LATE && A32;  // stage_next after the MFMAs (split-A only, see below)
    constexpr bool NT_AS = SART_MF_AS_NT != 0;
    // split-A: lane (r, g) loads voxels 4 g .. 4 g + 3 and 16 + 4 g .. of each 32-voxel block (two contiguous
    // 64-byte halves of a row per instruction instead of four 16-byte pieces); the X planes hold the same k order
    // (k_mf_split_x with perm)
    const AT* __restrict__ ap = A + (row0 + r) * ld + c0 + (A32 ? 4 : 8) * g;
    const int64_t xo = (int64_t)r * xfs + (c0 >> 5) * xbs + 8 * g;
    // uint4 slot of this lane's fragment (frame r, voxels 8 g..) inside a 1 KiB piece: the lane index itself. Every
    // wave's lane l reads what lane l of the loading wave wrote, so any bijection works; lane-linear slots put the 16
    // lanes of each ds_read_b128 group and the 8 of each ds_write_b128 group on distinct 16-B bank slots (the former
    // r * 4 + g was 2-way on the reads and 4-way on the writes: PMC SQ_LDS_BANK_CONFLICT ~4x the LDS-active cycles,
    // profiles/pmc_r3_mfb64.txt)
    const int lofs = lane;
    typedef typename ARaw<AT>::fwd AF;
    constexpr int R16 = 32 * KB * (int)sizeof(AT) / 16;  // 16-B slots per row and step (AS)
    constexpr int RPI = 64 / R16;                         // rows per staging load instruction
    constexpr int NI = 16 * RT / RPI;                     // staging loads per step and wave
    static_assert(!AS || R16 >= 8, "A staging needs full 128-B row segments");
    __shared__ __attribute__((aligned(16))) u32x4 s_a[AS ? 4 : 1][AS ? 16 * RT * R16 : 1];
    const AT* __restrict__ asp = A + (row0 + lane / R16) * ld + c0 + (lane % R16) * (16 / (int)sizeof(AT));
    static_assert(!H16 || (A32 && ABL == 0), "the f16-pair forward is a split-A kernel");
    float rs[RT];  // H16: this lane's row scales (row row0 + 16 rt + r of each row tile)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) rs[rt] = H16 ? fc.rsc[row0 + rt * 16 + r] : 1.f;

    // The second-level sum: registers, or (SART_MF_FLUSH_LDS) lane-private LDS slots as in k_mf_backproject_h16 where
    // the workgroup's LDS still fits. Either costs 8-12 % at 128 frames against no flush (SART_MF_FLUSH=0: 15.1k
    // frame-it/s), less than the 4x split-K that gives the same error (profiles/ab_r6_mf_flush.txt)
    constexpr size_t kLdsX = sizeof(u32x4) * 2 * C * 64, kLdsA = AS ? sizeof(u32x4) * 4 * 16 * RT * R16 : 16;
    // (split-A only: with bf16 storage the X pieces' 2^-17 sets the error and the chains do not matter; the flush cost
    // 3-5 % there, profiles/ab_r6_mf_flush.txt)
    constexpr int FLUSH = A32 ? SART_MF_FLUSH : 0;
    constexpr bool FL_LDS = SART_MF_FLUSH_LDS && FLUSH > 0 &&
                            kLdsX + kLdsA + sizeof(floatx4) * 4 * RT * NG * 64 <= 163840;
    floatx4 acc[RT][NG], sum[FL_LDS ? 1 : RT][FL_LDS ? 1 : NG];
    __shared__ __attribute__((aligned(16))) floatx4 s_acc[FL_LDS ? 4 : 1][FL_LDS ? RT * NG : 1][64];
    floatx4* sacc = s_acc[FL_LDS ? wave : 0][0] + lane;  // slot (t, j) of this lane: sacc[(t * NG + j) * 64]
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            acc[t][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            if constexpr (FL_LDS) sacc[(t * NG + j) * 64] = acc[t][j];
            else sum[t][j] = acc[t][j];
        }
    auto flush = [&] {  // the chain so far into the second-level sum (see SART_MF_FLUSH)
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int j = 0; j < NG; ++j) {
                if constexpr (FL_LDS) sacc[(t * NG + j) * 64] += acc[t][j];
                else sum[t][j] += acc[t][j];
                acc[t][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
    };

    const int64_t nst = c1 > c0 ? (c1 - c0) / (32 * KB) : 0;  // uniform for the workgroup
    if (nst > 0) {
        AF a[AS ? 1 : RS][RT][KB];
        u32x4 as_[AS ? RS : 1][NI];
        u32x4 xq[RS][XQ];
        auto piece = [&](int i) { return (C >= 4 ? wave * XQ + i : wave % C); };  // piece = (kb * 2 + plane) * NG + j
        auto load_x = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
#pragma unroll
            for (int i = 0; i < XQ; ++i) {
                const int pc = piece(i), j = pc % NG, plane = (pc / NG) & 1, kb = pc / (2 * NG);
                xq[sl][i] = *reinterpret_cast<const u32x4*>((plane ? Xl : Xh) + xo + (int64_t)j * 16 * xfs + (t * KB + kb) * xbs);
            }
        };
        auto load = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            const int64_t q = t * 32 * KB;
            if constexpr (AS) {
                // full 128-B row segments, 8 rows per instruction: with the non-temporal hint this shape streams at
                // 6.7 TB/s alone, 5.9-6.0 without (profiles/access_probe_r3.jsonl); A is read once per sweep
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    const u32x4* p = reinterpret_cast<const u32x4*>(asp + (int64_t)i * RPI * ld + q);
                    if constexpr (NT_AS) as_[sl][i] = __builtin_nontemporal_load(p);
                    else as_[sl][i] = *p;
                }
            } else {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int kb = 0; kb < KB; ++kb) {
                    if constexpr (A32) {
                        const AT* p = ap + rt * 16 * ld + q + 32 * kb;
                        const u32x4 h0 = *reinterpret_cast<const u32x4*>(p);
                        const u32x4 h1 = *reinterpret_cast<const u32x4*>(p + 16);
                        a[sl][rt][kb] = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
                    } else {
                        a[sl][rt][kb] = *reinterpret_cast<const AF*>(ap + rt * 16 * ld + q + 32 * kb);
                    }
                }
            }
            if constexpr (!EX) load_x(slc, t);
        };
        auto stage = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
#pragma unroll
            for (int i = 0; i < XQ; ++i) s_x[t & 1][piece(i)][lofs] = xq[sl][i];
        };
        if constexpr (EX) {  // X of steps 0 .. DEPTH into slots 0 .. DEPTH, ahead of A's prologue
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (load_x(std::integral_constant<int, Q>{}, Q < nst ? Q : nst - 1), ...);
            }(std::make_integer_sequence<int, RS>{});
        }
        [&]<int... Q>(std::integer_sequence<int, Q...>) {
            (load(std::integral_constant<int, Q>{}, Q < nst ? Q : nst - 1), ...);
        }(std::make_integer_sequence<int, DEPTH>{});
        stage(std::integral_constant<int, 0>{}, 0);
        __syncthreads();
        auto step = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            // EX: X of step t + DEPTH + 1 into this step's slot (X of step t was staged the step before)
            if constexpr (EX) load_x(slc, t + DEPTH + 1 < nst ? t + DEPTH + 1 : nst - 1);
            load(std::integral_constant<int, (sl + DEPTH) % RS>{}, t + DEPTH < nst ? t + DEPTH : nst - 1);
            if (t >= nst) return;  // uniform for the workgroup
            // X of step t + 1 goes into the other stage (its readers passed the last barrier). Split-A stages it AFTER
            // this step's MFMAs (stage_next): its loads were issued with A of step t + 1, and the vmcnt wait the staging
            // needs covers them, so staging first made every step wait for step t + 1's data before computing step t:
            // +3.3 % at 64 frames (9011 -> 9304 frame-it/s); bf16 A measured -0.8 % at 64 frames and equal at 32, so it
            // stages first (profiles/ab_r3_mf_stage_late.jsonl).
            auto stage_next = [&] {
                if constexpr (LATE) __builtin_amdgcn_sched_barrier(0);
                stage(std::integral_constant<int, (sl + 1) % RS>{}, t + 1);
            };
            if constexpr (!LATE && !(ABL & 4)) stage_next();
            const u32x4* xs = s_x[(ABL & 4) ? 0 : (t & 1)][0] + lofs;
            u32x4* img = s_a[AS ? wave : 0];
            if constexpr (AS) {  // this wave's tile into its LDS image (swizzled slots)
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    const int row = i * RPI + lane / R16;
                    img[row * R16 + ((lane % R16) ^ (row & 7))] = as_[sl][i];
                }
            }
            // fragment of tile row block rt, k block kb: (bf16) 8 consecutive voxels; (fp32) the two 16-B halves
            // of the permuted k order
            auto frag16 = [&](int rt, int seg) { return img[(rt * 16 + r) * R16 + (seg ^ (r & 7))]; };
            if constexpr (!A32 && !AS && SART_MF_XF_EARLY) {
                // bf16 A in registers: every X fragment of the step is read from LDS first (KB x 2 planes x NG
                // ds_read_b128), then the MFMAs run with counted waits. Left to itself the scheduler re-used a few
                // registers and issued each read ~4 MFMAs ahead of its use, which at one wave per SIMD exposes the
                // LDS latency before every MFMA group. Same accumulation order: bitwise unchanged.
                u32x4 xf[KB][2][NG];
#pragma unroll
                for (int kb = 0; kb < KB; ++kb)
#pragma unroll
                    for (int pl = 0; pl < 2; ++pl)
#pragma unroll
                        for (int j = 0; j < NG; ++j) xf[kb][pl][j] = xs[((kb * 2 + pl) * NG + j) * 64];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int kb = 0; kb < KB; ++kb)
#pragma unroll
                    for (int j = 0; j < NG; ++j)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) {
                            acc[rt][j] = mfma_b16(a[sl][rt][kb], xf[kb][0][j], acc[rt][j]);
                            acc[rt][j] = mfma_b16(a[sl][rt][kb], xf[kb][1][j], acc[rt][j]);
                        }
                if constexpr (LATE) stage_next();
                __syncthreads();
                return;
            }
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                if constexpr (A32) {
                    u32x4 ah[RT], al[RT];
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) {
                        if constexpr (AS && (ABL & 2)) {
                            ah[rt] = frag16(rt, kb * 8 + g);
                            al[rt] = frag16(rt, kb * 8 + 4 + g);
                        } else {
                            u32x8 v;
                            if constexpr (AS)
                                v = __builtin_shufflevector(frag16(rt, kb * 8 + g), frag16(rt, kb * 8 + 4 + g), 0, 1, 2,
                                                            3, 4, 5, 6, 7);
                            else
                                v = a[sl][rt][kb];
                            if constexpr (H16)
                                split_h8(v, rs[rt], ah[rt], al[rt]);
                            else
                                split_a8(v, ah[rt], al[rt]);
                        }
                    }
                    u32x4 xh[NG], xl[NG];
#pragma unroll
                    for (int j = 0; j < NG; ++j) {
                        xh[j] = xs[((kb * 2 + 0) * NG + j) * 64];
                        xl[j] = xs[((kb * 2 + 1) * NG + j) * 64];
                    }
                    // product-major: consecutive MFMAs write different accumulators (no dependent chains)
                    if constexpr ((ABL & 1) != 0) {
#pragma unroll
                        for (int j = 0; j < NG; ++j)
#pragma unroll
                            for (int rt = 0; rt < RT; ++rt)
                                acc[rt][j][0] += __uint_as_float((al[rt][0] ^ ah[rt][3] ^ xh[j][1] ^ xl[j][2]) & 0x3fffffu);
                    } else {
                    auto mm = [](const u32x4 p, const u32x4 q, floatx4 c) {
                        if constexpr (H16) return mfma_h16(p, q, c);
                        else return mfma_b16(p, q, c);
                    };
#pragma unroll
                    for (int j = 0; j < NG; ++j)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) acc[rt][j] = mm(al[rt], xh[j], acc[rt][j]);
#pragma unroll
                    for (int j = 0; j < NG; ++j)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) acc[rt][j] = mm(ah[rt], xl[j], acc[rt][j]);
#pragma unroll
                    for (int j = 0; j < NG; ++j)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) acc[rt][j] = mm(ah[rt], xh[j], acc[rt][j]);
                    }
                } else if constexpr (AS) {
                    u32x4 af[RT];
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) af[rt] = frag16(rt, kb * 4 + g);
#pragma unroll
                    for (int j = 0; j < NG; ++j) {
                        const u32x4 xh = xs[((kb * 2 + 0) * NG + j) * 64];
                        const u32x4 xl = xs[((kb * 2 + 1) * NG + j) * 64];
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) {
                            acc[rt][j] = mfma_b16(af[rt], xh, acc[rt][j]);
                            acc[rt][j] = mfma_b16(af[rt], xl, acc[rt][j]);
                        }
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < NG; ++j) {
                        const u32x4 xh = xs[((kb * 2 + 0) * NG + j) * 64];
                        const u32x4 xl = xs[((kb * 2 + 1) * NG + j) * 64];
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt) {
                            acc[rt][j] = mfma_b16(a[sl][rt][kb], xh, acc[rt][j]);
                            acc[rt][j] = mfma_b16(a[sl][rt][kb], xl, acc[rt][j]);
                        }
                    }
                }
            }
            if constexpr (ABL & 4) return;
            if constexpr (LATE) stage_next();
            __syncthreads();
        };
        // SART_MF_FLUSH groups of RS steps per trip, then the flush: no branch inside the trip (steps past nst only
        // re-issue the last step's loads, from cache)
        constexpr int FLF = FLUSH > 0 ? FLUSH : 1;
        auto group = [&](int64_t tb) __attribute__((always_inline)) {  // (not inlined: the ring went to scratch)
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (step(std::integral_constant<int, Q>{}, tb + Q), ...);
            }(std::make_integer_sequence<int, RS>{});
        };
        for (int64_t t0 = 0; t0 < nst; t0 += RS * FLF) {
            [&]<int... F>(std::integer_sequence<int, F...>) {
                (group(t0 + F * RS), ...);
            }(std::make_integer_sequence<int, FLF>{});
            if constexpr (FLUSH > 0) flush();
        }
    }
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            if constexpr (FL_LDS) acc[t][j] = sacc[(t * NG + j) * 64] + acc[t][j];
            else acc[t][j] = sum[t][j] + acc[t][j];
        }
    if (!live) return;
    if constexpr (H16) {  // 1 / (s_p s_f), exact (powers of two)
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            const float xi = fc.xinv[16 * j + r];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int64_t ra = row0 + rt * 16 + g * 4 + i;
                    if (ra < nrows) Fout[ra * NF + 16 * j + r] = acc[rt][j][i] * fc.rsc[nrows_pad + ra] * xi;
                }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < NG; ++j)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t ra = row0 + rt * 16 + g * 4 + i;
                if (ra < nrows) Fout[ra * NF + 16 * j + r] = acc[rt][j][i];
            }
}

// partial[s][v][f] = sum_{rows of split s} A[row][v] W[row][f] for the 64-voxel blocks from vb0 up to voxel
// vend; W planes [nf][ldw] (frame-major). Rows are processed up to nrows32 (rows rounded up to 32: the padding
// rows of A and W are zero). One wave: VT blocks of 64 voxels x nf frames (each W fragment feeds 4 VT MFMAs).
template <int NG, int DEPTH, int VT>
__global__ __launch_bounds__(256) void k_mf_backproject_b16(const bf16_t* __restrict__ A, int64_t ld,
                                                            int64_t nrows32, const bf16_t* __restrict__ Wh,
                                                            const bf16_t* __restrict__ Wl, int64_t ldw,
                                                            int64_t rows_per_split, float* __restrict__ partial,
                                                            int64_t vb0, int64_t vend, const int* __restrict__ skip) {
    if (skip && *skip) return;
    constexpr int NF = 16 * NG;
    constexpr int RS = DEPTH + 1;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t vb = (vb0 + (int64_t)blockIdx.x * 4 + wave) * VT;  // first block of 64 voxels
    if (vb * 64 >= vend) return;  // (the range is a multiple of 64 * VT voxels)
    const int g = lane >> 4, i16 = lane & 15;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows32) r_end = nrows32;
    const bf16_t* __restrict__ ap = A + (r_begin + 8 * g) * ld + vb * 64 + 4 * i16;  // + (32 t + j) ld
    const int64_t wo = (int64_t)i16 * ldw + r_begin + 8 * g;                        // + 16 j ldw + 32 t

    floatx4 acc[VT][4][NG];
#pragma unroll
    for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int j = 0; j < NG; ++j) acc[vt][p][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int64_t nst = r_end > r_begin ? (r_end - r_begin) / 32 : 0;
    if (nst > 0) {
        uint2 av[RS][VT][8];
        uint4 wh[RS][NG], wl[RS][NG];
        auto load = [&](int sl, int64_t t) {
            const bf16_t* at = ap + t * 32 * ld;
#pragma unroll
            for (int vt = 0; vt < VT; ++vt)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    av[sl][vt][j] = load_stream(reinterpret_cast<const uint2*>(at + j * ld + vt * 64));
#pragma unroll
            for (int j = 0; j < NG; ++j) {
                wh[sl][j] = *reinterpret_cast<const uint4*>(Wh + wo + (int64_t)j * 16 * ldw + t * 32);
                wl[sl][j] = *reinterpret_cast<const uint4*>(Wl + wo + (int64_t)j * 16 * ldw + t * 32);
            }
        };
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) load(d, d < nst ? d : nst - 1);
        auto step = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            load((sl + DEPTH) % RS, t + DEPTH < nst ? t + DEPTH : nst - 1);
            if (t >= nst) return;
#pragma unroll
            for (int vt = 0; vt < VT; ++vt) {
                const uint4 fr[4] = {phase_frag<0>(av[sl][vt]), phase_frag<1>(av[sl][vt]), phase_frag<2>(av[sl][vt]),
                                     phase_frag<3>(av[sl][vt])};
#pragma unroll
                for (int j = 0; j < NG; ++j)
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        acc[vt][p][j] = mfma_b16(fr[p], wh[sl][j], acc[vt][p][j]);
                        acc[vt][p][j] = mfma_b16(fr[p], wl[sl][j], acc[vt][p][j]);
                    }
            }
        };
        for (int64_t t0 = 0; t0 < nst; t0 += RS) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (step(std::integral_constant<int, Q>{}, t0 + Q), ...);
            }(std::make_integer_sequence<int, RS>{});
        }
    }
    // D: n = frame 16 j + i16, i = (lane >> 4) * 4 + q = voxel slot -> voxel 64 vb + 4 i + p
    float* out = partial + (int64_t)blockIdx.y * ld * NF;
#pragma unroll
    for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t v = (vb + vt) * 64 + 4 * (g * 4 + q) + p;
#pragma unroll
                for (int j = 0; j < NG; ++j) out[v * NF + 16 * j + i16] = acc[vt][p][j][q];
            }
}

// The back-projection with W shared through LDS: the four waves of a workgroup own different voxels of the
// same rows, so they need the same W fragments ([hi, lo][NG][16 frames][32 rows] per step, 1 KiB pieces), loaded
// once per workgroup and staged through two LDS stages like k_mf_forward_b16_lds. Waves past the voxel range
// clamp to the last wave tile of the range (they stage W, take the barriers and store nothing).
// Split-A occupancy: the six-product body takes ~260 registers at NG = 4 (one wave per SIMD); asking for two
// waves per SIMD makes the compiler fit it (tools/probe_mf_x3.py).
template <typename AT, int VT>
constexpr int mf_bwd_min_waves() {
    return std::is_same<AT, float>::value ? (VT == 1 ? 2 : 1) : SART_MF_MINW_BWD;
}

// ABL (diagnostic ablations, tools/probe_mf_x3.py with SART_MF_ABL; 0 in every production launch): bit 0 drops the
// MFMAs (each fragment folds into an accumulator with one VALU op, so no load is dead), bit 1 drops the split of A
// (split-A: the raw bits stand for all three pieces), bit 2 drops the W staging (no LDS writes, no barrier: the step
// re-reads the stage of step 0). Times of the ablated kernels locate the pipe that bounds a step.
// EW (early W): W of step u is loaded one step before A of step u's batch would be (at step u - DEPTH - 1, into ring
// slot u % RS, whose previous W was staged the step before). The wait that staging step t + 1's W needs then covers
// only loads issued at step t - DEPTH or earlier; loaded in one batch with A of step t + 1 (EW false), that wait also
// held every wave until A of step t + 1 had arrived, i.e. one step ahead instead of DEPTH (in-order vmcnt).
template <int NG, int DEPTH, int VT, typename AT = bf16_t, int ABL = 0, bool EW = false>
__global__ __launch_bounds__(256, (NG == 4 ? mf_bwd_min_waves<AT, VT>() : (std::is_same<AT, float>::value && VT == 1 ? 2 : 1))) void k_mf_backproject_b16_lds(const AT* __restrict__ A, int64_t ld,
                                                                int64_t nrows32, const bf16_t* __restrict__ Wh,
                                                                const bf16_t* __restrict__ Wl, int64_t ldw,
                                                                int64_t rows_per_split, float* __restrict__ partial,
                                                                int64_t vb0, int64_t vend, const int* __restrict__ skip) {
    if (skip && *skip) return;
    constexpr int NF = 16 * NG;
    constexpr int RS = DEPTH + 1;
    constexpr bool A32 = std::is_same<AT, float>::value;
    constexpr bool LATE = SART_MF_STAGE_LATE && A32;  // stage_next after the MFMAs (split-A only)
    constexpr int NPL = A32 ? 3 : 2;              // W planes: hi, (mid,) lo
    constexpr int C = NPL * NG;                   // 1 KiB W pieces per step
    constexpr int XQ = C >= 4 ? (C + 3) / 4 : 1;  // pieces per wave (clamped: a duplicate load writes equal data)
    __shared__ __attribute__((aligned(16))) u32x4 s_w[2][C][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t vb = (vb0 + (int64_t)blockIdx.x * 4 + wave) * VT;
    const bool live = vb * 64 < vend;
    if (!live) vb = vend / 64 - VT;  // vend is a multiple of 64 * VT
    const int g = lane >> 4, i16 = lane & 15;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows32) r_end = nrows32;
    const AT* __restrict__ ap = A + (r_begin + 8 * g) * ld + vb * 64 + 4 * i16;
    const int64_t wo = (int64_t)i16 * ldw + r_begin + 8 * g;
    const int lofs = lane;  // lane-linear W slots: conflict-free (see k_mf_forward_b16_lds)
    typedef typename ARaw<AT>::bwd AB;
    // plane pl of frame group j: hi, mid (split-A: stored after hi in Wh), lo
    auto plane_ptr = [&](int pl) { return pl == NPL - 1 ? Wl : Wh + (int64_t)pl * NF * ldw; };

    floatx4 acc[VT][4][NG];
#pragma unroll
    for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int j = 0; j < NG; ++j) acc[vt][p][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int64_t nst = r_end > r_begin ? (r_end - r_begin) / 32 : 0;  // uniform for the workgroup
    if (nst > 0) {
        AB av[RS][VT][8];
        u32x4 wq[RS][XQ];
        auto piece = [&](int i) {  // piece = plane * NG + j
            return C >= 4 ? (wave * XQ + i < C ? wave * XQ + i : C - 1) : wave % C;
        };
        auto load_a = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            const AT* at = ap + t * 32 * ld;
#pragma unroll
            for (int vt = 0; vt < VT; ++vt)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if constexpr (A32)
                        av[sl][vt][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(at + j * ld + vt * 64));
                    else
                        av[sl][vt][j] = load_stream(reinterpret_cast<const uint2*>(at + j * ld + vt * 64));
                }
        };
        auto load_w = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
#pragma unroll
            for (int i = 0; i < XQ; ++i) {
                const int pc = piece(i), j = pc % NG, plane = pc / NG;
                wq[sl][i] = *reinterpret_cast<const u32x4*>(plane_ptr(plane) + wo + (int64_t)j * 16 * ldw + t * 32);
            }
        };
        auto load = [&](auto slc, int64_t t) {
            load_a(slc, t);
            if constexpr (!EW) load_w(slc, t);
        };
        auto stage = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
#pragma unroll
            for (int i = 0; i < XQ; ++i) s_w[t & 1][piece(i)][lofs] = wq[sl][i];
        };
        if constexpr (EW) {  // W of steps 0 .. DEPTH into slots 0 .. DEPTH, ahead of A's prologue
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (load_w(std::integral_constant<int, Q>{}, Q < nst ? Q : nst - 1), ...);
            }(std::make_integer_sequence<int, RS>{});
        }
        [&]<int... Q>(std::integer_sequence<int, Q...>) {
            (load(std::integral_constant<int, Q>{}, Q < nst ? Q : nst - 1), ...);
        }(std::make_integer_sequence<int, DEPTH>{});
        stage(std::integral_constant<int, 0>{}, 0);
        __syncthreads();
        auto step = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            // EW: W of step t + DEPTH + 1 into this step's slot (W of step t was staged the step before)
            if constexpr (EW) load_w(slc, t + DEPTH + 1 < nst ? t + DEPTH + 1 : nst - 1);
            load(std::integral_constant<int, (sl + DEPTH) % RS>{}, t + DEPTH < nst ? t + DEPTH : nst - 1);
            if (t >= nst) return;  // uniform for the workgroup
            auto stage_next = [&] {  // W of step t + 1 after this step's MFMAs (see k_mf_forward_b16_lds)
                if constexpr (LATE) __builtin_amdgcn_sched_barrier(0);
                stage(std::integral_constant<int, (sl + 1) % RS>{}, t + 1);
            };
            if constexpr (!LATE && !(ABL & 4)) stage_next();
            const u32x4* ws = s_w[(ABL & 4) ? 0 : (t & 1)][0] + lofs;
            if constexpr (!A32 && SART_MF_XF_EARLY) {
                // bf16: the step's W fragments are read once for all VT voxel tiles (the loop below re-read them per
                // tile), all before the MFMAs (see k_mf_forward_b16_lds). Same accumulation order.
                u32x4 wf[2][NG];
#pragma unroll
                for (int j = 0; j < NG; ++j) wf[0][j] = ws[j * 64], wf[1][j] = ws[(NG + j) * 64];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int vt = 0; vt < VT; ++vt) {
                    const uint4 fr[4] = {phase_frag<0>(av[sl][vt]), phase_frag<1>(av[sl][vt]),
                                         phase_frag<2>(av[sl][vt]), phase_frag<3>(av[sl][vt])};
#pragma unroll
                    for (int j = 0; j < NG; ++j)
#pragma unroll
                        for (int p = 0; p < 4; ++p) {
                            acc[vt][p][j] = mfma_b16(fr[p], wf[0][j], acc[vt][p][j]);
                            acc[vt][p][j] = mfma_b16(fr[p], wf[1][j], acc[vt][p][j]);
                        }
                }
                if constexpr (LATE) stage_next();
                __syncthreads();
                return;
            }
#pragma unroll
            for (int vt = 0; vt < VT; ++vt) {
                if constexpr (A32) {
                    // six products: every piece pair of combined weight >= 2^-16 (hi, mid, lo of A and of W),
                    // smallest first into the accumulator
                    u32x4 fh[4], fm[4], fl[4];
                    if constexpr ((ABL & 2) != 0) {
#pragma unroll
                        for (int p = 0; p < 4; ++p) {
                            const u32x4 raw = {av[sl][vt][0][p], av[sl][vt][2][p], av[sl][vt][4][p], av[sl][vt][6][p]};
                            fh[p] = raw, fm[p] = raw, fl[p] = raw;
                        }
                    } else {
                        split_phase3<0>(av[sl][vt], fh[0], fm[0], fl[0]);
                        split_phase3<1>(av[sl][vt], fh[1], fm[1], fl[1]);
                        split_phase3<2>(av[sl][vt], fh[2], fm[2], fl[2]);
                        split_phase3<3>(av[sl][vt], fh[3], fm[3], fl[3]);
                    }
                    u32x4 wv[3][NG];
#pragma unroll
                    for (int j = 0; j < NG; ++j)
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) wv[pl][j] = ws[(pl * NG + j) * 64];
                    // product-major: consecutive MFMAs write different accumulators (no dependent chains); a
                    // phase-major order (split one phase, then its 6 x NG MFMAs) measured 0.6-1 % slower
                    // (profiles/ab_r2_mf_phase_major_negative.jsonl)
                    auto prod = [&](const u32x4(&fa)[4], int pl) {
#pragma unroll
                        for (int j = 0; j < NG; ++j)
#pragma unroll
                            for (int p = 0; p < 4; ++p) {
                                if constexpr ((ABL & 1) != 0)
                                    acc[vt][p][j][0] += __uint_as_float((fa[p][0] ^ fa[p][3] ^ wv[pl][j][1]) & 0x3fffffu);
                                else
                                    acc[vt][p][j] = mfma_b16(fa[p], wv[pl][j], acc[vt][p][j]);
                            }
                    };
                    prod(fh, 2);
                    prod(fm, 1);
                    prod(fl, 0);
                    prod(fh, 1);
                    prod(fm, 0);
                    prod(fh, 0);
                } else {
                    const uint4 fr[4] = {phase_frag<0>(av[sl][vt]), phase_frag<1>(av[sl][vt]),
                                         phase_frag<2>(av[sl][vt]), phase_frag<3>(av[sl][vt])};
#pragma unroll
                    for (int j = 0; j < NG; ++j) {
                        const u32x4 wh = ws[j * 64], wl = ws[(NG + j) * 64];
#pragma unroll
                        for (int p = 0; p < 4; ++p) {
                            acc[vt][p][j] = mfma_b16(fr[p], wh, acc[vt][p][j]);
                            acc[vt][p][j] = mfma_b16(fr[p], wl, acc[vt][p][j]);
                        }
                    }
                }
            }
            if constexpr (ABL & 4) return;
            if constexpr (LATE) stage_next();
            __syncthreads();
        };
        for (int64_t t0 = 0; t0 < nst; t0 += RS) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (step(std::integral_constant<int, Q>{}, t0 + Q), ...);
            }(std::make_integer_sequence<int, RS>{});
        }
    }
    if (!live) return;
    float* out = partial + (int64_t)blockIdx.y * ld * NF;
#pragma unroll
    for (int vt = 0; vt < VT; ++vt)
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t v = (vb + vt) * 64 + 4 * (g * 4 + q) + p;
#pragma unroll
                for (int j = 0; j < NG; ++j) out[v * NF + 16 * j + i16] = acc[vt][p][j][q];
            }
}

// ---------------------------------------------------------------------------------------------- launchers

// ----------------------------------------------------------------------------------------------------------------
// Split-A back-projection on f16 pairs (SART_MF_BWD16, default for fp32 shards at 32 / 64 / 128 frames). fp16 has
// 11 significant bits, so two rne pieces hold a scaled fp32 value to ~2^-22 (|a s - a1| <= 2^-11 |a s|, |a s - a1 -
// a2| <= 2^-11 |a s - a1|), where bf16 (8 bits) needs three pieces for the same. Two pieces of A s_v and of W s_f
// make three products (a2 w1, a1 w2, a1 w1; the dropped a2 w2 is ~2^-22 of a term) instead of the six of the bf16
// split, and the split is 3 VALU operations per element (scale, convert, residual) instead of 5.5. Not fp32-exact:
// ~2^-22 per product against fp32's 2^-24. The scales are powers of two: s_v per voxel COLUMN (max_p |A[p][v]|,
// launch_mf_col_scales: a column's entries within 2^-16 of its own maximum keep both pieces normal, whatever the
// range across columns; multiframe_glue.hip) and s_f per frame and sweep (launch_mf_split_w16); the epilogue
// multiplies by inv_scale[f] = 1 / s_f and 1 / s_v, exactly. Layout and staging as k_mf_backproject_b16_lds (VT = 1).
template <int P>
__device__ __forceinline__ void split_phase_h(const u32x4 (&v)[8], float s, u32x4& h1, u32x4& h2) {
    unsigned a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) split_h2(v[2 * q][P], v[2 * q + 1][P], s, a[q], b[q]);
    h1 = u32x4{a[0], a[1], a[2], a[3]};
    h2 = u32x4{b[0], b[1], b[2], b[3]};
}

// Two-level accumulation of the back-projection's split-K sums through LDS: every SART_MF_BWD_FLUSH outer iterations
// (of DEPTH + 1 steps of 32 rows) a lane adds its accumulators into its own LDS slots and restarts them, so no fp32
// MFMA chain runs over a whole split (a second register set spilled: 64 / 128 more VGPRs). Slots are lane-private
// (no barrier, no atomics): 16 NG KiB per wave, 64 / 128 KiB per workgroup at 64 / 128 frames beside the 16 / 32 KiB
// W stage (two workgroups per CU at 64 frames, one at 128: the occupancy the registers allow anyway). 0 disables
// (A/B builds); the split count then has to shorten the chains instead (SART_MF_BP_BLOCKS).
#ifndef SART_MF_BWD_FLUSH
#define SART_MF_BWD_FLUSH 4
#endif

// EW: W loaded a step ahead of A's batch (see k_mf_backproject_b16_lds); MW: waves per SIMD of the register budget
template <int NG, int DEPTH, bool EW = false, int MW = 2>
__global__ __launch_bounds__(256, MW) void k_mf_backproject_h16(const float* __restrict__ A, int64_t ld, int64_t nrows32,
                                                               const uint16_t* __restrict__ W1,
                                                               const uint16_t* __restrict__ W2, int64_t ldw,
                                                               int64_t rows_per_split, float* __restrict__ partial,
                                                               int64_t vb0, int64_t vend,
                                                               const float* __restrict__ csc,
                                                               const float* __restrict__ inv_scale,
                                                               const int* __restrict__ skip) {
    if (skip && *skip) return;
    constexpr int NF = 16 * NG;
    constexpr int RS = DEPTH + 1;
    constexpr int C = 2 * NG;                     // 1 KiB W pieces per step: (plane, frame group)
    constexpr int XQ = C >= 4 ? (C + 3) / 4 : 1;  // pieces per wave
    __shared__ __attribute__((aligned(16))) u32x4 s_w[2][C][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t vb = vb0 + (int64_t)blockIdx.x * 4 + wave;
    const bool live = vb * 64 < vend;
    if (!live) vb = vend / 64 - 1;  // vend is a multiple of 64
    const int g = lane >> 4, i16 = lane & 15;
    const int64_t r_begin = (int64_t)blockIdx.y * rows_per_split;
    int64_t r_end = r_begin + rows_per_split;
    if (r_end > nrows32) r_end = nrows32;
    const float* __restrict__ ap = A + (r_begin + 8 * g) * ld + vb * 64 + 4 * i16;
    const int64_t wo = (int64_t)i16 * ldw + r_begin + 8 * g;
    const float4 cs4 = *reinterpret_cast<const float4*>(csc + vb * 64 + 4 * i16);  // scales of voxel phases 0..3
    floatx4 acc[4][NG];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int j = 0; j < NG; ++j) acc[p][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int FLB = SART_MF_BWD_FLUSH;
    __shared__ __attribute__((aligned(16))) floatx4 s_acc[FLB > 0 ? 4 : 1][FLB > 0 ? 4 * NG : 1][64];
    floatx4* sacc = s_acc[FLB > 0 ? wave : 0][0] + lane;  // slot k of this lane: sacc[k * 64]
    if constexpr (FLB > 0) {
#pragma unroll
        for (int k = 0; k < 4 * NG; ++k) sacc[k * 64] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    auto flush = [&] {
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int j = 0; j < NG; ++j) {
                sacc[(p * NG + j) * 64] += acc[p][j];
                acc[p][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
    };
    const int64_t nst = r_end > r_begin ? (r_end - r_begin) / 32 : 0;  // uniform for the workgroup
    if (nst > 0) {
        u32x4 av[RS][8];
        u32x4 wq[RS][XQ];
        auto piece = [&](int i) { return C >= 4 ? (wave * XQ + i < C ? wave * XQ + i : C - 1) : wave % C; };
        auto load_w = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
#pragma unroll
            for (int i = 0; i < XQ; ++i) {
                const int pc = piece(i), j = pc % NG, plane = pc / NG;
                wq[sl][i] = *reinterpret_cast<const u32x4*>((plane ? W2 : W1) + wo + (int64_t)j * 16 * ldw + t * 32);
            }
        };
        auto load = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            const float* at = ap + t * 32 * ld;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                av[sl][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(at + j * ld));
            if constexpr (!EW) load_w(slc, t);
        };
        auto stage = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
#pragma unroll
            for (int i = 0; i < XQ; ++i) s_w[t & 1][piece(i)][lane] = wq[sl][i];
        };
        if constexpr (EW) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (load_w(std::integral_constant<int, Q>{}, Q < nst ? Q : nst - 1), ...);
            }(std::make_integer_sequence<int, RS>{});
        }
        [&]<int... Q>(std::integer_sequence<int, Q...>) {
            (load(std::integral_constant<int, Q>{}, Q < nst ? Q : nst - 1), ...);
        }(std::make_integer_sequence<int, DEPTH>{});
        stage(std::integral_constant<int, 0>{}, 0);
        __syncthreads();
        auto step = [&](auto slc, int64_t t) {
            constexpr int sl = decltype(slc)::value;
            if constexpr (EW) load_w(slc, t + DEPTH + 1 < nst ? t + DEPTH + 1 : nst - 1);
            load(std::integral_constant<int, (sl + DEPTH) % RS>{}, t + DEPTH < nst ? t + DEPTH : nst - 1);
            if (t >= nst) return;  // uniform for the workgroup
            const u32x4* ws = s_w[t & 1][0] + lane;
            u32x4 h1[4], h2[4];
            split_phase_h<0>(av[sl], cs4.x, h1[0], h2[0]);
            split_phase_h<1>(av[sl], cs4.y, h1[1], h2[1]);
            split_phase_h<2>(av[sl], cs4.z, h1[2], h2[2]);
            split_phase_h<3>(av[sl], cs4.w, h1[3], h2[3]);
            u32x4 wv[2][NG];
#pragma unroll
            for (int j = 0; j < NG; ++j) wv[0][j] = ws[j * 64], wv[1][j] = ws[(NG + j) * 64];
            auto prod = [&](const u32x4(&fa)[4], int pl) {
#pragma unroll
                for (int j = 0; j < NG; ++j)
#pragma unroll
                    for (int p = 0; p < 4; ++p) acc[p][j] = mfma_h16(fa[p], wv[pl][j], acc[p][j]);
            };
            prod(h2, 0);  // smallest first: a2 w1, a1 w2, a1 w1
            prod(h1, 1);
            prod(h1, 0);
            __builtin_amdgcn_sched_barrier(0);
            stage(std::integral_constant<int, (sl + 1) % RS>{}, t + 1);
            __syncthreads();
        };
        for (int64_t t0 = 0, it = 0; t0 < nst; t0 += RS, ++it) {
            [&]<int... Q>(std::integer_sequence<int, Q...>) {
                (step(std::integral_constant<int, Q>{}, t0 + Q), ...);
            }(std::make_integer_sequence<int, RS>{});
            if constexpr (FLB > 0)
                if (it % FLB == FLB - 1) flush();
        }
    }
    if constexpr (FLB > 0) {  // the LDS sum plus the chain since the last flush
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int j = 0; j < NG; ++j) acc[p][j] = sacc[(p * NG + j) * 64] + acc[p][j];
    }
    if (!live) return;
    float* out = partial + (int64_t)blockIdx.y * ld * NF;
    float isc[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) isc[j] = inv_scale[16 * j + i16];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t v = vb * 64 + 4 * (g * 4 + q) + p;
            const float iv = csc[ld + v];
#pragma unroll
            for (int j = 0; j < NG; ++j) out[v * NF + 16 * j + i16] = acc[p][j][q] * isc[j] * iv;
        }
}

// split128: the split-A forward and the f16-pair back-projection also take 128 frames (8 column groups)
static void check_nf_b16(int nf, const char* what, bool split128 = false) {
    if (nf == 128 && split128) return;
    if (nf != 16 && nf != 32 && nf != 64)
        throw std::runtime_error(std::string(what) + (split128 ? ": nf must be 16, 32, 64 or 128" : ": nf must be 16, 32 or 64"));
}

// Tunables (tools/probe_mf_b16.py): register-ring depth (SART_MF_DEPTH 1..3), forward tile (SART_MF_B16_FWD =
// "RT,KB": 16-row tiles per wave and 32-voxel blocks per step) and back-projection voxel blocks per wave
// (SART_MF_B16_VT 1 or 2). Defaults below from the probe at 64k x 64k (profiles/probe_r2_mf_b16.jsonl).
static int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return (e && *e) ? std::atoi(e) : dflt;
}

static int mf_b16_depth(bool forward, int nf) {
    const int d = env_int("SART_MF_DEPTH", 0);
    if (d >= 1 && d <= 3) return d;
    (void)forward;
    (void)nf;
    return 3;  // profiles/probe_r2_mf_b16_bwd.jsonl
}

struct FwdTile {
    int rt, kb;
    bool lds = false;  // X shared through LDS (k_mf_forward_b16_lds)
    bool as = false;   // A staged through LDS in full row segments (LDS kernel, 128-B rows: bf16 KB = 2, fp32)
};
static FwdTile mf_b16_fwd_tile(int nf) {
    const char* e = std::getenv("SART_MF_B16_FWD");
    if (e && *e) {
        // "RT,KB" or "RT,KB,lds"
        FwdTile t{std::atoi(e), std::strchr(e, ',') ? std::atoi(std::strchr(e, ',') + 1) : 1};
        t.lds = std::strstr(e, "lds") != nullptr;
        t.as = std::strstr(e, "as") != nullptr;  // "RT,2,lds,as": A staged through LDS (KB = 2 only)
        if ((t.rt == 2 || t.rt == 4 || t.rt == 8) && (t.kb == 1 || t.kb == 2)) return t;
    }
    // profiles/probe_r2_mf_b16_lds.jsonl, profiles/probe_r2_mf_as.jsonl (A staged: +9 % at 32 frames, a tie at 16 / 64)
    if (nf == 32) return FwdTile{2, 2, true, true};
    return nf == 16 ? FwdTile{2, 2, true} : FwdTile{4, 2, true};
}

static int mf_b16_vt(int64_t ld, int nf) {
    if (nf == 128) return 1;  // 8 column groups: one 64-voxel tile per wave
    const int v = env_int("SART_MF_B16_VT", 0);
    const int vt = (v == 1 || v == 2) ? v : 2;
    return (vt == 2 && ld % 128 == 0) ? 2 : 1;
}

// W shared through LDS in the back-projection (k_mf_backproject_b16_lds): SART_MF_B16_VT = "VT,lds" / "VT,reg"
static bool mf_b16_bwd_lds(int nf) {
    const char* e = std::getenv("SART_MF_B16_VT");
    if (e && std::strstr(e, "lds")) return true;
    if (e && std::strstr(e, "reg")) return false;
    (void)nf;
    return true;
}

template <int NG, int DEPTH, int RT, int KB, typename AT>
static void fwd_b16_t(FwdTile tl, dim3 grid, hipStream_t stream, const AT* A, int64_t ld, int64_t nrows,
                      int64_t nrows_pad, const bf16_t* Xh, const bf16_t* Xl, float* Fout, FwdCols cps) {
    constexpr bool A32 = std::is_same<AT, float>::value;
    constexpr bool CAN_AS = A32 || KB == 2;  // full 128-B row segments per step
    if constexpr (A32 && NG == 4 && DEPTH == 3 && RT == 2 && KB == 1) {
        const int abl = env_int("SART_MF_ABL", 0);  // diagnostics only (tools/probe_mf_abl.py)
        if (abl > 0 && tl.as) {
            auto go = [&](auto k) {
                hipLaunchKernelGGL((k_mf_forward_b16_lds<NG, DEPTH, RT, KB, AT, true, decltype(k)::value>), grid,
                                   dim3(256), 0, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps, g_mf_skip);
            };
            switch (abl & 7) {
                case 1: go(std::integral_constant<int, 1>{}); break;
                case 2: go(std::integral_constant<int, 2>{}); break;
                case 3: go(std::integral_constant<int, 3>{}); break;
                case 4: go(std::integral_constant<int, 4>{}); break;
                case 5: go(std::integral_constant<int, 5>{}); break;
                case 6: go(std::integral_constant<int, 6>{}); break;
                default: go(std::integral_constant<int, 7>{}); break;
            }
            return;
        }
    }
    // SART_MF_XEARLY=0 / 1: X loaded with A / a step earlier (A/B runs). Default: split-A only (+0.3 %; bf16 storage
    // -2.7 %, profiles/ab_r4_mf_early_operands.jsonl)
    const bool ex = env_int("SART_MF_XEARLY", A32 ? 1 : 0) != 0;
    if constexpr (CAN_AS) {
        if (tl.as) {
            if (ex)
                hipLaunchKernelGGL((k_mf_forward_b16_lds<NG, DEPTH, RT, KB, AT, true, 0, true>), grid, dim3(256), 0,
                                   stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps, g_mf_skip);
            else
                hipLaunchKernelGGL((k_mf_forward_b16_lds<NG, DEPTH, RT, KB, AT, true>), grid, dim3(256), 0, stream, A,
                                   ld, nrows, nrows_pad, Xh, Xl, Fout, cps, g_mf_skip);
            return;
        }
    }
    if ((A32 || tl.lds) && ex) {
        hipLaunchKernelGGL((k_mf_forward_b16_lds<NG, DEPTH, RT, KB, AT, false, 0, true>), grid, dim3(256), 0, stream, A,
                           ld, nrows, nrows_pad, Xh, Xl, Fout, cps, g_mf_skip);
    } else if (A32 || tl.lds) {  // split-A: the LDS kernels only
        hipLaunchKernelGGL((k_mf_forward_b16_lds<NG, DEPTH, RT, KB, AT>), grid, dim3(256), 0, stream, A, ld, nrows,
                           nrows_pad, Xh, Xl, Fout, cps, g_mf_skip);
    } else if constexpr (!A32) {
        hipLaunchKernelGGL((k_mf_forward_b16<NG, DEPTH, RT, KB>), grid, dim3(256), 0, stream, A, ld, nrows, nrows_pad,
                           Xh, Xl, Fout, cps, g_mf_skip);
    }
}

template <int NG, int DEPTH, typename AT>
static void fwd_b16_d(FwdTile tl, dim3 grid, hipStream_t stream, const AT* A, int64_t ld, int64_t nrows,
                      int64_t nrows_pad, const bf16_t* Xh, const bf16_t* Xl, float* Fout, FwdCols cps) {
    if (tl.rt == 2 && tl.kb == 2)
        fwd_b16_t<NG, DEPTH, 2, 2>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    else if (tl.rt == 4 && tl.kb == 2)
        fwd_b16_t<NG, DEPTH, 4, 2>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    else if (tl.rt == 2)
        fwd_b16_t<NG, DEPTH, 2, 1>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    else if constexpr (!std::is_same<AT, float>::value) {
        if (tl.rt == 8)
            fwd_b16_t<NG, DEPTH, 8, 1>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
        else
            fwd_b16_t<NG, DEPTH, 4, 1>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    } else {
        fwd_b16_t<NG, DEPTH, 4, 1>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    }
}

template <int NG, typename AT>
static void fwd_b16(int depth, FwdTile tl, dim3 grid, hipStream_t stream, const AT* A, int64_t ld, int64_t nrows,
                    int64_t nrows_pad, const bf16_t* Xh, const bf16_t* Xl, float* Fout, FwdCols cps) {
    if constexpr (!std::is_same<AT, float>::value) {
        if (depth == 1) {
            fwd_b16_d<NG, 1>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
            return;
        }
    }
    if (depth <= 2)
        fwd_b16_d<NG, 2>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    else
        fwd_b16_d<NG, 3>(tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
}

// Split-A tunables (fp32 A on the bf16 matrix cores): SART_MF_X3_FWD = "RT,KB", SART_MF_X3_VT = VT (1 or 2),
// SART_MF_X3_DEPTH (2 or 3). Twice the bytes of A per fragment as bf16 storage, so smaller register tiles.
static FwdTile mf_x3_fwd_tile(int nf, int64_t ld) {
    const char* e = std::getenv("SART_MF_X3_FWD");
    if (e && *e) {
        FwdTile t{std::atoi(e), std::strchr(e, ',') ? std::atoi(std::strchr(e, ',') + 1) : 1, true};
        t.as = std::strstr(e, "as") != nullptr;  // "RT,KB,as": A staged through LDS
        if ((t.rt == 2 || t.rt == 4) && (t.kb == 1 || t.kb == 2)) return t;
    }
    // profiles/probe_r2_mf_x3.jsonl, profiles/probe_r2_mf_as.jsonl; with blocked X planes (round 4,
    // profiles/probe_r4_mf_x3_fwd_tiles_xblk.jsonl) 64 frames on rows of >= 128k columns take two 32-voxel blocks per
    // step (16384 x 262144: 3.08 against 3.21 ms; 64k x 64k: 2.96 against 2.90, so narrower rows keep one)
    // 32 frames take the A-staged tile too since its loads are non-temporal (+3.2 % at 64k x 64k,
    // profiles/ab_r5_mf32_as.txt)
    if (nf == 64 || nf == 32) return ld >= 131072 ? FwdTile{2, 2, true, true} : FwdTile{2, 1, true, true};
    if (nf == 128) return FwdTile{2, 1, true, true};  // 128 frames: one 32-voxel block per step (registers)
    return FwdTile{2, 2, true};
}
static int mf_x3_depth(bool forward) {
    // the forward's ring: 2 steps ahead on blocked X planes (64k x 64k: 2.90 against 2.98 ms at 3, 16384 x 262144
    // equal; profiles/probe_r4_mf_x3_fwd_tiles_xblk.jsonl)
    (void)forward;
    const int d = env_int("SART_MF_X3_DEPTH", 0);
    return (d == 2 || d == 3) ? d : 2;
}
static int mf_x3_vt(int64_t ld) {
    const int v = env_int("SART_MF_X3_VT", 0);
    const int vt = (v == 1 || v == 2) ? v : 1;
    return (vt == 2 && ld % 128 == 0) ? 2 : 1;
}

template <typename AT>
static void launch_mf_forward_split(const AT* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const bf16_t* Xh,
                                    const bf16_t* Xl, float* Fout, int nsplit, int nf, hipStream_t stream,
                                    bool xblk) {
    constexpr bool A32 = std::is_same<AT, float>::value;
    const char* what = A32 ? "mf_forward_x3" : "mf_forward_b16";
    if (ld % 64 != 0) throw std::runtime_error(std::string(what) + ": ld must be a multiple of 64");
    if (nsplit < 1) throw std::runtime_error(std::string(what) + ": nsplit must be >= 1");
    check_nf_b16(nf, what, true);
    if (nrows_pad % 32 != 0) throw std::runtime_error(std::string(what) + ": padded rows must be a multiple of 32");
    FwdTile tl = A32 ? mf_x3_fwd_tile(nf, ld) : mf_b16_fwd_tile(nf);
    if (nrows_pad % (16 * tl.rt) != 0) tl = FwdTile{2, 1, tl.lds, A32 && tl.as};  // a wave's rows inside the padding
    // the 128-frame tilings (see below); bf16 storage stages A through LDS (+3.8 %, profiles/ab_r4_mfb128_variants.jsonl)
    if (nf == 128) tl = FwdTile{2, A32 ? tl.kb : 2, true, true};
    const FwdCols cps{((ld + nsplit - 1) / nsplit + 63) / 64 * 64, xblk ? 32 : ld, xblk ? 32 * (int64_t)nf : 32};
    const int64_t rows_per_block = 64 * tl.rt;
    const dim3 grid((unsigned)((nrows_pad + rows_per_block - 1) / rows_per_block), (unsigned)nsplit);
    const int d = A32 ? mf_x3_depth(true) : mf_b16_depth(true, nf);
    if constexpr (A32) {
        if (nf == 128) {  // 8 column groups (64 accumulator registers at RT = 2): A staged, X early
            auto run = [&](auto kern) {
                hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps,
                                   g_mf_skip);
            };
            if (tl.kb == 2 && d == 3) run(k_mf_forward_b16_lds<8, 3, 2, 2, float, true, 0, true>);
            else if (tl.kb == 2) run(k_mf_forward_b16_lds<8, 2, 2, 2, float, true, 0, true>);
            else if (d == 3) run(k_mf_forward_b16_lds<8, 3, 2, 1, float, true, 0, true>);
            else run(k_mf_forward_b16_lds<8, 2, 2, 1, float, true, 0, true>);
            check_launch("k_mf_forward_x3");
            return;
        }
    }
    if constexpr (!A32) {
        if (nf == 128) {  // bf16 storage, 128 frames: 8 column groups, RT = 2, two 32-voxel blocks per step, X in LDS
            auto run = [&](auto kern) {
                hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps,
                                   g_mf_skip);
            };
            if (tl.as && d >= 3) run(k_mf_forward_b16_lds<8, 3, 2, 2, bf16_t, true>);
            else if (tl.as) run(k_mf_forward_b16_lds<8, 2, 2, 2, bf16_t, true>);
            else if (d >= 3) run(k_mf_forward_b16_lds<8, 3, 2, 2, bf16_t>);
            else run(k_mf_forward_b16_lds<8, 2, 2, 2, bf16_t>);
            check_launch("k_mf_forward_b16");
            return;
        }
    }
    if (nf == 16)
        fwd_b16<1>(d, tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    else if (nf == 32)
        fwd_b16<2>(d, tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    else
        fwd_b16<4>(d, tl, grid, stream, A, ld, nrows, nrows_pad, Xh, Xl, Fout, cps);
    check_launch(A32 ? "k_mf_forward_x3" : "k_mf_forward_b16");
}

void launch_mf_forward_b16(const bf16_t* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const bf16_t* Xh,
                           const bf16_t* Xl, float* Fout, int nsplit, int nf, hipStream_t stream, bool xblk) {
    launch_mf_forward_split(A, ld, nrows, nrows_pad, Xh, Xl, Fout, nsplit, nf, stream, xblk);
}

void launch_mf_forward_x3(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const bf16_t* Xh,
                          const bf16_t* Xl, float* Fout, int nsplit, int nf, hipStream_t stream, bool xblk) {
    launch_mf_forward_split(A, ld, nrows, nrows_pad, Xh, Xl, Fout, nsplit, nf, stream, xblk);
}

// The f16-pair split-A forward (H16; default for fp32 shards at 32 / 64 / 128 frames): the x3 tilings with RT = 2 and
// a ring two steps deep, X loaded early; planes from launch_mf_split_x16 with perm (and blocked when xblk).
template <int NG>
static void fwd_h16_ng(const FwdTile& tl, dim3 grid, hipStream_t stream, const float* A, int64_t ld, int64_t nrows,
                       int64_t nrows_pad, const bf16_t* X1, const bf16_t* X2, float* Fout, FwdCols cps) {
    auto run = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, A, ld, nrows, nrows_pad, X1, X2, Fout, cps, g_mf_skip);
    };
    // SART_MF_H16_FDEPTH=3: a register ring three steps deep for the A-staged tilings (A/B runs)
    if (tl.as && env_int("SART_MF_H16_FDEPTH", 2) == 3) {
        if (tl.kb == 2) run(k_mf_forward_b16_lds<NG, 3, 2, 2, float, true, 0, true, true>);
        else run(k_mf_forward_b16_lds<NG, 3, 2, 1, float, true, 0, true, true>);
        return;
    }
    if (tl.kb == 2 && tl.as) run(k_mf_forward_b16_lds<NG, 2, 2, 2, float, true, 0, true, true>);
    else if (tl.kb == 2) run(k_mf_forward_b16_lds<NG, 2, 2, 2, float, false, 0, true, true>);
    else if (tl.as) run(k_mf_forward_b16_lds<NG, 2, 2, 1, float, true, 0, true, true>);
    else run(k_mf_forward_b16_lds<NG, 2, 2, 1, float, false, 0, true, true>);
}

void launch_mf_forward_h16(const float* A, int64_t ld, int64_t nrows, int64_t nrows_pad, const uint16_t* X1,
                           const uint16_t* X2, float* Fout, int nsplit, int nf, hipStream_t stream, bool xblk,
                           const float* rsc, const float* xinv) {
    const char* what = "mf_forward_h16";
    if (ld % 64 != 0) throw std::runtime_error(std::string(what) + ": ld must be a multiple of 64");
    if (nsplit < 1) throw std::runtime_error(std::string(what) + ": nsplit must be >= 1");
    check_nf_b16(nf, what, true);
    if (nrows_pad % 64 != 0) throw std::runtime_error(std::string(what) + ": padded rows must be a multiple of 64");
    if (!rsc || !xinv) throw std::runtime_error(std::string(what) + ": row scales and frame scales required");
    FwdTile tl = mf_x3_fwd_tile(nf, ld);
    if (nf == 128) tl.as = true;
    FwdCols cps{((ld + nsplit - 1) / nsplit + 63) / 64 * 64, xblk ? 32 : ld, xblk ? 32 * (int64_t)nf : 32};
    cps.rsc = rsc;
    cps.xinv = xinv;
    const dim3 grid((unsigned)((nrows_pad + 127) / 128), (unsigned)nsplit);  // 4 waves x 32 rows per workgroup
    const bf16_t* x1 = reinterpret_cast<const bf16_t*>(X1);
    const bf16_t* x2 = reinterpret_cast<const bf16_t*>(X2);
    if (nf == 16) fwd_h16_ng<1>(tl, grid, stream, A, ld, nrows, nrows_pad, x1, x2, Fout, cps);
    else if (nf == 32) fwd_h16_ng<2>(tl, grid, stream, A, ld, nrows, nrows_pad, x1, x2, Fout, cps);
    else if (nf == 64) fwd_h16_ng<4>(tl, grid, stream, A, ld, nrows, nrows_pad, x1, x2, Fout, cps);
    else fwd_h16_ng<8>(tl, grid, stream, A, ld, nrows, nrows_pad, x1, x2, Fout, cps);
    check_launch("k_mf_forward_h16");
}

// Split-K of the bf16 / split-A back-projection: ~1024 workgroups (4 waves x 64 VT voxels each), >= 64 rows per
// split.
int mf_backproject_b16_num_splits(int64_t ld, int64_t nrows, bool a32) {
    const int64_t nblk = (ld / (64 * (a32 ? mf_x3_vt(ld) : mf_b16_vt(ld, 0))) + 3) / 4;
    // bf16 storage: ~512 (fewer partial slices for k_mf_collect: +1.3 % with 512-block forwards at 64 frames,
    // profiles/ab_r4_mf_split_blocks_low.jsonl); split-A ~1024 (256: -5 %)
    // x 4 in round 6 (split-A 4096, bf16 storage 2048): each split's rows are one fp32 MFMA accumulation chain, the
    // larger share of the engine's error against the fp32 two-pass kernels at 64k x 64k (16k-row chains;
    // profiles/parity_r6_64k_mf_chains.jsonl)
    // (split-A with the LDS two-level sums of k_mf_backproject_h16: back to ~1024, chains of 12 steps)
    const int64_t target = env_int("SART_MF_BP_BLOCKS", a32 ? (SART_MF_BWD_FLUSH > 0 ? 1024 : 4096) : 2048);
    int64_t s = (target + nblk - 1) / nblk;
    const int64_t smax = (nrows + 63) / 64;
    if (s > smax) s = smax;
    if (s < 1) s = 1;
    return (int)s;
}

int mf_backproject_b16_vox_align(int64_t ld, bool a32) { return 64 * (a32 ? mf_x3_vt(ld) : mf_b16_vt(ld, 0)); }

template <int NG, int DEPTH, typename AT>
static void bwd_b16_d(int vt, dim3 grid, hipStream_t stream, const AT* A, int64_t ld, int64_t nrows32,
                      const bf16_t* Wh, const bf16_t* Wl, int64_t ldw, int64_t rps, float* partial, int64_t vb0,
                      int64_t vend) {
    if constexpr (std::is_same<AT, float>::value && NG == 4 && DEPTH == 2) {
        const int abl = env_int("SART_MF_ABL", 0);  // diagnostics only (tools/probe_mf_abl.py; read per launch)
        if (abl > 0 && vt == 1) {
            auto go = [&](auto k) {
                hipLaunchKernelGGL((k_mf_backproject_b16_lds<NG, DEPTH, 1, AT, decltype(k)::value>), grid, dim3(256), 0,
                                   stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vb0, vend, g_mf_skip);
            };
            switch (abl & 7) {
                case 1: go(std::integral_constant<int, 1>{}); break;
                case 2: go(std::integral_constant<int, 2>{}); break;
                case 3: go(std::integral_constant<int, 3>{}); break;
                case 4: go(std::integral_constant<int, 4>{}); break;
                case 5: go(std::integral_constant<int, 5>{}); break;
                case 6: go(std::integral_constant<int, 6>{}); break;
                default: go(std::integral_constant<int, 7>{}); break;
            }
            return;
        }
    }
    if (std::is_same<AT, float>::value || mf_b16_bwd_lds(16 * NG)) {
        // SART_MF_WEARLY=0 / 1: W loaded in one batch with A / one step earlier (A/B runs; read per launch). Default
        // on for bf16 storage (+0.9 %); off for split-A, whose two-waves-per-SIMD budget spills 40 VGPRs with the extra
        // W slot (-12 %, profiles/ab_r4_mf_early_operands.jsonl)
        if (env_int("SART_MF_WEARLY", std::is_same<AT, float>::value ? 0 : 1) != 0) {
            if (vt == 2)
                hipLaunchKernelGGL((k_mf_backproject_b16_lds<NG, DEPTH, 2, AT, 0, true>), grid, dim3(256), 0, stream, A,
                                   ld, nrows32, Wh, Wl, ldw, rps, partial, vb0, vend, g_mf_skip);
            else
                hipLaunchKernelGGL((k_mf_backproject_b16_lds<NG, DEPTH, 1, AT, 0, true>), grid, dim3(256), 0, stream, A,
                                   ld, nrows32, Wh, Wl, ldw, rps, partial, vb0, vend, g_mf_skip);
            return;
        }
        if (vt == 2)
            hipLaunchKernelGGL((k_mf_backproject_b16_lds<NG, DEPTH, 2, AT>), grid, dim3(256), 0, stream, A, ld,
                               nrows32, Wh, Wl, ldw, rps, partial, vb0, vend, g_mf_skip);
        else
            hipLaunchKernelGGL((k_mf_backproject_b16_lds<NG, DEPTH, 1, AT>), grid, dim3(256), 0, stream, A, ld,
                               nrows32, Wh, Wl, ldw, rps, partial, vb0, vend, g_mf_skip);
        return;
    }
    if constexpr (!std::is_same<AT, float>::value) {
        if (vt == 2)
            hipLaunchKernelGGL((k_mf_backproject_b16<NG, DEPTH, 2>), grid, dim3(256), 0, stream, A, ld, nrows32, Wh,
                               Wl, ldw, rps, partial, vb0, vend, g_mf_skip);
        else
            hipLaunchKernelGGL((k_mf_backproject_b16<NG, DEPTH, 1>), grid, dim3(256), 0, stream, A, ld, nrows32, Wh,
                               Wl, ldw, rps, partial, vb0, vend, g_mf_skip);
    }
}

template <int NG, typename AT>
static void bwd_b16(int depth, int vt, dim3 grid, hipStream_t stream, const AT* A, int64_t ld, int64_t nrows32,
                    const bf16_t* Wh, const bf16_t* Wl, int64_t ldw, int64_t rps, float* partial, int64_t vb0,
                    int64_t vend) {
    if constexpr (!std::is_same<AT, float>::value) {
        if (depth == 1) {
            bwd_b16_d<NG, 1>(vt, grid, stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vb0, vend);
            return;
        }
    }
    if (depth <= 2)
        bwd_b16_d<NG, 2>(vt, grid, stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vb0, vend);
    else
        bwd_b16_d<NG, 3>(vt, grid, stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vb0, vend);
}

template <typename AT>
static void launch_mf_backproject_split(const AT* A, int64_t ld, int64_t nrows, const bf16_t* Wh, const bf16_t* Wl,
                                        int64_t ldw, int nsplit, float* partial, int nf, hipStream_t stream,
                                        int64_t v0, int64_t v1) {
    constexpr bool A32 = std::is_same<AT, float>::value;
    const std::string what = A32 ? "mf_backproject_x3" : "mf_backproject_b16";
    if (ld % 64 != 0) throw std::runtime_error(what + ": ld must be a multiple of 64");
    check_nf_b16(nf, what.c_str(), !A32);  // 128 frames: bf16 storage (split-A takes launch_mf_backproject_h16)
    const int64_t nrows32 = (nrows + 31) / 32 * 32;
    if (ldw < nrows32 || ldw % 8 != 0)
        throw std::runtime_error(what + ": W planes must hold the rows rounded up to 32 (ldw % 8 == 0)");
    if (v1 < 0) v1 = ld;
    const int vt = A32 ? mf_x3_vt(ld) : mf_b16_vt(ld, nf);
    const int64_t align = 64 * vt;
    if (v0 < 0 || v1 > ld || v0 >= v1 || v0 % align != 0 || v1 % align != 0)
        throw std::runtime_error(what + ": voxel range must be aligned to the wave's voxel tile");
    if (nsplit < 1) throw std::runtime_error(what + ": nsplit must be >= 1");
    const int64_t rps = ((nrows32 + nsplit - 1) / nsplit + 31) / 32 * 32;
    const int64_t vw0 = v0 / align, nvw = (v1 - v0) / align;  // wave tiles
    const dim3 grid((unsigned)((nvw + 3) / 4), (unsigned)nsplit);
    const int d = A32 ? mf_x3_depth(false) : mf_b16_depth(false, nf);
    if constexpr (!A32) {
        if (nf == 128) {  // 8 column groups, one 64-voxel tile per wave (VT = 1), W in LDS, W loaded early
            auto run = [&](auto kern) {
                hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vw0, v1,
                                   g_mf_skip);
            };
            if (d >= 3) run(k_mf_backproject_b16_lds<8, 3, 1, bf16_t, 0, true>);
            else run(k_mf_backproject_b16_lds<8, 2, 1, bf16_t, 0, true>);
            check_launch("k_mf_backproject_b16");
            return;
        }
    }
    if (nf == 16)
        bwd_b16<1>(d, vt, grid, stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vw0, v1);
    else if (nf == 32)
        bwd_b16<2>(d, vt, grid, stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vw0, v1);
    else
        bwd_b16<4>(d, vt, grid, stream, A, ld, nrows32, Wh, Wl, ldw, rps, partial, vw0, v1);
    check_launch(A32 ? "k_mf_backproject_x3" : "k_mf_backproject_b16");
}

void launch_mf_backproject_b16(const bf16_t* A, int64_t ld, int64_t nrows, const bf16_t* Wh, const bf16_t* Wl,
                               int64_t ldw, int nsplit, float* partial, int nf, hipStream_t stream, int64_t v0,
                               int64_t v1) {
    launch_mf_backproject_split(A, ld, nrows, Wh, Wl, ldw, nsplit, partial, nf, stream, v0, v1);
}

void launch_mf_backproject_h16(const float* A, int64_t ld, int64_t nrows, const uint16_t* W1, const uint16_t* W2,
                               int64_t ldw, int nsplit, float* partial, int nf, hipStream_t stream, int64_t v0,
                               int64_t v1, const float* csc, const float* inv_scale) {
    const std::string what = "mf_backproject_h16";
    if (!csc || !inv_scale) throw std::runtime_error(what + ": column scales and frame scales required");
    if (ld % 64 != 0) throw std::runtime_error(what + ": ld must be a multiple of 64");
    check_nf_b16(nf, what.c_str(), true);
    const int64_t nrows32 = (nrows + 31) / 32 * 32;
    if (ldw < nrows32 || ldw % 8 != 0)
        throw std::runtime_error(what + ": W planes must hold the rows rounded up to 32 (ldw % 8 == 0)");
    if (v1 < 0) v1 = ld;
    if (v0 < 0 || v1 > ld || v0 >= v1 || v0 % 64 != 0 || v1 % 64 != 0)
        throw std::runtime_error(what + ": voxel range must be aligned to 64");
    if (nsplit < 1) throw std::runtime_error(what + ": nsplit must be >= 1");
    const int64_t rps = ((nrows32 + nsplit - 1) / nsplit + 31) / 32 * 32;
    const int64_t vw0 = v0 / 64, nvw = (v1 - v0) / 64;
    const dim3 grid((unsigned)((nvw + 3) / 4), (unsigned)nsplit);
    const int d = mf_x3_depth(false);
    // SART_MF_H16 (A/B runs): "ew" early W loads, "w1" one wave per SIMD (512 registers), "ew,w1"
    const char* hv = std::getenv("SART_MF_H16");
    const bool ew = hv && std::strstr(hv, "ew"), w1 = hv && std::strstr(hv, "w1");
    auto go = [&](auto ng) {
        constexpr int NG = decltype(ng)::value;
        auto run = [&](auto k) {
            hipLaunchKernelGGL(k, grid, dim3(256), 0, stream, A, ld, nrows32, W1, W2, ldw, rps, partial, vw0, v1,
                               csc, inv_scale, g_mf_skip);
        };
        if (w1 && ew && d == 3) run(k_mf_backproject_h16<NG, 3, true, 1>);
        else if (w1 && d == 3) run(k_mf_backproject_h16<NG, 3, false, 1>);
        else if (w1 && ew) run(k_mf_backproject_h16<NG, 2, true, 1>);
        else if (w1) run(k_mf_backproject_h16<NG, 2, false, 1>);
        else if (ew) run(k_mf_backproject_h16<NG, 2, true, 2>);
        else if (d == 3) run(k_mf_backproject_h16<NG, 3>);
        else run(k_mf_backproject_h16<NG, 2>);
    };
    if (nf == 16)
        go(std::integral_constant<int, 1>{});
    else if (nf == 32)
        go(std::integral_constant<int, 2>{});
    else if (nf == 64)
        go(std::integral_constant<int, 4>{});
    else {  // 128 frames: 8 column groups, one wave per SIMD (128 accumulator registers)
        auto run = [&](auto kern) {
            hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, A, ld, nrows32, W1, W2, ldw, rps, partial, vw0, v1,
                               csc, inv_scale, g_mf_skip);
        };
        if (ew && d == 3) run(k_mf_backproject_h16<8, 3, true, 1>);
        else if (ew) run(k_mf_backproject_h16<8, 2, true, 1>);
        else if (d == 3) run(k_mf_backproject_h16<8, 3, false, 1>);
        else run(k_mf_backproject_h16<8, 2, false, 1>);
    }
    check_launch("k_mf_backproject_h16");
}

void launch_mf_backproject_x3(const float* A, int64_t ld, int64_t nrows, const bf16_t* Wh, const bf16_t* Wl,
                              int64_t ldw, int nsplit, float* partial, int nf, hipStream_t stream, int64_t v0,
                              int64_t v1) {
    launch_mf_backproject_split(A, ld, nrows, Wh, Wl, ldw, nsplit, partial, nf, stream, v0, v1);
}

}  // namespace sart
