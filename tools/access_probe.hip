// HBM access-pattern probe (gfx950): streams an 8 GiB row-major matrix (65536 rows x 128 KiB) with the load shapes
// of the multi-frame kernels and measures the bandwidth, to separate the DRAM cost of a pattern from the kernels'
// compute. A wave owns RTI x rpi rows and walks a split of the columns; per step each of its lanes loads 16 bytes
// of RTI x KB (row group, column chunk) pairs, where one instruction covers rpi = 1024 / BPI rows x BPI bytes
// (BPI / 16 lanes per row). A row is therefore read in runs of KB x BPI contiguous bytes per step. DEPTH steps of
// loads are kept in flight (register ring, unconditional clamped loads like the solver kernels).
//   multi-frame forward (16x16x32 fragments, KB = 2): BPI 64, run 128 B
//   multi-frame back-projection (8-byte row loads):  BPI 128 (8 B x 16 lanes), run 128 B
//   fused sweep (a row per wave instruction):         BPI 1024, run 8 KiB
// Usage: access_probe [pitch_extra_bytes]      one JSON line per pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

template <int BPI, int KB, int RTI, int DEPTH, bool NT>
__global__ __launch_bounds__(256) void k_stream(const char* __restrict__ A, long pitch, long nrows, long row_bytes,
                                                long split_bytes, unsigned* __restrict__ out) {
    constexpr int LPR = BPI / 16;        // lanes per row
    constexpr int RPI = 64 / LPR;        // rows per instruction
    constexpr int RS = DEPTH + 1;
    constexpr long STEP = (long)BPI * KB;  // bytes of a row per step
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long row0 = ((long)blockIdx.x * 4 + wave) * (RPI * RTI);
    if (row0 >= nrows) return;
    const long c0 = (long)blockIdx.y * split_bytes;
    const long c1 = c0 + split_bytes < row_bytes ? c0 + split_bytes : row_bytes;
    const long nst = (c1 - c0) / STEP;
    const char* base = A + (row0 + lane / LPR) * pitch + c0 + (lane % LPR) * 16;
    uint4 ring[RS][RTI][KB];
    unsigned acc = 0;
    auto load = [&](int sl, long t) {
        const long tc = t < nst ? t : nst - 1;
#pragma unroll
        for (int r = 0; r < RTI; ++r)
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const uint4* p = reinterpret_cast<const uint4*>(base + (long)r * RPI * pitch + tc * STEP + k * BPI);
                if constexpr (NT) {
                    typedef unsigned u4 __attribute__((ext_vector_type(4)));
                    const u4 v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p));
                    ring[sl][r][k] = make_uint4(v.x, v.y, v.z, v.w);
                } else {
                    ring[sl][r][k] = *p;
                }
            }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) load(d, d);
    for (long t0 = 0; t0 < nst; t0 += RS) {
#pragma unroll
        for (int q = 0; q < RS; ++q) {
            const long t = t0 + q;
            load((q + DEPTH) % RS, t + DEPTH);
            if (t < nst) {
#pragma unroll
                for (int r = 0; r < RTI; ++r)
#pragma unroll
                    for (int k = 0; k < KB; ++k) {
                        const uint4 v = ring[q][r][k];
                        acc ^= v.x ^ v.y ^ v.z ^ v.w;
                    }
            }
        }
    }
    out[((long)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x] = acc;
}

template <int BPI, int KB, int RTI, int DEPTH, bool NT>
static void run(const char* name, const char* A, long pitch, long nrows, long row_bytes, unsigned* out) {
    constexpr int RPI = 64 / (BPI / 16);
    const long rows_per_wg = 4L * RPI * RTI;
    const long nblk = nrows / rows_per_wg;
    long nsplit = (1024 + nblk - 1) / nblk;  // >= 1024 workgroups like the solver kernels
    while ((row_bytes / nsplit) % ((long)BPI * KB) != 0) ++nsplit;
    const long split_bytes = row_bytes / nsplit;
    const dim3 grid((unsigned)nblk, (unsigned)nsplit);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_stream<BPI, KB, RTI, DEPTH, NT>), grid, dim3(256), 0, 0, A, pitch, nrows, row_bytes,
                           split_bytes, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
    }
    const double gb = (double)nrows * row_bytes / 1e9;
    std::printf("{\"pattern\": \"%s\", \"BPI\": %d, \"KB\": %d, \"run_bytes\": %d, \"RTI\": %d, \"rows_per_wave\": %d, "
                "\"depth\": %d, \"nt\": %d, \"pitch\": %ld, \"workgroups\": %ld, \"ms\": %.4f, \"GBps\": %.1f}\n",
                name, BPI, KB, BPI * KB, RTI, RPI * RTI, DEPTH, (int)NT, pitch, nblk * nsplit, best, gb / best * 1e3);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const long extra = argc > 1 ? std::atol(argv[1]) : 0;
    const long nrows = 65536, row_bytes = 131072, pitch = row_bytes + extra;
    char* A;
    unsigned* out;
    CHECK(hipMalloc(&A, nrows * pitch));
    CHECK(hipMemset(A, 1, nrows * pitch));
    CHECK(hipMalloc(&out, 64L << 20));
    run<64, 2, 4, 3, false>("mf_forward (64 B x 16 rows, KB 2)", A, pitch, nrows, row_bytes, out);
    run<64, 8, 1, 3, false>("64 B x 16 rows, KB 8 (512 B runs)", A, pitch, nrows, row_bytes, out);
    run<64, 16, 1, 2, false>("64 B x 16 rows, KB 16 (1 KiB runs)", A, pitch, nrows, row_bytes, out);
    run<128, 1, 8, 3, true>("mf_backproject-like (128 B x 8 rows, KB 1)", A, pitch, nrows, row_bytes, out);
    run<128, 4, 2, 3, true>("128 B x 8 rows, KB 4 (512 B runs)", A, pitch, nrows, row_bytes, out);
    run<256, 2, 4, 3, false>("256 B x 4 rows, KB 2 (512 B runs)", A, pitch, nrows, row_bytes, out);
    run<256, 4, 2, 3, false>("256 B x 4 rows, KB 4 (1 KiB runs)", A, pitch, nrows, row_bytes, out);
    run<512, 2, 4, 3, false>("512 B x 2 rows, KB 2 (1 KiB runs)", A, pitch, nrows, row_bytes, out);
    run<1024, 2, 4, 3, true>("1 KiB x 1 row, KB 2 (2 KiB runs)", A, pitch, nrows, row_bytes, out);
    run<1024, 8, 1, 3, true>("fused-like (1 KiB x 1 row, KB 8: 8 KiB runs)", A, pitch, nrows, row_bytes, out);
    CHECK(hipFree(A));
    CHECK(hipFree(out));
    return 0;
}
