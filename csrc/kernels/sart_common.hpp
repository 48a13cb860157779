// Shared definitions for the gfx950 (CDNA4) SART kernels.
//
// Storage conventions (all kernels):
//   * A is the local row shard of the ray-transfer matrix, row-major fp32, P_pad rows x ld columns.
//     ld is a multiple of 64 floats (256 B rows) and the padding columns/rows are zero, so every
//     16-byte vector load is aligned and in bounds and no kernel needs a column tail branch.
//   * Vectors over voxels (x, ray density, corrections) are padded to ld with zeros.
//   * Vectors over pixels (measurement, weights, ray length) are padded to P_pad with zeros.
//
// Everything that the reference recomputed on the host per iteration (convergence test,
// iteration counter, solution update) lives in a device-resident SartState, so a whole frame
// solve runs without host synchronisation (reference: sartsolver_cuda.cpp:231-262 synchronises
// twice per iteration through cublasSdot and MPI_Allreduce on host buffers).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sart {

constexpr int kWave = 64;

// Layout shared with python (mpi_cuda_sartsolver_amd/ops/state.py). 128 bytes.
struct alignas(16) SartState {
    double G;           //  0: sum_{g>0} g^2 / s^2 over all ranks (reference "measurement_squared")
    double conv_prev;   //  8: convergence metric of the previous SART iteration
    double conv_last;   // 16: convergence metric of the last SART iteration
    double F_last;      // 24: ||A x||^2 of the last sweep (fp32 semantics, as the reference)
    int32_t sweep;      // 32: number of sweeps whose decision has been taken
    int32_t done;       // 36: 1 once the frame is finished (converged or max iterations)
    int32_t status;     // 40: 0 SUCCESS, -1 MAX_ITERATIONS_EXCEEDED, -2 running
    int32_t iterations; // 44: number of SART updates applied to x
    int32_t max_iter;   // 48
    int32_t error;      // 52: nonzero when a persistent kernel gave up waiting (protocol timeout)
    double tol;         // 56: convergence tolerance
    int32_t epoch;      // 64: exchange epoch of the fused sweep (strictly increasing, never 0)
    int32_t flags;      // 68: bit 0 = the sweep produced a non-finite ||A x||^2 (solve stopped)
    double reserved[7]; // 72..127
};
static_assert(sizeof(SartState) == 128, "SartState must be 128 bytes");

enum Status : int32_t { kSuccess = 0, kMaxIterationsExceeded = -1, kRunning = -2 };

// Device-resident convergence state of a multi-frame batch (multi-frame solver): one column per frame.
// A batch holds nf = 16, 32, 64 or 128 frames (the MFMA N dimension is 16; 32 .. 128 use 2 .. 8 column groups;
// 128 on bf16 storage and the f16-pair split-A path; 64 on the fp32 MFMA and bf16 six-product paths).
constexpr int kMfMaxFrames = 128;
struct alignas(16) MfState {
    double G[kMfMaxFrames];          // sum_{g>0} g^2 / s^2 per frame
    double conv_prev[kMfMaxFrames];
    double conv[kMfMaxFrames];       // last convergence metric per frame
    int32_t done[kMfMaxFrames];      // frame finished (converged, non-finite, or unused slot)
    int32_t status[kMfMaxFrames];
    int32_t iters[kMfMaxFrames];
    int32_t sweep;
    int32_t max_iter;
    int32_t all_done;                // every frame done, or max_iter reached (no further update)
    int32_t nf;                      // frames per batch (columns in use by the kernels)
    unsigned long long flags[kMfMaxFrames / 64];     // bit f % 64 of word f / 64: frame f produced a non-finite ||A x||^2
    double tol;
    unsigned long long rollback[kMfMaxFrames / 64];  // frame f stopped at sweep >= 1 (last finite iterate in Xprev)
    int32_t sweep0[kMfMaxFrames];    // sweep at which the slot's current frame started (continuous batching)
};

// ---- device-side slot refill (MultiFrameEngine::solve_series) ----
// The host stages frames into a device queue (normalised pixels, scalars; cold starts / observed back-projections
// where needed) ahead of the sweeps; the decision kernel of every sweep retires the frames that finished (their
// solutions into an output ring the host drains) and admits queued frames into the freed slots in the SAME sweep,
// each starting from the current iterate of the newest frame in flight (a time series) -- no host round trip
// between a frame finishing and its slot working on the next one.
constexpr int kMfQueueMax = 2 * kMfMaxFrames;  // queue entries / output ring entries (2 nf)
enum MfSrc : int32_t {
    kSrcNone = 0,     // no start value known: x = 1e-7 (only when every earlier frame went non-finite)
    kSrcSlot = 1,     // the iterate of a slot after this sweep's update (in flight, or finished at this sweep)
    kSrcLast = 2,     // the newest finished frame's solution kept on the device (MfQueue::xlast_*)
    kSrcHostX0 = 3,   // the caller's start value (fp64, de-normalised)
    kSrcCold = 4,     // the entry's staged cold start max(A^T max(ghat, 0) / rho, 1e-7)
};
struct MfFinish {      // one finished frame in the output ring (read by the host from the state snapshot)
    int32_t frame, status, iters, flags;  // flags: bit 0 non-finite, bit 1 rolled back to the last finite iterate
    int32_t warm_from, warm_iter;         // the start value's frame and its update count (-1: x0 / cold)
    int32_t warm_live, pad;               // that frame was still in flight (its iterate extrapolated, src_extrap)
    double conv, norm;
};
struct alignas(16) MfQueue {
    int64_t q_head, q_tail;  // staged entries [q_head, q_tail) (entry e at ring position e % qcap)
    int64_t fin, drained;    // frames written to the output ring / copied out by the host (position fin % rcap)
    int32_t qcap, rcap;
    int32_t chain;        // admitted frames start from the newest frame in flight (time series)
    int32_t admit_cap;    // admissions per sweep (0: any number)
    int32_t src_age;      // an in-flight source needs at least this many updates
    int32_t src_finished; // sources: finished frames only (xlast and the frames retiring now), not frames in flight
    int32_t lead;         // chain without x0: the first frame runs alone until it has finished (a converged source)
    float src_extrap;     // linear mode: an in-flight source's iterate is extrapolated, x + c (x - x_prev)
    int32_t src_live;     // this sweep's source is in flight (its Xprev is the iterate before this sweep's update)
    int64_t x0_below;     // frames below this index start from the host x0 when no chain source exists (!chain: always)
    int32_t n_ret, n_adm, upd_any, skip_bwd;  // this sweep's plan; skip_bwd: the next sweep's back-projection is unused
    int32_t xlast_frame, xlast_iter, xlast_slot, pad0;  // xlast_slot: the slot copied into xlast at this sweep (-1)
    double xlast_norm;
    // Drift (linear mode): the previous xlast is kept (xlast2), and an admitted frame q chained from source frame p
    // starts at X_p + drift (q - p) (X_xlast - X_xlast2) / (xlast_frame - xlast2_frame) in de-normalised units -- the
    // per-frame change between the two newest finished solutions, carried over the frame gap a pipelined chain
    // leaves (a source is >= src_age sweeps old, so several newer frames are already in flight). drift_*: this
    // sweep's snapshot of the pair, taken before xlast / xlast2 move on.
    int32_t xlast2_frame, drift_frame1, drift_frame2, pad1;
    double xlast2_norm, drift_norm1, drift_norm2;
    float drift;
    int32_t pad2;
    int32_t src_kind, src_slot, src_frame, src_iter;  // the chain source of this sweep's admissions
    double src_norm;
    int32_t slot_frame[kMfMaxFrames];  // frame in each slot (-1: empty)
    int32_t slot_warm_from[kMfMaxFrames], slot_warm_iter[kMfMaxFrames], slot_warm_live[kMfMaxFrames];
    double slot_norm[kMfMaxFrames];
    int32_t ret_pos[kMfMaxFrames];    // output ring position written at this sweep (-1), from X or Xprev (ret_prev)
    int32_t ret_prev[kMfMaxFrames];
    int32_t adm_pos[kMfMaxFrames];    // queue ring position admitted at this sweep (-1)
    int32_t adm_kind[kMfMaxFrames];   // MfSrc of that admission
    int32_t q_frame[kMfQueueMax];     // per queue ring position: frame index, cold start staged, norm, G
    int32_t q_cold[kMfQueueMax];
    double q_norm[kMfQueueMax], q_G[kMfQueueMax];
    MfFinish log[kMfQueueMax];        // per output ring position
};
// Device buffers of the refill (k_mf_update with a queue): output ring [rcap][ld], xlast [ld], host x0 (fp64 [nvox]),
// staged cold starts and observed back-projections [qcap][ld] (null when not staged), optional start-value record
// [frames][ld] (tests)
struct MfRefill {
    float* ring;
    float* xlast;
    float* xlast2;  // the previous xlast (drift; may be null: no drift)
    const double* x0;
    const float* x0q;
    const float* oq;
    float* starts;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Streaming read of the RTM: every byte of A is read once per sweep by one CU and never again before it
// has left every cache, so the loads carry the non-temporal hint (MI355X_MICROARCH.md 'nt-weights').
#ifndef SART_STREAM_NT
#define SART_STREAM_NT 1
#endif
typedef float sart_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 load_stream(const float4* p) {
#if SART_STREAM_NT
    const sart_f4v v = __builtin_nontemporal_load(reinterpret_cast<const sart_f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}

__device__ __forceinline__ uint2 load_stream(const uint2* p) {
#if SART_STREAM_NT
    typedef unsigned sart_u2v __attribute__((ext_vector_type(2)));
    const sart_u2v v = __builtin_nontemporal_load(reinterpret_cast<const sart_u2v*>(p));
    return make_uint2(v.x, v.y);
#else
    return *p;
#endif
}

// RTM element access of the two-pass kernels, by storage type. fp32 (the reference's storage) or bf16 (opt-in
// storage precision, SURVEY 7.3 8(d): half the HBM bytes per sweep and twice the matrix per GPU; products
// and sums stay fp32). One 16-byte vector load per call: 4 fp32 or 8 bf16 columns, widened to NF4 float4.
typedef uint16_t bf16_t;  // raw bf16 bit pattern (upper half of an fp32)
typedef unsigned sart_u4v __attribute__((ext_vector_type(4)));

template <typename AT>
struct RtmVec;

template <>
struct RtmVec<float> {
    static constexpr int NF4 = 1;  // float4 per 16-byte load
    __device__ __forceinline__ static void load(const float* row, int64_t v, float4 (&o)[1]) {
        o[0] = load_stream(reinterpret_cast<const float4*>(row) + v);
    }
};

__device__ __forceinline__ float4 bf16x4_to_f4(unsigned lo, unsigned hi) {
    return make_float4(__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u), __uint_as_float(hi << 16),
                       __uint_as_float(hi & 0xffff0000u));
}

template <>
struct RtmVec<bf16_t> {
    static constexpr int NF4 = 2;
    __device__ __forceinline__ static void load(const bf16_t* row, int64_t v, float4 (&o)[2]) {
#if SART_STREAM_NT
        const sart_u4v u = __builtin_nontemporal_load(reinterpret_cast<const sart_u4v*>(row) + v);
#else
        const sart_u4v u = reinterpret_cast<const sart_u4v*>(row)[v];
#endif
        o[0] = bf16x4_to_f4(u.x, u.y);
        o[1] = bf16x4_to_f4(u.z, u.w);
    }
};

__device__ __forceinline__ float dot4(const float4 a, const float4 b) {
    return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

__device__ __forceinline__ void fma4(float4& acc, const float4 a, const float s) {
    acc.x = fmaf(a.x, s, acc.x);
    acc.y = fmaf(a.y, s, acc.y);
    acc.z = fmaf(a.z, s, acc.z);
    acc.w = fmaf(a.w, s, acc.w);
}

__device__ __forceinline__ void add4(float4& acc, const float4 a) {
    acc.x += a.x;
    acc.y += a.y;
    acc.z += a.z;
    acc.w += a.w;
}

// Launch-time error check used by every host launcher.
void check_launch(const char* what);
// Checked HIP runtime call (throws std::runtime_error with `what` and the HIP error string).
void hip_call(hipError_t e, const char* what);

constexpr float kEpsLog = 1e-7f;  // reference EPSILON_LOG_CUDA (sart_kernels.cu:17-19)

// Single lane. Consumes ||A x_s||^2 of sweep s and decides, exactly as the reference loop does
// at its iteration s-1 (its forward projection after the update is our next sweep's forward).
// Fslot[1] is the error word of the sweep, summed over the ranks by the same collective that carries
// ||A x||^2 (k_reduce_partials writes the local SartState::error there): when ANY rank's persistent sweep
// gave up, every rank stops the frame at this sweep and sees error bit 8, so the fallback decision is
// identical on all ranks (a rank-local decision would leave its peers waiting in the next collective).
// The decision on a copy of the state (shared by k_decide and k_decide_update): a pure function of the state
// before the sweep and of the sweep's reduced Fslot, so every workgroup that evaluates it gets the same answer.
__device__ inline void decide_next(SartState& st, const float* __restrict__ Fslot) {
    if (st.done) return;
    const int s = st.sweep;
    const double F = (double)Fslot[0];
    st.F_last = F;
    int done = 0;
    int status = kRunning;
    if (Fslot[1] != 0.f) {
        st.error |= 8;
        st.sweep = s + 1;
        st.status = kMaxIterationsExceeded;
        st.done = 1;
        st.epoch = st.epoch + 1;
        return;
    }
    if (!isfinite(F)) {
        // NaN/Inf guard: x_s produced a non-finite ||A x||^2. Stop; the engine returns the
        // last finite iterate x_{s-1}, which the update kernels saved in xprev, so s - 1 updates count.
        st.flags |= 1;
        st.iterations = s > 0 ? s - 1 : 0;
        st.sweep = s + 1;
        st.status = kMaxIterationsExceeded;
        st.done = 1;
        st.epoch = st.epoch + 1;
        return;
    }
    if (s >= 1) {
        const double conv = (st.G - F) / st.G;
        if (s >= 2 && fabs(conv - st.conv_prev) < st.tol) {
            done = 1;
            status = kSuccess;
        }
        st.conv_prev = conv;
        st.conv_last = conv;
    }
    if (!done && s >= st.max_iter) {
        done = 1;
        status = kMaxIterationsExceeded;
    }
    st.iterations = done ? s : s + 1;
    st.sweep = s + 1;
    st.status = status;
    st.done = done;
    st.epoch = st.epoch + 1;
}

// One voxel's SART update (k_decide_update, k_reduce_decide_update, the P2P kernel's fused update: one definition, so
// every path rounds the same way; callers compile it with contraction off)
template <bool LOGV>
__device__ __forceinline__ float sart_update_voxel(float x0, float d, float o, const float* pen, float pn, float alpha) {
#pragma clang fp contract(off)
    if constexpr (LOGV) {
        float r = powf((o + kEpsLog) / (d + kEpsLog), alpha);
        if (pen) r *= expf(-pn);
        return x0 * r;
    } else {
        float v = x0 + d;
        if (pen) v -= pn;
        return (v > 0.f) ? v : 0.f;
    }
}

}  // namespace sart
