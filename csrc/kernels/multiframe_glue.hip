// Element-wise and reduction kernels of the multi-frame solver (nf = 16, 32, 64 or 128 frames as the N columns
// of the MFMA projections in multiframe.hip). Layouts: pixel-major [rows][nf] for measurements, weights and
// forward projections (the MFMA B/D fragments), frame-major [nf][ld] for solutions and penalties (the MFMA A
// operand of the forward projection), voxel-major [ld][nf] for the reduced corrections (the back-projection
// partials' layout): a voxel range of every frame is one contiguous chunk, so the per-sweep all-reduce can
// run chunk by chunk next to the back-projection of the following chunks.
//
// Per-frame semantics are those of the single-frame solver (sart_update.hip) and the reference GPU path
// (reference sartsolver_cuda.cpp:138-354): every frame has its own normalisation, saturation mask,
// convergence history, status and iteration count; finished frames are frozen.
#include "sart_common.hpp"
#include "launchers.hpp"

#include <math.h>

#include <algorithm>
#include <stdexcept>
#include <string>

namespace sart {

constexpr int kMaxNF = kMfMaxFrames;

thread_local const int* g_mf_skip = nullptr;

// Position of frame f inside a row of a back-projection operand ([rows][16][nf / 16], multiframe.hip
// k_mf_backproject): frame f = 16 j + i sits at i * (nf / 16) + j, so a lane's column groups are adjacent.
__device__ __forceinline__ int mf_bp_slot(int f, int nf) { return (f & 15) * (nf >> 4) + (f >> 4); }

// F = sum_s Fsplit[s] (fixed order); W = a F (log) or a (ghat - F) (linear), written in the
// back-projection layout (mf_bp_slot), or with wplane > 0 in frame order as planes [nf / wplane][rows][wplane] (the
// sparse SpMM back-projection, sparse.hip: one 16-byte store per thread); per-block, per-frame partial sums of F^2 in
// fp64 (deterministic: fixed thread-to-row assignment, fixed tree).
constexpr int kWRows = 64;  // rows per block (>= 1024 blocks at 64k rows: the kernel is latency-bound)
__global__ __launch_bounds__(256) void k_mf_weights(const float* __restrict__ Fs, int nsplit, int64_t nrows_pad,
                                                    const float* __restrict__ ghat, const float* __restrict__ arow,
                                                    int logmode, float* __restrict__ W, double* __restrict__ F2part,
                                                    int nf, const int* __restrict__ skip,
                                                    unsigned* __restrict__ wmax, int wplane) {
    if (skip && *skip) return;
    __shared__ double red[1024];
    // four consecutive frames of one row per thread (16-byte loads of every split, in split order); q threads per
    // row, rstep rows per pass
    const int q = nf / 4, fq = threadIdx.x % q, rsub = threadIdx.x / q, rstep = 256 / q;
    const int f0 = fq * 4;
    const int64_t r0 = (int64_t)blockIdx.x * kWRows;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    unsigned wm[4] = {0u, 0u, 0u, 0u};  // max |w| bits per frame (finite values only, as k_mf_wmax)
    for (int rr = rsub; rr < kWRows; rr += rstep) {
        const int64_t row = r0 + rr;
        if (row >= nrows_pad) break;
        const int64_t i = row * nf + f0;
        float4 F = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s = 0; s < nsplit; ++s) {
            const float4 p = *reinterpret_cast<const float4*>(Fs + (int64_t)s * nrows_pad * nf + i);
            F.x += p.x, F.y += p.y, F.z += p.z, F.w += p.w;
        }
        const float4 a = *reinterpret_cast<const float4*>(arow + i);
        const float Fv[4] = {F.x, F.y, F.z, F.w}, av[4] = {a.x, a.y, a.z, a.w};
        float gv[4] = {0.f, 0.f, 0.f, 0.f};
        if (!logmode) {
            const float4 g = *reinterpret_cast<const float4*>(ghat + i);
            gv[0] = g.x, gv[1] = g.y, gv[2] = g.z, gv[3] = g.w;
        }
        float wv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float w = logmode ? av[k] * Fv[k] : av[k] * (gv[k] - Fv[k]);
            wv[k] = w;
            if (wplane == 0) W[row * nf + mf_bp_slot(f0 + k, nf)] = w;
            if (fabsf(w) <= 3.0e38f) wm[k] = max(wm[k], __float_as_uint(fabsf(w)));
            acc[k] += (double)Fv[k] * (double)Fv[k];
        }
        if (wplane > 0)  // f0 .. f0 + 3 lie in one plane (wplane is a multiple of 4)
            *reinterpret_cast<float4*>(W + ((int64_t)(f0 / wplane) * nrows_pad + row) * wplane + f0 % wplane) =
                make_float4(wv[0], wv[1], wv[2], wv[3]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[threadIdx.x * 4 + k] = acc[k];
    __syncthreads();
    if (threadIdx.x < nf) {  // frame f: its rstep partial sums in fixed order (deterministic)
        const int f = threadIdx.x;
        double t = 0.0;
        for (int r = 0; r < rstep; ++r) t += red[(r * q + f / 4) * 4 + (f & 3)];
        F2part[(int64_t)blockIdx.x * nf + f] = t;
    }
    if (wmax) {  // the block's max |w| per frame, then one atomic per frame (the max is order-free)
        __syncthreads();
        unsigned* redu = reinterpret_cast<unsigned*>(red);
#pragma unroll
        for (int k = 0; k < 4; ++k) redu[threadIdx.x * 4 + k] = wm[k];
        __syncthreads();
        if (threadIdx.x < nf) {
            const int f = threadIdx.x;
            unsigned m = 0u;
            for (int r = 0; r < rstep; ++r) m = max(m, redu[(r * q + f / 4) * 4 + (f & 3)]);
            if (m) atomicMax(&wmax[f], m);
        }
    }
}

// D[v][f] = scale[v] * sum_s part[s][v][f] for v in [v0, v1) (voxel-major, contiguous; fixed summation
// order); block f < nf also writes F2out[f] = (float) sum_b F2part[b][f] when F2part is given.
__global__ __launch_bounds__(256) void k_mf_collect(const float* __restrict__ part, int nsplit, int64_t ld, int64_t v0,
                                                    int64_t v1, const float* __restrict__ scale, float* __restrict__ D,
                                                    const double* __restrict__ F2part, int nF2, float* __restrict__ F2out,
                                                    int nf, const int* __restrict__ skip) {
    if (skip && *skip) return;
    // four consecutive (voxel, frame) elements per thread (one voxel: nf % 4 == 0), 16-byte loads of every split in
    // split order (the scalar version issued 4-byte loads: 72 us per 64-frame sweep at 64k voxels x 8 splits)
    const int64_t i = v0 * nf + ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i < v1 * nf) {
        const int64_t v = i / nf;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s = 0; s < nsplit; ++s) {
            const float4 p = *reinterpret_cast<const float4*>(part + (int64_t)s * ld * nf + i);
            acc.x += p.x, acc.y += p.y, acc.z += p.z, acc.w += p.w;
        }
        if (scale) {
            const float sc = scale[v];
            acc.x *= sc, acc.y *= sc, acc.z *= sc, acc.w *= sc;
        }
        *reinterpret_cast<float4*>(D + i) = acc;
    }
    if (F2part && blockIdx.x < nf) {  // block-uniform branch: block f sums frame f's nF2 partials
        // (fixed assignment and tree: deterministic). Block 0 for every frame made this kernel 15 us per 64-frame
        // sweep (32 dependent loads per thread), which a sparse shard's sweep of ~330 us felt.
        __shared__ double f2[256];
        const int f = blockIdx.x;
        double sp[4] = {0.0, 0.0, 0.0, 0.0};
        int b = threadIdx.x;
        for (; b + 3 * 256 < nF2; b += 4 * 256)
#pragma unroll
            for (int k = 0; k < 4; ++k) sp[k] += F2part[(int64_t)(b + k * 256) * nf + f];
        for (; b < nF2; b += 256) sp[0] += F2part[(int64_t)b * nf + f];
        f2[threadIdx.x] = (sp[0] + sp[1]) + (sp[2] + sp[3]);
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (threadIdx.x < w) f2[threadIdx.x] += f2[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) F2out[f] = (float)f2[0];
    }
}

// pen[f][v] = beta * sum_j L[v, j] x[f][j] (or log x), one thread per (row, frame), fixed order. Frame f is
// blockIdx.y: a wave reads 64 consecutive CSR rows and the x / pen entries of one frame row (coalesced; with the
// frame index fastest, every lane read a different frame row: 566 us per 64-frame sweep at 262144 voxels,
// profiles/rocprof_r4_2tb_kernel_stats.csv), and a finished frame's blocks return at once.
__global__ __launch_bounds__(256) void k_mf_penalty(const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                                                    const float* __restrict__ val, int64_t n, float beta, int logx,
                                                    const float* __restrict__ X, int64_t ld, float* __restrict__ pen,
                                                    const MfState* __restrict__ st) {
    if (st->all_done) return;
    const int f = blockIdx.y;
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n || st->done[f]) return;
    const float* x = X + (int64_t)f * ld;
    float s = 0.f;  // same arithmetic as k_penalty_csr (sart_update.hip)
    for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
        const float xv = x[col[k]];
        s = fmaf(val[k], logx ? logf(xv) : xv, s);
    }
    pen[(int64_t)f * ld + r] = beta * s;
}

__device__ __forceinline__ unsigned long long mf_below(int lane) { return (1ull << lane) - 1ull; }

// Device-side refill plan (k_mf_decide with a queue; one block of kMaxNF threads, thread f = slot f), after the
// decisions of this sweep: sweep_new is the sweep counter after it, ran: some slot runs this sweep's update.
// 1. Retire: every occupied slot whose frame is done gets the next output ring position while the ring has room
//    (slot order), its MfFinish entry, and is emptied; the update kernel copies its iterate (X, or Xprev after a
//    rollback) into the ring. The newest retired finite frame also replaces xlast (the device copy of the newest
//    finished solution) when it is newer.
// 2. Source (time series): the newest frame among the occupied finite slots (their iterate after this sweep's
//    update; in flight with >= src_age updates, or finished) and xlast.
// 3. Admit: empty slots (slot order) take queue entries [q_head, ...) up to the entries staged and admit_cap; each
//    starts from the source rescaled to its own normalisation (else the host x0, its staged cold start, or 1e-7) with
//    a fresh convergence history and sweep0 = sweep_new. The update kernel writes the start values (after reading
//    every source), k_mf_admit_rows the pixel columns.
// Everything depends on device state only (identical on every rank: it follows all-reduced sums), so all ranks
// retire and admit the same frames at the same sweep.
__device__ void mf_plan(MfState* __restrict__ st, MfQueue* __restrict__ q, int sweep_new, bool ran) {
    __shared__ unsigned long long m_fin[kMaxNF / 64], m_free[kMaxNF / 64], m_run[kMaxNF / 64], m_max[kMaxNF / 64];
    __shared__ int best, best_ret;
    __shared__ int s_kind, s_slot, s_iter, s_live;
    __shared__ double s_norm;
    const int f = threadIdx.x, w = f >> 6, lane = f & 63;
    const int nf = st->nf;
    const bool in = f < nf;
    const int fr = in ? q->slot_frame[f] : -1;
    const bool occ = fr >= 0;
    const bool dn = in ? st->done[f] != 0 : true;
    const bool nonfin = in && ((st->flags[f >> 6] >> (f & 63)) & 1ull);
    const bool rb = in && ((st->rollback[f >> 6] >> (f & 63)) & 1ull);
    const int sw0 = in ? st->sweep0[f] : 0;
    const int upd = sweep_new - sw0;  // updates applied to a running slot's iterate after this sweep
    const bool finished = occ && dn;
    if (f == 0) {
        best = best_ret = -1, s_kind = kSrcNone, s_slot = -1, s_iter = -1, s_norm = 1.0, s_live = 0;
        // the drift pair as the update kernel finds it in xlast / xlast2 (before this sweep's retirement moves them)
        q->drift_frame1 = q->xlast_frame, q->drift_norm1 = q->xlast_norm;
        q->drift_frame2 = q->xlast2_frame, q->drift_norm2 = q->xlast2_norm;
    }
    const unsigned long long bf = __ballot(finished);
    if (lane == 0) m_fin[w] = bf;
    __syncthreads();
    const int64_t fin = q->fin;
    const int room = q->rcap - (int)(fin - q->drained);
    const int nfin = __popcll(m_fin[0]) + __popcll(m_fin[1]);
    const int rank_fin = (w ? __popcll(m_fin[0]) : 0) + __popcll(m_fin[w] & mf_below(lane));
    const bool retire = finished && rank_fin < room;
    const int nret = nfin < room ? nfin : (room > 0 ? room : 0);
    // source candidates: occupied finite slots (in flight: at least src_age updates) and xlast
    if (q->chain && occ && !nonfin && (dn || (!q->src_finished && upd >= q->src_age))) atomicMax(&best, fr);
    if (retire && !nonfin && fr > q->xlast_frame) atomicMax(&best_ret, fr);
    const bool fre = in && (!occ || retire);
    const unsigned long long bfree = __ballot(fre);
    if (lane == 0) m_free[w] = bfree;
    __syncthreads();
    if (f == 0 && q->chain && q->xlast_frame > best && q->xlast_frame >= 0) {
        best = q->xlast_frame;  // (xlast is older than every retiring finite frame it would be replaced by)
        s_kind = kSrcLast, s_iter = q->xlast_iter, s_norm = q->xlast_norm;
    }
    __syncthreads();
    if (occ && fr == best)
        s_kind = kSrcSlot, s_slot = f, s_iter = dn ? st->iters[f] : upd, s_norm = q->slot_norm[f], s_live = dn ? 0 : 1;
    const bool xl = retire && fr == best_ret;
    const int xlast_iter = xl ? st->iters[f] : 0;
    const double xlast_norm = xl ? q->slot_norm[f] : 0.0;
    __syncthreads();  // every read of this slot's old state and of the source is done
    if (retire) {
        const int pos = (int)((fin + rank_fin) % q->rcap);
        MfFinish& L = q->log[pos];
        L.frame = fr;
        L.status = st->status[f] == kSuccess ? kSuccess : kMaxIterationsExceeded;
        L.iters = st->iters[f];
        L.flags = (nonfin ? 1 : 0) | (rb ? 2 : 0);
        L.warm_from = q->slot_warm_from[f];
        L.warm_iter = q->slot_warm_iter[f];
        L.warm_live = q->slot_warm_live[f];
        L.conv = st->conv[f];
        L.norm = q->slot_norm[f];
        q->ret_pos[f] = pos;
        q->ret_prev[f] = rb ? 1 : 0;
        q->slot_frame[f] = -1;
    } else if (in) {
        q->ret_pos[f] = -1;
    }
    if (xl) {
        q->xlast2_frame = q->xlast_frame;  // (k_mf_update copies xlast into xlast2 before overwriting it)
        q->xlast2_norm = q->xlast_norm;
        q->xlast_slot = f;
        q->xlast_frame = fr;
        q->xlast_iter = xlast_iter;
        q->xlast_norm = xlast_norm;
    }
    const int64_t avail = q->q_tail - q->q_head;
    const int nfree = __popcll(m_free[0]) + __popcll(m_free[1]);
    int nadm = nfree;
    if (q->admit_cap > 0 && nadm > q->admit_cap) nadm = q->admit_cap;
    // lead: before any frame has finished finite, one frame runs alone (its cold start converges first; frames
    // chained from its young iterates would all inherit the cold start's error: a transient of ~100 frames)
    if (q->lead && best_ret < 0 && q->xlast_frame < 0) nadm = (nfree == nf && nadm > 0) ? 1 : 0;
    if ((int64_t)nadm > avail) nadm = (int)avail;
    const int rank_free = (w ? __popcll(m_free[0]) : 0) + __popcll(m_free[w] & mf_below(lane));
    const bool adm = fre && rank_free < nadm;
    if (adm) {
        const int pos = (int)((q->q_head + rank_free) % q->qcap);
        const int frame = q->q_frame[pos];
        int kind = kSrcNone;
        if (q->chain && s_kind != kSrcNone) kind = s_kind;
        else if ((int64_t)frame < q->x0_below) kind = kSrcHostX0;
        else if (q->q_cold[pos]) kind = kSrcCold;
        q->adm_pos[f] = pos;
        q->adm_kind[f] = kind;
        q->slot_frame[f] = frame;
        q->slot_norm[f] = q->q_norm[pos];
        const bool chained = kind == kSrcSlot || kind == kSrcLast;
        q->slot_warm_from[f] = chained ? best : -1;
        q->slot_warm_iter[f] = chained ? s_iter : -1;
        q->slot_warm_live[f] = chained && s_kind == kSrcSlot ? s_live : 0;
        st->G[f] = q->q_G[pos];
        st->conv_prev[f] = 0.0;
        st->conv[f] = 0.0;
        st->done[f] = 0;
        st->status[f] = kMaxIterationsExceeded;
        st->iters[f] = st->max_iter;
        st->sweep0[f] = sweep_new;
        atomicAnd(&st->flags[f >> 6], ~(1ull << (f & 63)));
        atomicAnd(&st->rollback[f >> 6], ~(1ull << (f & 63)));
    } else if (in) {
        q->adm_pos[f] = -1;
    }
    // the next sweep: slots that run it, and whether every one of them is decided at max_iter there (then that
    // sweep's back-projection and update would be discarded: only its forward and ||A x||^2 are used)
    const bool run_next = adm || (occ && !dn);
    const bool at_max = run_next && !adm && sweep_new - sw0 >= st->max_iter;
    const unsigned long long br = __ballot(run_next), bm = __ballot(at_max);
    if (lane == 0) m_run[w] = br, m_max[w] = bm;
    __syncthreads();
    if (f == 0) {
        const int nrun = __popcll(m_run[0]) + __popcll(m_run[1]);
        const int nmax = __popcll(m_max[0]) + __popcll(m_max[1]);
        q->fin = fin + nret;
        q->q_head += nadm;
        q->n_ret = nret;
        q->n_adm = nadm;
        q->upd_any = ran ? 1 : 0;
        q->src_kind = s_kind;
        q->src_slot = s_slot;
        q->src_frame = best;
        q->src_iter = s_iter;
        q->src_norm = s_norm;
        q->src_live = s_live;
        if (best_ret < 0) q->xlast_slot = -1;
        st->all_done = nrun == 0 ? 1 : 0;
        q->skip_bwd = (nrun == 0 || nmax == nrun) ? 1 : 0;
    }
}

// Per-frame decision of sweep s (same rule as k_decide): conv_f = (G_f - F2_f) / G_f; a frame converges
// when s >= 2 and |conv_f - conv_prev_f| < tol; frames done earlier keep their conv_prev. With a queue (device
// refill) the refill plan follows (mf_plan); it also runs when every slot is done (no decision, no sweep counted).
__global__ void k_mf_decide(MfState* __restrict__ st, const float* __restrict__ F2, MfQueue* __restrict__ q) {
    __shared__ int alld;
    const int f = threadIdx.x;
    const bool active = !st->all_done;
    if (!active && !q) return;
    const int s = st->sweep;
    if (f == 0) alld = 1;
    __syncthreads();
    if (active && f < st->nf) {
        const double F = (double)F2[f];
        const int sf = s - st->sweep0[f];  // this frame's own sweep (continuous batching refills slots)
        int done = st->done[f];
        if (!isfinite(F)) {
            if (!done) {  // NaN/Inf guard: the frame stops; its last finite iterate (sf - 1 updates) is in Xprev
                atomicOr(&st->flags[f >> 6], 1ull << (f & 63));
                if (sf > 0) atomicOr(&st->rollback[f >> 6], 1ull << (f & 63));
                st->iters[f] = sf > 0 ? sf - 1 : 0;
                done = 1;
            }
        } else if (sf >= 1) {
            const double conv = (st->G[f] - F) / st->G[f];
            const bool newly = !done && sf >= 2 && fabs(conv - st->conv_prev[f]) < st->tol;
            if (newly) {
                st->status[f] = kSuccess;
                st->iters[f] = sf;
            }
            if (!(done && !newly)) st->conv_prev[f] = conv;
            st->conv[f] = conv;
            done = done || newly;
        }
        if (sf >= st->max_iter) done = 1;  // max_iter updates applied: status stays MAX_ITERATIONS_EXCEEDED
        st->done[f] = done;
        if (!done) atomicAnd(&alld, 0);
    }
    __syncthreads();
    if (!q) {
        if (f == 0) {
            st->all_done = alld ? 1 : 0;
            st->sweep = s + 1;
        }
        return;
    }
    if (active && f == 0) st->sweep = s + 1;
    mf_plan(st, q, active ? s + 1 : s, active && !alld);
}

// Update of the frames that are still running (after the decision of this sweep). D and O are voxel-major
// [ld][nf] (the reduced back-projections), X / pen / Xprev frame-major [nf][ld]: a block transposes a
// 64-voxel tile of D (and O) through LDS so both sides stay coalesced. Xprev (optional) receives the
// iterate before the update: the rollback point of the NaN/Inf guard.
// TN: LDS tile columns (64, or 128 for 128-frame batches; the narrower tile keeps 4 blocks per CU at <= 64 frames)
// With a queue (device refill, mf_plan) the same block then, for its 64 voxels: copies the iterates of the frames
// retired at this sweep into the output ring (and xlast), computes the start values of the admitted frames from
// their sources (after the update: a source is the iterate after this sweep), and writes them after a barrier,
// since a retiring slot may be both a source and re-admitted. Log mode: the admitted frames' staged O columns.
template <int TN>
__global__ __launch_bounds__(256) void k_mf_update(float* __restrict__ X, const float* __restrict__ D,
                                                   float* __restrict__ O, const float* __restrict__ pen,
                                                   float alpha, int logmode, int64_t nvox, int64_t ld,
                                                   const MfState* __restrict__ st, float* __restrict__ Xprev,
                                                   const MfQueue* __restrict__ q, MfRefill rf) {
    __shared__ float dt[64][TN + 1];
    __shared__ float ot[64][TN + 1];
    const bool refill = q && (q->n_ret || q->n_adm || q->xlast_slot >= 0);
    if (q ? (!q->upd_any && !refill) : st->all_done) return;
    const int nf = st->nf;  // 16 .. 128 (<= TN): four consecutive e of a voxel-major row share one voxel
    const int64_t v0 = (int64_t)blockIdx.x * 64;  // v0 + 63 < ld (ld % 64 == 0, grid ld / 64)
    // float4 accesses throughout (D, O: the block's 64 nf contiguous floats; X, Xprev, pen: 4 voxels of one frame)
    const float4* D4 = reinterpret_cast<const float4*>(D + v0 * nf);
    const float4* O4 = logmode ? reinterpret_cast<const float4*>(O + v0 * nf) : nullptr;
    const bool upd = !q || q->upd_any;
    for (int e4 = threadIdx.x; upd && e4 < 16 * nf; e4 += 256) {
        const int r = (4 * e4) / nf, c = (4 * e4) % nf;
        const float4 d = D4[e4];
        dt[r][c] = d.x, dt[r][c + 1] = d.y, dt[r][c + 2] = d.z, dt[r][c + 3] = d.w;
        if (logmode) {
            const float4 o = O4[e4];
            ot[r][c] = o.x, ot[r][c + 1] = o.y, ot[r][c + 2] = o.z, ot[r][c + 3] = o.w;
        }
    }
    __syncthreads();
    for (int e4 = threadIdx.x; upd && e4 < 16 * nf; e4 += 256) {
        const int f = e4 / 16, vq = 4 * (e4 % 16);
        const int64_t v = v0 + vq;
        if (v >= nvox || st->done[f] || (q && q->adm_pos[f] >= 0)) continue;  // (a slot admitted now: its new frame)
        const int64_t i = (int64_t)f * ld + v;
        const int m = nvox - v < 4 ? (int)(nvox - v) : 4;  // voxels of this quad inside the shard
        const float4 x4 = *reinterpret_cast<const float4*>(X + i);
        const float4 p4 = pen ? *reinterpret_cast<const float4*>(pen + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float xs[4] = {x4.x, x4.y, x4.z, x4.w}, ps[4] = {p4.x, p4.y, p4.z, p4.w};
        float out[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float x0 = xs[k], p = ps[k];
            if (logmode) {
                const float eps = 1e-7f;  // reference EPSILON_LOG_CUDA (sart_kernels.cu:17-19)
                float r = powf((ot[vq + k][f] + eps) / (dt[vq + k][f] + eps), alpha);
                if (pen) r *= expf(-p);
                out[k] = x0 * r;
            } else {
                const float x = x0 + dt[vq + k][f] - p;
                out[k] = x > 0.f ? x : 0.f;
            }
        }
        if (m == 4) {
            if (Xprev) *reinterpret_cast<float4*>(Xprev + i) = x4;
            *reinterpret_cast<float4*>(X + i) = make_float4(out[0], out[1], out[2], out[3]);
        } else {
            for (int k = 0; k < m; ++k) {
                if (Xprev) Xprev[i + k] = xs[k];
                X[i + k] = out[k];
            }
        }
    }
    if (!refill) return;
    // drift per voxel of this block (physical units per frame) from xlast / xlast2 before they move on (below)
    __shared__ float drift_s[64];
    const bool use_drift = q->n_adm > 0 && q->drift != 0.f && !logmode && rf.xlast2 && q->drift_frame2 >= 0 &&
                           q->drift_frame1 > q->drift_frame2;
    if (use_drift && threadIdx.x < 64) {
        const int64_t v = v0 + threadIdx.x;
        drift_s[threadIdx.x] =
            v < nvox ? (float)(((double)rf.xlast[v] * q->drift_norm1 - (double)rf.xlast2[v] * q->drift_norm2) /
                               (double)(q->drift_frame1 - q->drift_frame2))
                     : 0.f;
    }
    __syncthreads();  // this block's updated iterates are visible to the whole block
    // retired frames into the output ring (and the newest finite one into xlast); start values of the admissions
    constexpr int kMaxQ = 16 * TN / 256;
    float4 nv[kMaxQ];
    const int src_kind = q->src_kind, src_slot = q->src_slot;
    const double src_norm = q->src_norm;
    // an in-flight source extrapolated along its last update (linear mode): x + c (x - x_prev)
    const float cx = (q->src_live && !logmode) ? q->src_extrap : 0.f;
#pragma unroll
    for (int k = 0; k < kMaxQ; ++k) {
        const int e4 = threadIdx.x + 256 * k;
        if (e4 >= 16 * nf) break;
        const int f = e4 / 16;
        const int64_t v = v0 + 4 * (e4 % 16);
        const int rp = q->ret_pos[f];
        if (rp >= 0 || f == q->xlast_slot) {
            const float4 val = *reinterpret_cast<const float4*>((rp >= 0 && q->ret_prev[f] ? Xprev : X) + f * ld + v);
            if (rp >= 0) *reinterpret_cast<float4*>(rf.ring + rp * ld + v) = val;
            if (f == q->xlast_slot) {
                if (rf.xlast2) *reinterpret_cast<float4*>(rf.xlast2 + v) = *reinterpret_cast<const float4*>(rf.xlast + v);
                *reinterpret_cast<float4*>(rf.xlast + v) = val;
            }
        }
        const int ap = q->adm_pos[f];
        if (ap < 0) continue;
        const int kind = q->adm_kind[f];
        const double s_new = q->slot_norm[f];
        const bool chained = kind == kSrcSlot || kind == kSrcLast;
        const float dgap = (use_drift && chained) ? q->drift * (float)(q->slot_frame[f] - q->src_frame) : 0.f;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t vv = v + j;
            float x = 0.f;
            if (vv < nvox) {
                if (kind == kSrcSlot) {
                    float xs = X[src_slot * ld + vv];
                    if (cx != 0.f) xs = fmaf(cx, xs - Xprev[src_slot * ld + vv], xs);
                    x = (float)(((double)xs * src_norm + (double)(dgap * drift_s[vv - v0])) / s_new);
                }
                else if (kind == kSrcLast)
                    x = (float)(((double)rf.xlast[vv] * src_norm + (double)(dgap * drift_s[vv - v0])) / s_new);
                else if (kind == kSrcHostX0)
                    x = (float)(rf.x0[vv] / s_new);
                else if (kind == kSrcCold)
                    x = rf.x0q[ap * ld + vv];
                x = x > 1e-7f ? x : 1e-7f;  // (reference sartsolver_cuda.cpp:176-180)
            }
            o[j] = x;
            if (logmode) O[vv * nf + f] = rf.oq[ap * ld + vv];  // the frame's observed back-projection (staged)
        }
        nv[k] = make_float4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();  // every source read: the admitted slots may be overwritten (a retiring slot can be both)
#pragma unroll
    for (int k = 0; k < kMaxQ; ++k) {
        const int e4 = threadIdx.x + 256 * k;
        if (e4 >= 16 * nf) break;
        const int f = e4 / 16;
        const int64_t v = v0 + 4 * (e4 % 16);
        if (q->adm_pos[f] < 0) continue;
        *reinterpret_cast<float4*>(X + f * ld + v) = nv[k];
        if (rf.starts) *reinterpret_cast<float4*>(rf.starts + (int64_t)q->slot_frame[f] * ld + v) = nv[k];
    }
}

__global__ void k_mf_state_begin(MfState* __restrict__ st, const double* __restrict__ G, int nused, double tol,
                                 int max_iter, int nf) {
    const int f = threadIdx.x;
    if (f < kMaxNF) {
        const bool used = f < nf;
        st->G[f] = used ? G[f] : 1.0;
        st->conv_prev[f] = 0.0;
        st->conv[f] = 0.0;
        st->done[f] = f < nused ? 0 : 1;
        st->status[f] = kMaxIterationsExceeded;
        st->iters[f] = max_iter;
        st->sweep0[f] = 0;
    }
    if (f == 0) {
        st->sweep = 0;
        st->max_iter = max_iter;
        st->all_done = nused > 0 ? 0 : 1;
        st->nf = nf;
        for (int w = 0; w < kMfMaxFrames / 64; ++w) st->flags[w] = 0, st->rollback[w] = 0;
        st->tol = tol;
    }
}

// bf16 operand planes of the bf16 MFMA projections (multiframe_bf16.hip): hi = rne(x) and lo = x - hi rounded
// stochastically to bf16 (a hash of the element index picks the rounding point: deterministic, zero mean and
// independent across elements), so the 2^-17 representation error of hi + lo does not bias sums over equal or
// clustered values (the same reasoning and measurement as the fused sweep's bf16 x slab, fused_sweep.hip).
__device__ __forceinline__ void split_bf16(float x, uint32_t key, bf16_t& hi, bf16_t& lo) {
    const __bf16 h = (__bf16)x;
    hi = __builtin_bit_cast(bf16_t, h);
    uint32_t r = key * 0x9E3779B1u;
    r ^= r >> 15;
    r *= 0x85EBCA77u;
    r ^= r >> 13;
    lo = (bf16_t)((__float_as_uint(x - (float)h) + (r & 0xffffu)) >> 16);
}

// X [nf][ld] fp32 -> planes of the same layout (n % 4 == 0). perm (the split-A forward, multiframe_bf16.hip):
// within every block of 32 voxels, plane position 8 g + j holds voxel 4 g + j (j < 4) or 16 + 4 g + j - 4, the
// k order in which that kernel's lanes load A as two contiguous 64-byte halves of a row.
__global__ __launch_bounds__(256) void k_mf_split_x(const float* __restrict__ X, int64_t n4, bf16_t* __restrict__ hi,
                                                    bf16_t* __restrict__ lo, const int* __restrict__ skip, int perm,
                                                    int64_t ld, int64_t nf) {
    if (skip && *skip) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4 v = reinterpret_cast<const float4*>(X)[i];
    bf16_t h[4], l[4];
    const uint32_t key = (uint32_t)(4 * i);
    split_bf16(v.x, key, h[0], l[0]);
    split_bf16(v.y, key + 1, h[1], l[1]);
    split_bf16(v.z, key + 2, h[2], l[2]);
    split_bf16(v.w, key + 3, h[3], l[3]);
    int64_t o = i;  // 4-element unit: frame-major, or blocked [ld / 32][nf][32] (8 units per 32 voxels)
    if (ld > 0) {
        const int64_t f = (4 * i) / ld, c = (4 * i) % ld;
        o = ((c >> 5) * nf + f) * 8 + ((c & 31) >> 2);
    }
    if (perm) o = (o & ~(int64_t)7) | ((o & 3) << 1) | ((o >> 2) & 1);
    reinterpret_cast<uint2*>(hi)[o] = make_uint2(h[0] | (unsigned)h[1] << 16, h[2] | (unsigned)h[3] << 16);
    reinterpret_cast<uint2*>(lo)[o] = make_uint2(l[0] | (unsigned)l[1] << 16, l[2] | (unsigned)l[3] << 16);
}

// W [rows][16][nf / 16] (back-projection layout, mf_bp_slot) -> frame-major planes [nf][ldw]: 64 rows per block
// through an LDS tile, so both the reads and the 128-byte plane writes are coalesced.
// three (the split-A back-projection): hi, mid = rne(w - hi) at hi + nf * ldw and lo = rne(w - hi - mid), so
// hi + mid + lo holds w to 2^-27: the weights are residuals of both signs whose back-projection cancels, and the
// 2^-17 of a two-piece split would show at full size in A^T W (fp32 keeps w exact).
template <int TN>
__global__ __launch_bounds__(256) void k_mf_split_w(const float* __restrict__ W, int64_t nrows_pad, int nf,
                                                    int64_t ldw, bf16_t* __restrict__ hi, bf16_t* __restrict__ lo,
                                                    const int* __restrict__ skip, int three) {
    if (skip && *skip) return;
    __shared__ float tile[64][TN + 1];
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    for (int i = threadIdx.x; i < 64 * nf; i += 256) {
        const int rr = i / nf, s = i % nf;
        tile[rr][s] = (r0 + rr < nrows_pad) ? W[(r0 + rr) * nf + s] : 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * nf; i += 256) {
        const int f = i / 64, rr = i % 64;
        if (r0 + rr >= ldw) continue;
        const float w = tile[rr][mf_bp_slot(f, nf)];
        bf16_t h, l;
        if (three) {
            const __bf16 h1 = (__bf16)w;
            const float r1 = w - (float)h1;
            const __bf16 m1 = (__bf16)r1;
            const __bf16 l1 = (__bf16)(r1 - (float)m1);
            h = __builtin_bit_cast(bf16_t, h1);
            l = __builtin_bit_cast(bf16_t, l1);
            hi[(int64_t)(nf + f) * ldw + r0 + rr] = __builtin_bit_cast(bf16_t, m1);
        } else {
            split_bf16(w, (uint32_t)((int64_t)f * ldw + r0 + rr), h, l);
        }
        hi[(int64_t)f * ldw + r0 + rr] = h;
        lo[(int64_t)f * ldw + r0 + rr] = l;
    }
}

// ---- device-side refill (MultiFrameEngine::solve_series; plan in mf_plan)

// The pixel columns of the frames admitted at this sweep: ghat / arow [rows][nf] from the staged normalised pixels
// ghq [qcap][rows_pad] (same arithmetic as k_mf_prep_slots: a = 1 / ray length above the threshold where ghat >= 0).
__global__ __launch_bounds__(256) void k_mf_admit_rows(const MfQueue* __restrict__ q, const float* __restrict__ ghq,
                                                       int64_t nrows, int64_t nrows_pad,
                                                       const float* __restrict__ ray_length, float len_thres,
                                                       float* __restrict__ ghat, float* __restrict__ arow, int nf) {
    if (q->n_adm == 0) return;
    __shared__ int lf[kMaxNF], lp[kMaxNF];
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    if (threadIdx.x < nf) {
        const int p = q->adm_pos[threadIdx.x];
        if (p >= 0) {
            const int j = atomicAdd(&cnt, 1);
            lf[j] = threadIdx.x, lp[j] = p;
        }
    }
    __syncthreads();
    const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (row >= nrows_pad) return;
    float inv_len = 0.f;
    if (row < nrows) {
        const float len = ray_length[row];
        inv_len = (len > len_thres) ? 1.f / len : 0.f;
    }
    for (int j = 0; j < cnt; ++j) {
        const float gh = row < nrows ? ghq[(int64_t)lp[j] * nrows_pad + row] : 0.f;
        ghat[row * nf + lf[j]] = gh;
        arow[row * nf + lf[j]] = (row < nrows && gh >= 0.f) ? inv_len : 0.f;
    }
}

// Back-projection operands of k staged entries (positions (e0 + j) % qcap, j < k) in the back-projection layout of
// columns j: gpos = max(ghat, 0) (the cold start), wo = a ghat (the observed back-projection, log mode); columns
// j >= k zero.
__global__ __launch_bounds__(256) void k_mf_stage_ops(const float* __restrict__ ghq, int64_t e0, int qcap, int k,
                                                      int64_t nrows, int64_t nrows_pad,
                                                      const float* __restrict__ ray_length, float len_thres,
                                                      float* __restrict__ gpos, float* __restrict__ wo, int nf) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // element of [rows_pad][nf]
    if (i >= nrows_pad * nf) return;
    const int64_t row = i / nf;
    const int j = (int)(i % nf);
    float gh = 0.f, a = 0.f;
    if (j < k && row < nrows) {
        gh = ghq[((e0 + j) % qcap) * nrows_pad + row];
        const float len = ray_length[row];
        a = (gh >= 0.f && len > len_thres) ? 1.f / len : 0.f;
    }
    const int64_t ib = row * nf + mf_bp_slot(j, nf);
    gpos[ib] = gh > 0.f ? gh : 0.f;
    if (wo) wo[ib] = a * gh;
}

// Staged columns j < k of a reduced voxel-major D [ld][nf] into queue rows (e0 + j) % qcap of out [qcap][ld]:
// cold: max(D * dinv, 1e-7) (k_mf_init_slots_cold's arithmetic; 0 past nvox), else a copy (log O).
__global__ __launch_bounds__(256) void k_mf_stage_cols(const float* __restrict__ D, const float* __restrict__ dinv,
                                                       int64_t e0, int qcap, int k, int64_t nvox, int64_t ld, int nf,
                                                       float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // element of [k][ld]
    if (i >= (int64_t)k * ld) return;
    const int j = (int)(i / ld);
    const int64_t v = i % ld;
    float x = D[v * nf + j];
    if (dinv) {
        x = v < nvox ? x * dinv[v] : 0.f;
        if (v < nvox) x = x > 1e-7f ? x : 1e-7f;
    }
    out[((e0 + j) % qcap) * ld + v] = x;
}

// Staging on the device (the host only copies the frames' raw pixels in): per staged frame j (one block each) the
// maximum and the sum of squares of the positive pixels over this rank's rows (non-finite pixels count as -1, masked
// like saturated ones; reference sartsolver_cuda.cpp:146-157), in a fixed order (deterministic): stats[j] (max) and
// stats[nf + j] (sum), all-reduced over the ranks by the caller.
__global__ __launch_bounds__(1024) void k_mf_stage_stats(const double* __restrict__ g64q, int64_t e0, int qcap,
                                                         int64_t nrows, int64_t nrows_pad, double* __restrict__ stats,
                                                         int nf) {
    __shared__ double rm[1024], rs[1024];
    const int j = blockIdx.x;
    const double* g = g64q + ((e0 + j) % qcap) * nrows_pad;
    double m = -INFINITY, s = 0.0;
    for (int64_t r = threadIdx.x; r < nrows; r += 1024) {
        double v = g[r];
        if (!isfinite(v)) v = -1.0;
        m = fmax(m, v);
        if (v > 0) s += v * v;
    }
    rm[threadIdx.x] = m, rs[threadIdx.x] = s;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            rm[threadIdx.x] = fmax(rm[threadIdx.x], rm[threadIdx.x + w]);
            rs[threadIdx.x] += rs[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) stats[j] = rm[0], stats[nf + j] = rs[0];
}

// The staged frames' normalisation s = max(g) (1 if not positive) and G = sum_{g>0} g^2 / s^2 (1 if not positive)
// into the queue's metadata, with the frame index frame0 + j and the cold-start flag; ghq = (float)(g / s) (the
// arithmetic of the oracle and of the single-frame engine's prep). Grid (row blocks, k).
__global__ __launch_bounds__(256) void k_mf_stage_norm(MfQueue* __restrict__ q, const double* __restrict__ g64q,
                                                       float* __restrict__ ghq, const double* __restrict__ stats,
                                                       int64_t e0, int64_t frame0, int cold, int64_t nrows,
                                                       int64_t nrows_pad, int nf) {
    const int j = blockIdx.y;
    const int pos = (int)((e0 + j) % q->qcap);
    const double mx = stats[j];
    const double norm = mx > 0 ? mx : 1.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        double G = stats[nf + j] / (norm * norm);
        if (!(G > 0)) G = 1.0;
        q->q_norm[pos] = norm;
        q->q_G[pos] = G;
        q->q_frame[pos] = (int32_t)(frame0 + j);
        q->q_cold[pos] = cold;
    }
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= nrows_pad) return;
    float gh = 0.f;
    if (r < nrows) {
        double v = g64q[(int64_t)pos * nrows_pad + r];
        if (!isfinite(v)) v = -1.0;
        gh = (float)(v / norm);
    }
    ghq[(int64_t)pos * nrows_pad + r] = gh;
}

// Entries below q_tail become visible to the plan (their metadata was written by k_mf_stage_norm before).
__global__ void k_mf_publish(MfQueue* __restrict__ q, int64_t q_tail) {
    if (threadIdx.x == 0) q->q_tail = q_tail;
}

__global__ void k_mf_drained(MfQueue* __restrict__ q, int64_t drained) {
    if (threadIdx.x == 0 && drained > q->drained) q->drained = drained;
}

__global__ void k_mf_queue_begin(MfQueue* __restrict__ q, int qcap, int rcap, int chain, int admit_cap, int src_age,
                                 int64_t x0_below, int src_finished, int lead, float src_extrap, float drift) {
    const int f = threadIdx.x;
    if (f < kMaxNF) {
        q->slot_frame[f] = -1;
        q->slot_warm_from[f] = q->slot_warm_iter[f] = -1;
        q->slot_warm_live[f] = 0;
        q->slot_norm[f] = 1.0;
        q->ret_pos[f] = q->adm_pos[f] = -1;
        q->ret_prev[f] = 0;
        q->adm_kind[f] = kSrcNone;
    }
    if (f == 0) {
        q->q_head = q->q_tail = q->fin = q->drained = 0;
        q->qcap = qcap, q->rcap = rcap;
        q->chain = chain, q->admit_cap = admit_cap, q->src_age = src_age, q->x0_below = x0_below;
        q->src_finished = src_finished, q->lead = lead, q->src_extrap = src_extrap, q->src_live = 0;
        q->n_ret = q->n_adm = q->upd_any = q->skip_bwd = 0;
        q->xlast_frame = q->xlast_iter = q->xlast_slot = -1;
        q->xlast_norm = 1.0;
        q->xlast2_frame = q->drift_frame1 = q->drift_frame2 = -1;
        q->xlast2_norm = q->drift_norm1 = q->drift_norm2 = 1.0;
        q->drift = drift;
        q->src_kind = kSrcNone, q->src_slot = q->src_frame = q->src_iter = -1;
        q->src_norm = 1.0;
    }
}

static inline unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }

static void check_nf(int nf, const char* what) {
    if (nf != 16 && nf != 32 && nf != 64 && nf != 128)
        throw std::runtime_error(std::string(what) + ": nf must be 16, 32, 64 or 128");
}

int mf_weights_num_blocks(int64_t nrows_pad) { return (int)((nrows_pad + kWRows - 1) / kWRows); }

void launch_mf_weights(const float* Fs, int nsplit, int64_t nrows_pad, const float* ghat, const float* arow,
                       bool logmode, float* W, double* F2part, int nf, hipStream_t stream, unsigned* wmax,
                       int wplane) {
    check_nf(nf, "mf_weights");
    if (wplane < 0 || (wplane > 0 && (wplane % 16 != 0 || nf % wplane != 0)))
        throw std::runtime_error("mf_weights: plane width must divide nf and be a multiple of 16");
    if (wmax) hip_call(hipMemsetAsync(wmax, 0, nf * sizeof(unsigned), stream), "hipMemsetAsync");
    hipLaunchKernelGGL(k_mf_weights, dim3((unsigned)mf_weights_num_blocks(nrows_pad)), dim3(256), 0, stream, Fs,
                       nsplit, nrows_pad, ghat, arow, logmode ? 1 : 0, W, F2part, nf, g_mf_skip, wmax, wplane);
    check_launch("k_mf_weights");
}

void launch_mf_collect(const float* part, int nsplit, int64_t ld, int64_t v0, int64_t v1, const float* scale,
                       float* D, const double* F2part, int nF2, float* F2out, int nf, hipStream_t stream) {
    check_nf(nf, "mf_collect");
    if (v0 < 0 || v1 > ld || v1 < v0) throw std::runtime_error("mf_collect: voxel range outside [0, ld)");
    const int64_t n = (v1 - v0) * nf;  // a multiple of 4 (nf is 16 .. 128): 4 elements per thread
    const unsigned blocks = std::max<unsigned>(F2part ? (unsigned)nf : 1u, nb(n / 4));  // F2: one block per frame
    hipLaunchKernelGGL(k_mf_collect, dim3(blocks), dim3(256), 0, stream, part, nsplit, ld, v0, v1,
                       scale, D, F2part, nF2, F2out, nf, g_mf_skip);
    check_launch("k_mf_collect");
}

// The kernels below take nf from the state (set by k_mf_state_begin): nf = frames of the engine's batch.
void launch_mf_penalty(const int64_t* row_ptr, const int32_t* col, const float* val, int64_t n, float beta, bool logx,
                       const float* X, int64_t ld, float* pen, const MfState* st, int nf, hipStream_t stream) {
    check_nf(nf, "mf_penalty");
    hipLaunchKernelGGL(k_mf_penalty, dim3(nb(n), nf), dim3(256), 0, stream, row_ptr, col, val, n, beta,
                       logx ? 1 : 0, X, ld, pen, st);
    check_launch("k_mf_penalty");
}

void launch_mf_decide(MfState* st, const float* F2, hipStream_t stream, MfQueue* q) {
    hipLaunchKernelGGL(k_mf_decide, dim3(1), dim3(kMaxNF), 0, stream, st, F2, q);
    check_launch("k_mf_decide");
}

void launch_mf_update(float* X, const float* D, float* O, const float* pen, float alpha, bool logmode,
                      int64_t nvox, int64_t ld, const MfState* st, int nf, hipStream_t stream, float* Xprev,
                      const MfQueue* q, const MfRefill* rf) {
    check_nf(nf, "mf_update");
    if (q && (!rf || !rf->ring || !rf->xlast || (logmode && !rf->oq)))
        throw std::runtime_error("mf_update: a refill needs the output ring, xlast and (log) the staged O");
    const MfRefill r = rf ? *rf : MfRefill{};
    hipLaunchKernelGGL((nf > 64 ? k_mf_update<128> : k_mf_update<64>), dim3((unsigned)((ld + 63) / 64)), dim3(256), 0,
                       stream, X, D, O, pen, alpha,
                       logmode ? 1 : 0, nvox, ld, st, Xprev, q, r);
    check_launch("k_mf_update");
}

void launch_mf_admit_rows(const MfQueue* q, const float* ghq, int64_t nrows, int64_t nrows_pad, const float* ray_length,
                          float len_thres, float* ghat, float* arow, int nf, hipStream_t stream) {
    check_nf(nf, "mf_admit_rows");
    if (nrows_pad <= 0) return;
    hipLaunchKernelGGL(k_mf_admit_rows, dim3(nb(nrows_pad)), dim3(256), 0, stream, q, ghq, nrows, nrows_pad, ray_length,
                       len_thres, ghat, arow, nf);
    check_launch("k_mf_admit_rows");
}

void launch_mf_stage_ops(const float* ghq, int64_t e0, int qcap, int k, int64_t nrows, int64_t nrows_pad,
                         const float* ray_length, float len_thres, float* gpos, float* wo, int nf, hipStream_t stream) {
    check_nf(nf, "mf_stage_ops");
    if (k < 0 || k > nf || qcap < k) throw std::runtime_error("mf_stage_ops: 0 <= k <= nf, k <= qcap");
    if (nrows_pad <= 0) return;
    hipLaunchKernelGGL(k_mf_stage_ops, dim3(nb(nrows_pad * nf)), dim3(256), 0, stream, ghq, e0, qcap, k, nrows,
                       nrows_pad, ray_length, len_thres, gpos, wo, nf);
    check_launch("k_mf_stage_ops");
}

void launch_mf_stage_cols(const float* D, const float* dinv, int64_t e0, int qcap, int k, int64_t nvox, int64_t ld,
                          int nf, float* out, hipStream_t stream) {
    check_nf(nf, "mf_stage_cols");
    if (k < 0 || k > nf || qcap < k) throw std::runtime_error("mf_stage_cols: 0 <= k <= nf, k <= qcap");
    if (k == 0) return;
    hipLaunchKernelGGL(k_mf_stage_cols, dim3(nb((int64_t)k * ld)), dim3(256), 0, stream, D, dinv, e0, qcap, k, nvox, ld,
                       nf, out);
    check_launch("k_mf_stage_cols");
}

void launch_mf_stage_stats(const double* g64q, int64_t e0, int qcap, int k, int64_t nrows, int64_t nrows_pad,
                           double* stats, int nf, hipStream_t stream) {
    check_nf(nf, "mf_stage_stats");
    if (k < 0 || k > nf || qcap < k) throw std::runtime_error("mf_stage_stats: 0 <= k <= nf, k <= qcap");
    if (k == 0) return;
    hipLaunchKernelGGL(k_mf_stage_stats, dim3((unsigned)k), dim3(1024), 0, stream, g64q, e0, qcap, nrows, nrows_pad,
                       stats, nf);
    check_launch("k_mf_stage_stats");
}

void launch_mf_stage_norm(MfQueue* q, const double* g64q, float* ghq, const double* stats, int64_t e0, int64_t frame0,
                          bool cold, int k, int64_t nrows, int64_t nrows_pad, int nf, hipStream_t stream) {
    check_nf(nf, "mf_stage_norm");
    if (k < 0 || k > nf) throw std::runtime_error("mf_stage_norm: 0 <= k <= nf");
    if (k == 0) return;
    const dim3 grid((unsigned)std::max<int64_t>(1, (nrows_pad + 255) / 256), (unsigned)k);
    hipLaunchKernelGGL(k_mf_stage_norm, grid, dim3(256), 0, stream, q, g64q, ghq, stats, e0, frame0, cold ? 1 : 0,
                       nrows, nrows_pad, nf);
    check_launch("k_mf_stage_norm");
}

void launch_mf_publish(MfQueue* q, int64_t q_tail, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_publish, dim3(1), dim3(64), 0, stream, q, q_tail);
    check_launch("k_mf_publish");
}

void launch_mf_drained(MfQueue* q, int64_t drained, hipStream_t stream) {
    hipLaunchKernelGGL(k_mf_drained, dim3(1), dim3(64), 0, stream, q, drained);
    check_launch("k_mf_drained");
}

void launch_mf_queue_begin(MfQueue* q, int qcap, int rcap, bool chain, int admit_cap, int src_age, int64_t x0_below,
                           bool src_finished, bool lead, float src_extrap, hipStream_t stream, float drift) {
    if (qcap < 1 || qcap > kMfQueueMax || rcap < 1 || rcap > kMfQueueMax)
        throw std::runtime_error("mf_queue_begin: queue and ring capacities in [1, 256]");
    hipLaunchKernelGGL(k_mf_queue_begin, dim3(1), dim3(kMaxNF), 0, stream, q, qcap, rcap, chain ? 1 : 0, admit_cap,
                       src_age, x0_below, src_finished ? 1 : 0, lead ? 1 : 0, src_extrap, drift);
    check_launch("k_mf_queue_begin");
}

void launch_mf_state_begin(MfState* st, const double* G, int nused, double tol, int max_iter, int nf,
                           hipStream_t stream) {
    check_nf(nf, "mf_state_begin");
    if (nused > nf) throw std::runtime_error("mf_state_begin: more frames than the batch holds");
    hipLaunchKernelGGL(k_mf_state_begin, dim3(1), dim3(kMaxNF), 0, stream, st, G, nused, tol, max_iter, nf);
    check_launch("k_mf_state_begin");
}

void launch_mf_split_x(const float* X, int64_t n, bf16_t* hi, bf16_t* lo, hipStream_t stream, bool perm,
                       int64_t ld) {
    if (n % (perm ? 32 : 4) != 0) throw std::runtime_error("mf_split_x: length must be a multiple of 4 (32 permuted)");
    if (ld > 0 && (ld % 32 != 0 || n % ld != 0))
        throw std::runtime_error("mf_split_x: blocked planes need ld a multiple of 32 dividing the length");
    hipLaunchKernelGGL(k_mf_split_x, dim3(std::max<unsigned>(1, nb(n / 4))), dim3(256), 0, stream, X, n / 4, hi, lo, g_mf_skip,
                       (int)perm, ld, ld > 0 ? n / ld : (int64_t)0);
    check_launch("k_mf_split_x");
}

// fp16-pair back-projection operands (launch_mf_backproject_h16). Per-frame max |w| over the rows (non-negative
// floats order like their bit patterns: an unsigned atomic max), then w s_f = w1 + w2 + e with w1 = rne_f16(w s_f),
// w2 = rne_f16(w s_f - w1), |e| <= 2^-24 |w s_f|, s_f = 2^(14 - e_f) for max |w| = m 2^e_f (m in [0.5, 1)): the
// scaled frame stays below 2^14 (f16 max 65504) and its values down to 2^-16 of the frame's max keep both pieces
// normal. inv_scale[f] = 1 / (a_scale s_f) (exact: powers of two) undoes both scalings in the back-projection.
__global__ __launch_bounds__(256) void k_mf_wmax(const float* __restrict__ W, int64_t nrows_pad, int nf,
                                                 unsigned* __restrict__ wmax, const int* __restrict__ skip) {
    if (skip && *skip) return;
    // thread (slot sl, row class q): a register max over the block's rows of its class (coalesced: consecutive threads
    // read consecutive slots), then the nq classes of a slot combined through LDS; one global atomic per slot
    __shared__ unsigned red[256];
    const int sl = threadIdx.x % nf, q = threadIdx.x / nf, nq = 256 / nf;
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    unsigned m = 0u;
    for (int rr = q; rr < 64; rr += nq)
        if (r0 + rr < nrows_pad) {
            const float w = fabsf(W[(r0 + rr) * nf + sl]);
            if (w <= 3.0e38f) m = max(m, __float_as_uint(w));  // finite values only
        }
    red[threadIdx.x] = m;
    __syncthreads();
    if (q == 0) {
        for (int k = 1; k < nq; ++k) m = max(m, red[k * nf + sl]);
        const int f = (sl % (nf >> 4)) * 16 + sl / (nf >> 4);  // inverse of mf_bp_slot
        if (m) atomicMax(&wmax[f], m);
    }
}

__device__ __forceinline__ int mf_w16_exp(unsigned mbits) {  // e with max |w| = m 2^e, m in [0.5, 1)
    if (mbits == 0u) return 0;
    int e;
    (void)frexpf(__uint_as_float(mbits), &e);
    return e;
}
// The f16 scale exponent 14 - e of a maximum m 2^e, clamped so that the scale and its inverse are both normal
// floats (a maximum below 2^-106 would otherwise give an infinite scale, and w * inf non-finite pieces)
__device__ __host__ __forceinline__ int mf_f16_shift(int e) {
    const int s = 14 - e;
    return s > 120 ? 120 : (s < -120 ? -120 : s);
}

template <int TN>
__global__ __launch_bounds__(256) void k_mf_split_w16(const float* __restrict__ W, int64_t nrows_pad, int nf,
                                                      int64_t ldw, uint16_t* __restrict__ w1, uint16_t* __restrict__ w2,
                                                      const unsigned* __restrict__ wmax, float a_scale,
                                                      float* __restrict__ inv_scale, const int* __restrict__ skip) {
    if (skip && *skip) return;
    __shared__ float tile[64][TN + 1];
    __shared__ float sc[TN];
    for (int f = threadIdx.x; f < nf; f += 256) {
        const int s = mf_f16_shift(mf_w16_exp(wmax[f]));
        sc[f] = ldexpf(1.f, s);
        if (blockIdx.x == 0) inv_scale[f] = ldexpf(1.f / a_scale, -s);
    }
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    for (int i = threadIdx.x; i < 64 * nf; i += 256) {
        const int rr = i / nf, s = i % nf;
        tile[rr][s] = (r0 + rr < nrows_pad) ? W[(r0 + rr) * nf + s] : 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * nf; i += 256) {
        const int f = i / 64, rr = i % 64;
        if (r0 + rr >= ldw) continue;
        const float w = tile[rr][mf_bp_slot(f, nf)] * sc[f];
        const _Float16 h1 = (_Float16)w;
        const _Float16 h2 = (_Float16)(w - (float)h1);
        w1[(int64_t)f * ldw + r0 + rr] = __builtin_bit_cast(uint16_t, h1);
        w2[(int64_t)f * ldw + r0 + rr] = __builtin_bit_cast(uint16_t, h2);
    }
}

// max |a| over n floats (unsigned atomic max of the bit patterns; non-finite values ignored)
__global__ __launch_bounds__(256) void k_absmax_f32(const float* __restrict__ A, int64_t n, unsigned* __restrict__ out) {
    __shared__ unsigned red[256];
    unsigned m = 0u;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * 256) {
        const float4 v = reinterpret_cast<const float4*>(A)[i];
        const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a = fabsf(xs[k]);
            if (a <= 3.0e38f) m = max(m, __float_as_uint(a));
        }
    }
    if (blockIdx.x == 0)
        for (int64_t i = (n / 4) * 4 + threadIdx.x; i < n; i += 256) {
            const float a = fabsf(A[i]);
            if (a <= 3.0e38f) m = max(m, __float_as_uint(a));
        }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0 && red[0]) atomicMax(out, red[0]);
}

// ---------------------------------------------------------------------------------------------------------------
// Range-safe f16-pair operands of the split-A projections (multiframe_bf16.hip). An f16 piece has a 5-bit exponent,
// so one scale for a whole shard keeps only entries within ~2^16 of the shard's max |A| at full precision; a
// ray-transfer matrix with reflections spans 1e8 .. 1e20 (tests/test_gpu_realistic.py). Each kernel therefore
// scales A where its sums run: the forward F[p][f] = sum_v A[p][v] X[f][v] per ROW (s_p from max_v |A[p][v]|), the
// back-projection D[v][f] = sum_p A[p][v] W[p][f] per COLUMN (s_v from max_p |A[p][v]|), and the fp32 operand per
// frame (X by max_v |X[f][v]|, W by max_p |W[p][f]|). Every scale is a power of two 2^mf_f16_shift(e) (scaled maxima
// in [2^13, 2^14)); the inverse is applied to each output in the epilogue, exactly. What is left is an absolute
// floor of ~2^-39 of the row / column / frame maximum per element (subnormal f16), against fp32's 2^-24 relative.
// Scale arrays hold the scale at [i] and its inverse at [n + i].

// max_v |A[p][v]| of every row (one wave per row, 4 rows per block) -> rsc[p] = 2^s, rsc[nrows_pad + p] = 2^-s
__global__ __launch_bounds__(256) void k_mf_row_scales(const float* __restrict__ A, int64_t ld, int64_t nrows_pad,
                                                       float* __restrict__ rsc) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= nrows_pad) return;
    const float4* a = reinterpret_cast<const float4*>(A + row * ld);
    unsigned m = 0u;
    for (int64_t i = lane; i < ld / 4; i += 64) {
        const float4 v = a[i];
        const float xs[4] = {fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (xs[k] <= 3.0e38f) m = max(m, __float_as_uint(xs[k]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
    if (lane == 0) {
        const int s = m ? mf_f16_shift(mf_w16_exp(m)) : 0;
        rsc[row] = ldexpf(1.f, s);
        rsc[nrows_pad + row] = ldexpf(1.f, -s);
    }
}

// max_p |A[p][v]| over a range of rows per block (4 columns per thread, 1024 per block), combined by an unsigned
// atomic max of the bit patterns (order-free)
__global__ __launch_bounds__(256) void k_mf_col_max(const float* __restrict__ A, int64_t ld, int64_t nrows_pad,
                                                    int64_t rows_per_block, unsigned* __restrict__ cmax) {
    const int64_t c4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c4 * 4 >= ld) return;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < nrows_pad ? r0 + rows_per_block : nrows_pad;
    unsigned m[4] = {0u, 0u, 0u, 0u};
    for (int64_t r = r0; r < r1; ++r) {
        const float4 v = reinterpret_cast<const float4*>(A + r * ld)[c4];
        const float xs[4] = {fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (xs[k] <= 3.0e38f) m[k] = max(m[k], __float_as_uint(xs[k]));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (m[k]) atomicMax(&cmax[c4 * 4 + k], m[k]);
}

__global__ __launch_bounds__(256) void k_mf_col_scales(const unsigned* __restrict__ cmax, int64_t ld,
                                                       float* __restrict__ csc) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= ld) return;
    const int s = cmax[v] ? mf_f16_shift(mf_w16_exp(cmax[v])) : 0;
    csc[v] = ldexpf(1.f, s);
    csc[ld + v] = ldexpf(1.f, -s);
}

// per-frame max |X[f][v]| of frame-major X [nf][ld] (finite values only)
__global__ __launch_bounds__(256) void k_mf_xmax(const float* __restrict__ X, int64_t ld, unsigned* __restrict__ xmax,
                                                 const int* __restrict__ skip) {
    if (skip && *skip) return;
    __shared__ unsigned red[256];
    const int f = blockIdx.y;
    const float4* x = reinterpret_cast<const float4*>(X + (int64_t)f * ld);
    unsigned m = 0u;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ld / 4; i += (int64_t)gridDim.x * 256) {
        const float4 v = x[i];
        const float xs[4] = {fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (xs[k] <= 3.0e38f) m = max(m, __float_as_uint(xs[k]));
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0 && red[0]) atomicMax(&xmax[f], red[0]);
}

// X [nf][ld] fp32 -> f16 pieces x s_f = x1 + x2 (+ |e| <= 2^-22 |x s_f|, both rne) in the layout of k_mf_split_x
// (perm: the split-A forward's k order; blocked: [ld / 32][nf][32]); xinv[f] = 1 / s_f
__global__ __launch_bounds__(256) void k_mf_split_x16(const float* __restrict__ X, int64_t ld, int nf,
                                                      uint16_t* __restrict__ x1, uint16_t* __restrict__ x2,
                                                      const unsigned* __restrict__ xmax, float* __restrict__ xinv,
                                                      const int* __restrict__ skip, int perm, int blocked) {
    if (skip && *skip) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nf && blockIdx.x == 0) {
        const int f = (int)i;
        xinv[f] = ldexpf(1.f, xmax[f] ? -mf_f16_shift(mf_w16_exp(xmax[f])) : 0);
    }
    if (i >= (int64_t)nf * ld / 4) return;
    const int64_t f = (4 * i) / ld, c = (4 * i) % ld;
    const float sc = ldexpf(1.f, xmax[f] ? mf_f16_shift(mf_w16_exp(xmax[f])) : 0);
    const float4 v = reinterpret_cast<const float4*>(X)[i];
    const float xs[4] = {v.x * sc, v.y * sc, v.z * sc, v.w * sc};
    uint16_t h[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const _Float16 a = (_Float16)xs[k];
        h[k] = __builtin_bit_cast(uint16_t, a);
        l[k] = __builtin_bit_cast(uint16_t, (_Float16)(xs[k] - (float)a));
    }
    int64_t o = i;
    if (blocked) o = ((c >> 5) * nf + f) * 8 + ((c & 31) >> 2);
    if (perm) o = (o & ~(int64_t)7) | ((o & 3) << 1) | ((o >> 2) & 1);
    reinterpret_cast<uint2*>(x1)[o] = make_uint2(h[0] | (unsigned)h[1] << 16, h[2] | (unsigned)h[3] << 16);
    reinterpret_cast<uint2*>(x2)[o] = make_uint2(l[0] | (unsigned)l[1] << 16, l[2] | (unsigned)l[3] << 16);
}

void launch_mf_row_scales(const float* A, int64_t ld, int64_t nrows_pad, float* rsc, hipStream_t stream) {
    if (ld % 4 != 0) throw std::runtime_error("mf_row_scales: ld must be a multiple of 4");
    if (nrows_pad <= 0) return;
    hipLaunchKernelGGL(k_mf_row_scales, dim3((unsigned)((nrows_pad + 3) / 4)), dim3(256), 0, stream, A, ld, nrows_pad,
                       rsc);
    check_launch("k_mf_row_scales");
}

void launch_mf_col_scales(const float* A, int64_t ld, int64_t nrows_pad, unsigned* scratch, float* csc,
                          hipStream_t stream) {
    if (ld % 4 != 0) throw std::runtime_error("mf_col_scales: ld must be a multiple of 4");
    hip_call(hipMemsetAsync(scratch, 0, ld * sizeof(unsigned), stream), "hipMemsetAsync");
    const int64_t rpb = 256;
    if (nrows_pad > 0) {
        const dim3 grid((unsigned)((ld / 4 + 255) / 256), (unsigned)((nrows_pad + rpb - 1) / rpb));
        hipLaunchKernelGGL(k_mf_col_max, grid, dim3(256), 0, stream, A, ld, nrows_pad, rpb, scratch);
        check_launch("k_mf_col_max");
    }
    hipLaunchKernelGGL(k_mf_col_scales, dim3(nb(ld)), dim3(256), 0, stream, scratch, ld, csc);
    check_launch("k_mf_col_scales");
}

void launch_mf_split_x16(const float* X, int64_t ld, int nf, uint16_t* x1, uint16_t* x2, unsigned* xmax, float* xinv,
                         hipStream_t stream, bool perm, bool blocked) {
    check_nf(nf, "mf_split_x16");
    if (ld % 32 != 0) throw std::runtime_error("mf_split_x16: ld must be a multiple of 32");
    hip_call(hipMemsetAsync(xmax, 0, nf * sizeof(unsigned), stream), "hipMemsetAsync");
    const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(16, (ld / 4 + 1023) / 1024));
    hipLaunchKernelGGL(k_mf_xmax, dim3(bx, (unsigned)nf), dim3(256), 0, stream, X, ld, xmax, g_mf_skip);
    check_launch("k_mf_xmax");
    hipLaunchKernelGGL(k_mf_split_x16, dim3(std::max<unsigned>(1, nb((int64_t)nf * ld / 4))), dim3(256), 0, stream, X,
                       ld, nf, x1, x2, xmax, xinv, g_mf_skip, (int)perm, (int)blocked);
    check_launch("k_mf_split_x16");
}

void launch_mf_split_w16(const float* W, int64_t nrows_pad, int nf, int64_t ldw, uint16_t* w1, uint16_t* w2,
                         unsigned* wmax, float a_scale, float* inv_scale, hipStream_t stream, bool have_max) {
    check_nf(nf, "mf_split_w16");
    if (ldw > nrows_pad) throw std::runtime_error("mf_split_w16: plane stride exceeds the padded rows");
    if (!have_max) {
        hip_call(hipMemsetAsync(wmax, 0, nf * sizeof(unsigned), stream), "hipMemsetAsync");
        const unsigned nb64 = (unsigned)((nrows_pad + 63) / 64);
        hipLaunchKernelGGL(k_mf_wmax, dim3(nb64), dim3(256), 0, stream, W, nrows_pad, nf, wmax, g_mf_skip);
        check_launch("k_mf_wmax");
    }
    hipLaunchKernelGGL((nf > 64 ? k_mf_split_w16<128> : k_mf_split_w16<64>), dim3((unsigned)((ldw + 63) / 64)), dim3(256),
                       0, stream, W, nrows_pad, nf, ldw,
                       w1, w2, wmax, a_scale, inv_scale, g_mf_skip);
    check_launch("k_mf_split_w16");
}

float absmax_pow2_scale(const float* A, int64_t n, unsigned* scratch, hipStream_t stream) {
    hip_call(hipMemsetAsync(scratch, 0, sizeof(unsigned), stream), "hipMemsetAsync");
    const int64_t nb = std::min<int64_t>(4096, std::max<int64_t>(1, (n / 4 + 255) / 256));
    hipLaunchKernelGGL(k_absmax_f32, dim3((unsigned)nb), dim3(256), 0, stream, A, n, scratch);
    check_launch("k_absmax_f32");
    unsigned bits = 0;
    hip_call(hipMemcpyAsync(&bits, scratch, sizeof(unsigned), hipMemcpyDeviceToHost, stream), "D2H");
    hip_call(hipStreamSynchronize(stream), "hipStreamSynchronize");
    if (bits == 0u) return 1.f;
    int e;
    (void)frexpf(__builtin_bit_cast(float, bits), &e);
    return ldexpf(1.f, mf_f16_shift(e));  // scaled max in [2^13, 2^14)
}

void launch_mf_split_w(const float* W, int64_t nrows_pad, int nf, int64_t ldw, bf16_t* hi, bf16_t* lo,
                       hipStream_t stream, bool three) {
    check_nf(nf, "mf_split_w");
    if (ldw > nrows_pad) throw std::runtime_error("mf_split_w: plane stride exceeds the padded rows");
    hipLaunchKernelGGL((nf > 64 ? k_mf_split_w<128> : k_mf_split_w<64>), dim3((unsigned)((ldw + 63) / 64)), dim3(256), 0,
                       stream, W, nrows_pad, nf, ldw,
                       hi, lo, g_mf_skip, (int)three);
    check_launch("k_mf_split_w");
}


}  // namespace sart
