// One-shot peer-to-peer all-reduce over xGMI. The reference reduces the
// per-iteration correction through host memory (D2H, MPI_Allreduce, H2D: reference
// sartsolver_cuda.cpp:242-244); RCCL rings over xGMI use one link per direction and 2(N-1) latency steps.
// Here every rank PUSHES its vector into a per-source slot of every peer's receive buffer (IPC-mapped,
// all 7 links at once), raises one epoch flag per chunk in each peer, then waits for the N-1 flags of its
// chunk and sums the N slots locally in rank order 0..N-1 -- the same order on every rank, so the result
// is bitwise identical everywhere (the replicated solution x never drifts between GPUs).
//
// Buffer reuse: slots alternate with the call parity. A peer can be at most one call ahead of this
// rank (it needs this rank's flags of call k to finish call k), so it writes the other parity's slots
// while this rank still reads call k; flags hold monotonically increasing epochs (compared with >=).
//
// Memory: receive buffers and flags are uncached device memory (hipDeviceMallocUncached). Producer:
// every pushing wave waits for its stores, then (behind a barrier) each flag lane issues a system-scope
// release, waits again (cdna_hip_programming.md Guideline 16 Pitfall 12) and stores the flag. Consumer:
// relaxed system-scope polls, one acquire + wait per polling lane, a barrier, then plain loads. Polls
// are bounded (s_memrealtime, 100 MHz) and also end when a peer that aborts sets this rank's abort
// word: the chunk is then filled with NaN (the engine's non-finite guard stops the frame) and *err is
// raised for the host.
#include "launchers.hpp"

#include <stdexcept>
#include <string>

namespace sart {

namespace {

__device__ inline float red(float a, float b, int op) { return op == 0 ? a + b : fmaxf(a, b); }

// Poll flag f (>= epoch) as one lane, bounded by the timeout and this rank's abort word; true on arrival.
__device__ inline bool p2p_wait_flag(const unsigned* f, unsigned epoch, const unsigned* abort_word,
                                     uint64_t timeout_ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks ||
            __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
            return false;
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// `in` may alias `out` (in place): each element is read in phase 1 and written in phase 2 by one thread.
// RED: there is no `in`; phase 1 forms the pushed values from src in k_reduce_partials' summation order (n = ld + 2).
// UPD (RED only; 1 linear, 2 log): launch_decide_update fused in (launchers.hpp UpdateArgs): the state is read
// before anything else, ||A x||^2 and the error word of every rank come from the tail chunk's slots (this rank's own
// computed here, in the tail workgroup's order), the decision is decide_next's, the update that of
// k_reduce_decide_update, and the last workgroup to take the ticket writes the new state.
template <bool RED, int UPD = 0>
__global__ __launch_bounds__(256) void k_p2p_allreduce(const float* in, float* out, int64_t n, int64_t chunk,
                                                       P2pArgs a, int rank, int nranks, unsigned epoch, int parity,
                                                       int64_t cap, int op, unsigned* err, uint64_t timeout_ticks,
                                                       int vec_io, int skip_flags, ReduceSrc src, UpdateArgs u) {
#pragma clang fp contract(off)
    static_assert(UPD == 0 || RED, "the fused update follows the reduce + all-reduce");
    __shared__ SartState s_next;
    __shared__ int s_apply;
    if constexpr (UPD != 0) {
        if (threadIdx.x == 0) s_next = *u.st;  // before this workgroup's ticket (taken last)
        if (u.xcnt && blockIdx.x == 0 && threadIdx.x < 16) u.xcnt[threadIdx.x] = 0u;  // see k_update_linear
    }
    const int64_t c0 = (int64_t)blockIdx.x * chunk;
    const int64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    // After a timeout on this rank the device path is being abandoned (the engines agree on it after the solve and
    // switch to the base communicator): later calls fail at once, without pushing or raising flags, so a solve
    // pays one timeout per rank instead of one per queued sweep. One load per workgroup, broadcast through LDS: the
    // whole workgroup takes the same branch (a per-thread load could split it while another workgroup of this
    // launch raises *err, and the threads that went on would raise flags for a partly pushed chunk).
    __shared__ unsigned err0;
    if (threadIdx.x == 0) err0 = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (err0 != 0) {
        for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) out[i] = __builtin_nanf("");
        if constexpr (UPD != 0) {  // as the separate update on this NaN output: the NaN guard stops the frame (the
            if (threadIdx.x == 0) {  // engines re-solve it on the base communicator); state and ticket as usual
                const float F[2] = {__builtin_nanf(""), 0.f};
                decide_next(s_next, F);
                const unsigned tk = atomicAdd(u.ticket, 1u);
                if (tk == gridDim.x - 1) {
                    *u.st = s_next;
                    *u.ticket = 0u;
                }
            }
        }
        return;
    }
    const int64_t mine = (int64_t)(parity * kP2pMaxRanks + rank) * cap;  // my slot in every receive buffer

    // RED: the chunk holding [ld] and [ld + 1] (never split: chunks are multiples of 1024, ld of 64) sums Fpart first.
    // With the fused update (UPD != 0) EVERY workgroup sums the nF partials to get this rank's tail values for its
    // decision: blocks x nF fp64 loads, all L2 hits after the first workgroup (dense fused grid: nF <= 512; a sparse
    // 64k-row shard: ~2k, i.e. ~16 KiB per workgroup, a few microseconds per sweep over the whole grid). Reading the
    // own tail from the receive slot instead would make every workgroup wait for the tail chunk's flag first.
    __shared__ float tailv[2];
    if constexpr (RED) {
        if (UPD != 0 || (c0 <= src.ld && src.ld < c1)) {  // uniform over the workgroup
            __shared__ double red4[4];
            double acc = 0.0;
            for (int64_t i = threadIdx.x; i < src.nF; i += 256) acc += src.Fpart[i];
            acc = wave_sum(acc);
            if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = acc;
            __syncthreads();
            if (threadIdx.x == 0) {
                tailv[0] = (float)(((red4[0] + red4[1]) + red4[2]) + red4[3]);
                tailv[1] = src.st != nullptr ? (float)src.st->error : 0.f;
            }
            __syncthreads();
        }
    }
    const int64_t ld4 = src.ld >> 2;

    // phase 1: push this chunk into slot [parity][rank] of every rank's receive buffer (self included)
    for (int64_t i = c0 + 4 * (int64_t)threadIdx.x; i < c1; i += 4 * (int64_t)blockDim.x) {
        if (i + 4 <= c1) {
            float4 v;
            if constexpr (RED) {  // i + 4 <= ld here: only the chunk's tail [ld, ld + 2) is shorter than 4
                const float4* __restrict__ p4 = reinterpret_cast<const float4*>(src.partial) + (i >> 2);
                v = p4[0];
                for (int k = 1; k < src.nsplit; ++k) {
                    const float4 w = p4[(int64_t)k * ld4];
                    v.x += w.x;
                    v.y += w.y;
                    v.z += w.z;
                    v.w += w.w;
                }
                if (src.scale != nullptr) {
                    const float4 sc = reinterpret_cast<const float4*>(src.scale)[i >> 2];
                    v.x *= sc.x;
                    v.y *= sc.y;
                    v.z *= sc.z;
                    v.w *= sc.w;
                }
            } else {
                v = vec_io ? *reinterpret_cast<const float4*>(in + i)
                           : make_float4(in[i], in[i + 1], in[i + 2], in[i + 3]);  // unaligned caller buffer
            }
            for (int j = 0; j < nranks; ++j) *reinterpret_cast<float4*>(a.recv[j] + mine + i) = v;
        } else {
            for (int64_t k = i; k < c1; ++k) {
                float v;
                if constexpr (RED) {
                    v = k == src.ld ? tailv[0] : tailv[1];  // k >= ld: ld % 4 == 0 and n = ld + 2
                } else {
                    v = in[k];
                }
                for (int j = 0; j < nranks; ++j) a.recv[j][mine + k] = v;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int timed_out;
    if (threadIdx.x == 0) timed_out = 0;
    __syncthreads();
    if ((int)threadIdx.x < nranks && (int)threadIdx.x != rank && !skip_flags) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the pushed bytes reach every peer
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.flags[threadIdx.x] + rank * kP2pMaxBlocks + blockIdx.x, epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }

    // phase 2: wait for this chunk from every peer, then reduce the N local slots in rank order. UPD: also for the
    // tail chunk (||A x||^2 and the error word of every peer) when this is not the tail chunk's workgroup.
    const int64_t tail_blk = RED ? src.ld / chunk : 0;
    if ((int)threadIdx.x < nranks && (int)threadIdx.x != rank) {
        const unsigned* f = a.flags[rank] + threadIdx.x * kP2pMaxBlocks + blockIdx.x;
        bool ok = p2p_wait_flag(f, epoch, a.abort_word, timeout_ticks);
        if (UPD != 0 && ok && tail_blk != (int64_t)blockIdx.x)
            ok = p2p_wait_flag(a.flags[rank] + threadIdx.x * kP2pMaxBlocks + tail_blk, epoch, a.abort_word,
                               timeout_ticks);
        if (!ok) timed_out = 1;  // a peer is gone (timeout) or told us it aborted
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const float* base = a.recv[rank] + (int64_t)parity * kP2pMaxRanks * cap;
    if (timed_out) {
        if (threadIdx.x == 0) atomicOr(err, 1u);
        for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) out[i] = __builtin_nanf("");
        if constexpr (UPD != 0) {  // non-finite ||A x||^2: the NaN guard stops the frame (decide_next advances the
            if (threadIdx.x == 0) {  // sweep and epoch as on any NaN); the engines re-solve it
                const float F[2] = {__builtin_nanf(""), 0.f};
                decide_next(s_next, F);
                const unsigned tk = atomicAdd(u.ticket, 1u);
                if (tk == gridDim.x - 1) {
                    *u.st = s_next;
                    *u.ticket = 0u;
                }
            }
        }
        return;
    }
    if constexpr (UPD != 0) {  // {||A x||^2, error word}: the tail slots of every rank summed in rank order
        if (threadIdx.x == 0) {
            float F[2];
            for (int k = 0; k < 2; ++k) {
                auto slot = [&](int r) { return r == rank ? tailv[k] : base[(int64_t)r * cap + src.ld + k]; };
                float t = slot(0);
                for (int r = 1; r < nranks; ++r) t = t + slot(r);
                F[k] = t;
            }
            decide_next(s_next, F);
            s_apply = !s_next.done;
        }
        __syncthreads();
    }
    for (int64_t i = c0 + 4 * (int64_t)threadIdx.x; i < c1; i += 4 * (int64_t)blockDim.x) {
        if (i + 4 <= c1) {
            float4 s = *reinterpret_cast<const float4*>(base + i);
            for (int r = 1; r < nranks; ++r) {
                const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)r * cap + i);
                s.x = red(s.x, v.x, op);
                s.y = red(s.y, v.y, op);
                s.z = red(s.z, v.z, op);
                s.w = red(s.w, v.w, op);
            }
            if (vec_io) {
                *reinterpret_cast<float4*>(out + i) = s;
            } else {
                out[i] = s.x, out[i + 1] = s.y, out[i + 2] = s.z, out[i + 3] = s.w;
            }
            if constexpr (UPD != 0) {  // i + 4 <= ld here (the chunk's short tail holds [ld, ld + 2) only)
                if (s_apply && i < u.n) {
                    const float dv[4] = {s.x, s.y, s.z, s.w};
                    float x0[4], o[4] = {0.f, 0.f, 0.f, 0.f}, pn[4] = {0.f, 0.f, 0.f, 0.f}, t[4];
                    const float4 xv = *reinterpret_cast<const float4*>(u.x + i);
                    x0[0] = xv.x, x0[1] = xv.y, x0[2] = xv.z, x0[3] = xv.w;
                    if constexpr (UPD == 2) {
                        const float4 ov = *reinterpret_cast<const float4*>(u.O + i);
                        o[0] = ov.x, o[1] = ov.y, o[2] = ov.z, o[3] = ov.w;
                    }
                    if (u.pen) {
                        const float4 pv = *reinterpret_cast<const float4*>(u.pen + i);
                        pn[0] = pv.x, pn[1] = pv.y, pn[2] = pv.z, pn[3] = pv.w;
                    }
#pragma unroll
                    for (int c = 0; c < 4; ++c) t[c] = sart_update_voxel<UPD == 2>(x0[c], dv[c], o[c], u.pen, pn[c], u.alpha);
                    if (i + 4 <= u.n) {
                        if (u.xprev) *reinterpret_cast<float4*>(u.xprev + i) = xv;
                        *reinterpret_cast<float4*>(u.x + i) = make_float4(t[0], t[1], t[2], t[3]);
                    } else {
                        for (int c = 0; c < 4 && i + c < u.n; ++c) {
                            if (u.xprev) u.xprev[i + c] = x0[c];
                            u.x[i + c] = t[c];
                        }
                    }
                }
            }
        } else {
            for (int64_t k = i; k < c1; ++k) {
                float s = base[k];
                for (int r = 1; r < nranks; ++r) s = red(s, base[(int64_t)r * cap + k], op);
                out[k] = s;
            }
        }
    }
    if constexpr (UPD != 0) {
        if (threadIdx.x == 0) {
            const unsigned tk = atomicAdd(u.ticket, 1u);  // after this workgroup's read of the state (kernel start)
            if (tk == gridDim.x - 1) {
                *u.st = s_next;
                *u.ticket = 0u;
            }
        }
    }
}

}  // namespace

int64_t p2p_chunk(int64_t n, int max_blocks) {
    // 1024 floats per workgroup (one float4 per thread) up to max_blocks workgroups, then wider chunks
    const int64_t per = 1024;
    const int64_t mb = max_blocks > 0 && max_blocks < kP2pMaxBlocks ? max_blocks : kP2pMaxBlocks;
    const int64_t groups = (n + per - 1) / per;
    const int64_t mult = (groups + mb - 1) / mb;
    return per * (mult > 0 ? mult : 1);
}

void launch_p2p_allreduce(const float* in, float* out, int64_t n, const P2pArgs& a, int rank, int nranks,
                          unsigned epoch, int64_t cap, int op, unsigned* err, double timeout_s, hipStream_t stream,
                          bool skip_flags) {
    if (n <= 0) return;
    if (nranks < 1 || nranks > kP2pMaxRanks || rank < 0 || rank >= nranks || n > cap || cap % 4 != 0)
        throw std::runtime_error("launch_p2p_allreduce: bad arguments (n=" + std::to_string(n) + ", cap=" +
                                 std::to_string(cap) + ", ranks=" + std::to_string(nranks) + ")");
    // the receive slots are always 16-B aligned; the caller's buffer may not be (4-B element accesses then)
    const int vec_io = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) % 16) == 0;
    const int64_t chunk = p2p_chunk(n, a.max_blocks);
    const int64_t blocks = (n + chunk - 1) / chunk;
    if (blocks > kP2pMaxBlocks) throw std::runtime_error("launch_p2p_allreduce: too many chunks");
    const uint64_t ticks = (uint64_t)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
    hipLaunchKernelGGL(k_p2p_allreduce<false>, dim3((unsigned)blocks), dim3(256), 0, stream, in, out, n, chunk, a,
                       rank, nranks, epoch, (int)(epoch & 1u), cap, op, err, ticks, vec_io, skip_flags ? 1 : 0,
                       ReduceSrc{}, UpdateArgs{});
    check_launch("k_p2p_allreduce");
}

void launch_p2p_reduce_allreduce(const ReduceSrc& src, float* out, const P2pArgs& a, int rank, int nranks,
                                 unsigned epoch, int64_t cap, unsigned* err, double timeout_s, hipStream_t stream,
                                 bool skip_flags, const UpdateArgs* upd) {
    const int64_t n = src.ld + 2;
    const bool aligned = ((reinterpret_cast<uintptr_t>(src.partial) | reinterpret_cast<uintptr_t>(src.scale) |
                           reinterpret_cast<uintptr_t>(out)) % 16) == 0;
    if (nranks < 1 || nranks > kP2pMaxRanks || rank < 0 || rank >= nranks || n > cap || cap % 4 != 0 ||
        src.ld <= 0 || src.ld % 64 != 0 || src.nsplit < 1 || src.nF < 0 || src.partial == nullptr || !aligned)
        throw std::runtime_error("launch_p2p_reduce_allreduce: bad arguments (ld=" + std::to_string(src.ld) +
                                 ", cap=" + std::to_string(cap) + ", ranks=" + std::to_string(nranks) + ")");
    const int64_t chunk = p2p_chunk(n, a.max_blocks);
    const int64_t blocks = (n + chunk - 1) / chunk;
    if (blocks > kP2pMaxBlocks) throw std::runtime_error("launch_p2p_reduce_allreduce: too many chunks");
    const uint64_t ticks = (uint64_t)(timeout_s * 1e8);
    if (upd) {
        const UpdateArgs& u = *upd;
        if (!u.st || !u.x || !u.ticket || (u.logmode && !u.O) || u.n > src.ld ||
            ((reinterpret_cast<uintptr_t>(u.x) | reinterpret_cast<uintptr_t>(u.O) | reinterpret_cast<uintptr_t>(u.pen) |
              reinterpret_cast<uintptr_t>(u.xprev)) % 16) != 0)
            throw std::runtime_error("launch_p2p_reduce_allreduce: bad update arguments");
        auto run = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, stream, nullptr, out, n, chunk, a, rank, nranks,
                               epoch, (int)(epoch & 1u), cap, 0, err, ticks, 1, skip_flags ? 1 : 0, src, u);
        };
        if (u.logmode) run(k_p2p_allreduce<true, 2>);
        else run(k_p2p_allreduce<true, 1>);
        check_launch("k_p2p_reduce_allreduce (fused update)");
        return;
    }
    hipLaunchKernelGGL(k_p2p_allreduce<true>, dim3((unsigned)blocks), dim3(256), 0, stream, nullptr, out, n, chunk, a,
                       rank, nranks, epoch, (int)(epoch & 1u), cap, 0, err, ticks, 1, skip_flags ? 1 : 0, src,
                       UpdateArgs{});
    check_launch("k_p2p_reduce_allreduce");
}

}  // namespace sart
