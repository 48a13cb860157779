// Device communicators of the native engine. The reference reduces through host memory
// with CUDA-unaware MPI: D2H, MPI_Allreduce, H2D, plus a scalar MPI_Allreduce, every iteration
// (reference sartsolver_cuda.cpp:242-255). Backends here (host collectives come from a HostComm,
// csrc/native/host_comm.hpp):
//   * local  -- one rank; every collective is the identity.
//   * staged -- device buffers staged through host memory over the TCP HostComm (several ranks
//               sharing one GPU in tests, hosts without RCCL).
//   * rccl   -- RCCL (NCCL API) on device buffers over xGMI, ordered on the caller's HIP stream and
//               capturable into HIP graphs; host collectives ride on its TCP bootstrap HostComm.
//   * p2p    -- one-shot push all-reduce through IPC-mapped peer buffers over all xGMI links at once
//               (csrc/kernels/p2p_allreduce.hip) for fp32 vectors up to SART_P2P_MAX_BYTES, wrapping a
//               base communicator (RCCL in production) that serves everything else. Enabled after an
//               exact self-test on every rank; SART_P2P=0 off, 1 on, auto (default): rank 0 times both at
//               the message sizes the engine announces (Communicator::prepare) and P2P serves the sizes at
//               which it won.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../kernels/launchers.hpp"
#include "../native/host_comm.hpp"

namespace sart {

class Communicator {
   public:
    virtual ~Communicator() = default;
    virtual HostComm& host() = 0;
    virtual const char* backend() const = 0;
    // In-place reductions of device buffers, stream-ordered on `stream`.
    virtual void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) = 0;
    virtual void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t stream) = 0;
    // The single-frame engine's per-sweep collective: out[0, ld + 2) = the ReduceSrc vector (launchers.hpp), summed
    // over the ranks. Default: launch_reduce_partials, then all_reduce; p2p: one kernel forms and pushes the vector.
    virtual void reduce_all_reduce(const ReduceSrc& src, float* out, hipStream_t stream);
    // reduce_all_reduce, and where the backend can, the decision and update of the sweep in the same launch
    // (p2p: launch_p2p_reduce_allreduce with UpdateArgs). Returns true when the update ran; false: the caller runs
    // launch_decide_update on out (default).
    virtual bool reduce_all_reduce_update(const ReduceSrc& src, float* out, const UpdateArgs& upd, hipStream_t stream) {
        (void)upd;
        reduce_all_reduce(src, out, stream);
        return false;
    }
    // Device collectives may be captured into a HIP graph.
    virtual bool graph_capturable() const { return false; }
    // Tear down after a fatal error so that peers blocked in a collective fail instead of hanging.
    virtual void abort() { host().abort(); }
    // Throws when a device collective reported a failure (p2p: a peer aborted, or never arrived while the
    // p2p path is still active). Call after a sync.
    virtual void check() {}
    // Recoverable device-collective failure on THIS rank since construction (p2p: a peer did not arrive within
    // SART_P2P_TIMEOUT_S; the call's output is NaN). Call after a sync; the engines agree on it over the host
    // communicator, then every rank calls degrade() and re-solves.
    virtual bool device_failed() { return false; }
    // True while degrade() has something to switch to (the engines agree on failures only then).
    virtual bool degradable() const { return false; }
    // Serve every device collective from the base path from now on (p2p -> RCCL / staged). Collective in the
    // sense that every rank must call it after the same solve.
    virtual bool degrade() { return false; }
    // The engines announce the fp32 message sizes of their collectives (collective: every rank, same sizes). The
    // p2p communicator in auto mode times itself against its base at exactly those sizes (once per size) and
    // serves a size from the p2p path when it won there; sizes never announced are served by the base.
    virtual void prepare(const std::vector<int64_t>& float_sizes) { (void)float_sizes; }
    // Host-side start-up cost of the communicator so far (p2p: IPC mapping, self-test, probes), seconds.
    virtual double setup_seconds() const { return 0.0; }
    // Human-readable selection (backend and why), e.g. for benchmark logs.
    virtual std::string describe() const { return backend(); }
    int rank() { return host().rank(); }
    int size() { return host().size(); }
};

// The largest number of ranks of `host` that run on one physical GPU (identity: boot id + host name + PCI bus id),
// identical on every rank. Collective over the host communicator.
int ranks_sharing_device(HostComm& host, int device);

std::unique_ptr<Communicator> make_local_comm();
std::unique_ptr<Communicator> make_staged_comm(std::unique_ptr<HostComm> host);
std::string rccl_unique_id();  // NCCL_UNIQUE_ID_BYTES opaque bytes (call on one rank)
// `bootstrap` carries the host collectives; `uid` must be the same bytes on every rank.
std::unique_ptr<Communicator> make_rccl_comm(int device, const std::string& uid, std::unique_ptr<HostComm> bootstrap);
// One-shot P2P all-reduce over `base` (which keeps serving doubles, large vectors and host collectives).
// Collective: every rank of base calls it. Falls back to plain `base` behaviour (backend() == base's) when
// the ranks span several hosts, IPC mapping or the self-test fails, or SART_P2P=0.
std::unique_ptr<Communicator> make_p2p_comm(int device, std::shared_ptr<Communicator> base);
// From the launcher environment: local for one rank; else RCCL (with the P2P all-reduce, SART_P2P) over a
// TCP or MPI bootstrap, or staged when SART_DIST_BACKEND is "tcp"/"gloo".
std::unique_ptr<Communicator> comm_from_env(int device);

}  // namespace sart
