// Communicators of the native engine. The reference reduces through host memory with
// CUDA-unaware MPI: D2H, MPI_Allreduce, H2D, plus a scalar MPI_Allreduce, every iteration
// (reference sartsolver_cuda.cpp:242-255). Backends here:
//   * LocalComm  -- one rank; every collective is the identity.
//   * TcpComm    -- host collectives over TCP sockets (star through rank 0, reductions in fixed rank
//                   order, so results are bitwise reproducible); device buffers are staged through host
//                   memory. Bootstrap channel of RCCL, and the backend of the --use_cpu path and of
//                   multi-rank runs that share one GPU (tests).
//   * RcclComm   -- RCCL (NCCL API) on device buffers over xGMI, ordered on the caller's HIP stream and
//                   capturable into HIP graphs; host collectives ride on its TcpComm bootstrap.
// Rendezvous follows torchrun / MPI launchers: RANK, WORLD_SIZE, LOCAL_RANK (or OMPI_COMM_WORLD_*,
// PMI_*), MASTER_ADDR (default 127.0.0.1), MASTER_PORT (default 29500); the engine's own TCP port is
// SART_COMM_PORT or MASTER_PORT + 17 (torchrun's store owns MASTER_PORT).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace sart {

enum class ReduceOp { kSum = 0, kMax = 1 };

class Communicator {
   public:
    virtual ~Communicator() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    virtual const char* backend() const = 0;
    // In-place reductions of device buffers, stream-ordered on `stream`.
    virtual void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) = 0;
    virtual void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t stream) = 0;
    // Blocking host collectives (small messages).
    virtual void all_reduce_host(double* v, size_t n, ReduceOp op) = 0;
    virtual void broadcast_host(void* buf, size_t nbytes, int root) = 0;
    virtual void barrier() = 0;
    // Device collectives may be captured into a HIP graph.
    virtual bool graph_capturable() const { return false; }
    // Tear down after a fatal error so that peers blocked in a collective fail instead of hanging.
    virtual void abort() {}
    double all_reduce_scalar(double v, ReduceOp op) {
        all_reduce_host(&v, 1, op);
        return v;
    }
};

struct EnvWorld {
    int rank = 0, size = 1, local_rank = 0;
    std::string master_addr = "127.0.0.1";
    int port = 29517;
};
EnvWorld env_world();

std::unique_ptr<Communicator> make_local_comm();
std::unique_ptr<Communicator> make_tcp_comm(int rank, int size, const std::string& host, int port,
                                            double timeout_s = 3600.0);
std::string rccl_unique_id();  // NCCL_UNIQUE_ID_BYTES opaque bytes (call on one rank)
// `bootstrap` (moved in) carries the host collectives; `uid` must be the same bytes on every rank.
std::unique_ptr<Communicator> make_rccl_comm(int device, const std::string& uid, std::unique_ptr<Communicator> bootstrap);
// From the launcher environment: Local for one rank; else TcpComm, upgraded to RCCL when `gpu` and
// SART_DIST_BACKEND is not "tcp".
std::unique_ptr<Communicator> comm_from_env(bool gpu, int device);

}  // namespace sart
