// Host-side collectives of the native runtime (the CPU path, bootstrap of the device communicators and
// every small host reduction: normalisation maxima, sums of squares, barriers).
//
// The reference uses host MPI_Allreduce / MPI_Barrier on MPI_COMM_WORLD (reference sartsolver.cpp:47,
// 158-329; main.cpp:84). Backends here:
//   * local -- one rank, identity;
//   * tcp   -- TCP sockets, star through rank 0, reductions in fixed rank order (bitwise reproducible and
//              independent of the launcher), no MPI library needed;
//   * mpi   -- MPI_COMM_WORLD through libmpi loaded at run time (mpiexec launches, multi-node bootstrap).
// Rendezvous follows torchrun / MPI launchers (env_world): RANK, WORLD_SIZE, LOCAL_RANK (or
// OMPI_COMM_WORLD_*, PMI_*), MASTER_ADDR (default 127.0.0.1); the port is SART_COMM_PORT, else
// MASTER_PORT + 17 (torchrun's own store owns MASTER_PORT).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace sart {

enum class ReduceOp { kSum = 0, kMax = 1 };

class HostComm {
   public:
    virtual ~HostComm() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    virtual const char* backend() const = 0;
    virtual void all_reduce_host(double* v, size_t n, ReduceOp op) = 0;
    virtual void all_reduce_host(float* v, size_t n, ReduceOp op) = 0;
    virtual void broadcast_host(void* buf, size_t nbytes, int root) = 0;
    virtual void barrier() = 0;
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

std::unique_ptr<HostComm> make_local_host_comm();
std::unique_ptr<HostComm> make_tcp_host_comm(int rank, int size, const std::string& host, int port,
                                             double timeout_s = 3600.0);
// MPI_COMM_WORLD through a run-time loaded libmpi (MPICH or Open MPI ABI, detected; host_comm_mpi.cpp).
std::unique_ptr<HostComm> make_mpi_host_comm();
// MPI_Get_library_version of the loaded libmpi (loads it).
std::string mpi_library_version();
// SART_HOST_COMM=mpi, or an MPI launcher (PMI_SIZE or OMPI_COMM_WORLD_SIZE > 1 without torchrun's RANK).
bool mpi_launch_detected();
// MPI when mpi_launch_detected(); else local for one rank, TCP otherwise (SART_HOST_COMM=tcp forces TCP).
// timeout_s < 0: SART_HOST_TIMEOUT_S, default 1800 s -- every TCP send / receive / accept of the host collectives is
// bounded by it (a peer that died or never came is an error on every rank, not a hang; rank 0 writing output between
// frames is far below it)
std::unique_ptr<HostComm> host_comm_from_env(double timeout_s = -1.0);

// Balanced 1-D block partition (reference main.cpp:67-68): the first n % parts parts get one more.
struct Block {
    uint64_t offset = 0, size = 0;
};
Block block_partition(uint64_t n, int parts, int part);

}  // namespace sart
