#include "comm.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace sart {

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void nccl_ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

int env_int(const char* const* names, int dflt) {
    for (const char* const* n = names; *n; ++n) {
        const char* v = std::getenv(*n);
        if (v && *v) return std::atoi(v);
    }
    return dflt;
}

// ------------------------------------------------------------------------------------------------
class LocalComm final : public Communicator {
   public:
    int rank() const override { return 0; }
    int size() const override { return 1; }
    const char* backend() const override { return "local"; }
    void all_reduce(float*, size_t, ReduceOp, hipStream_t) override {}
    void all_reduce(double*, size_t, ReduceOp, hipStream_t) override {}
    void all_reduce_host(double*, size_t, ReduceOp) override {}
    void broadcast_host(void*, size_t, int) override {}
    void barrier() override {}
    bool graph_capturable() const override { return true; }
};

// ------------------------------------------------------------------------------------------------
class TcpComm final : public Communicator {
   public:
    TcpComm(int rank, int size, const std::string& host, int port, double timeout_s)
        : rank_(rank), size_(size), fds_(size, -1) {
        if (size < 1 || rank < 0 || rank >= size) throw std::runtime_error("TcpComm: bad rank/size");
        if (size == 1) return;
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
        if (rank == 0) {
            listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
            if (listen_fd_ < 0) throw std::runtime_error("TcpComm: socket failed");
            int one = 1;
            ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_addr.s_addr = htonl(INADDR_ANY);
            a.sin_port = htons((uint16_t)port);
            if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0)
                throw std::runtime_error("TcpComm: bind to port " + std::to_string(port) + " failed: " +
                                         std::strerror(errno));
            if (::listen(listen_fd_, size) != 0) throw std::runtime_error("TcpComm: listen failed");
            for (int k = 1; k < size; ++k) {
                int fd = ::accept(listen_fd_, nullptr, nullptr);
                if (fd < 0) throw std::runtime_error("TcpComm: accept failed");
                tune(fd, timeout_s);
                int32_t r = -1;
                recv_all(fd, &r, sizeof(r));
                if (r <= 0 || r >= size || fds_[r] >= 0) throw std::runtime_error("TcpComm: bad peer rank");
                fds_[r] = fd;
            }
        } else {
            addrinfo hints{}, *res = nullptr;
            hints.ai_family = AF_INET;
            hints.ai_socktype = SOCK_STREAM;
            if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
                throw std::runtime_error("TcpComm: cannot resolve " + host);
            int fd = -1;
            while (true) {
                fd = ::socket(AF_INET, SOCK_STREAM, 0);
                if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
                if (fd >= 0) ::close(fd);
                if (std::chrono::steady_clock::now() > deadline) {
                    ::freeaddrinfo(res);
                    throw std::runtime_error("TcpComm: rank " + std::to_string(rank) + " cannot reach " + host + ":" +
                                             std::to_string(port));
                }
                std::this_thread::sleep_for(std::chrono::milliseconds(20));
            }
            ::freeaddrinfo(res);
            tune(fd, timeout_s);
            int32_t r = rank;
            send_all(fd, &r, sizeof(r));
            fds_[0] = fd;
        }
    }
    ~TcpComm() override {
        for (int fd : fds_)
            if (fd >= 0) ::close(fd);
        if (listen_fd_ >= 0) ::close(listen_fd_);
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    const char* backend() const override { return "tcp"; }

    void all_reduce_host(double* v, size_t n, ReduceOp op) override { reduce_host(v, n, op); }
    void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) override { staged(dev, n, op, stream); }
    void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t stream) override { staged(dev, n, op, stream); }

    void broadcast_host(void* buf, size_t nbytes, int root) override {
        if (size_ == 1) return;
        if (rank_ == 0) {
            if (root != 0) recv_all(fds_[root], buf, nbytes);
            for (int r = 1; r < size_; ++r)
                if (r != root) send_all(fds_[r], buf, nbytes);
        } else {
            if (rank_ == root)
                send_all(fds_[0], buf, nbytes);
            else
                recv_all(fds_[0], buf, nbytes);
        }
    }
    void barrier() override {
        double z = 0.0;
        reduce_host(&z, 1, ReduceOp::kSum);
    }

   private:
    template <typename T>
    void staged(T* dev, size_t n, ReduceOp op, hipStream_t stream) {
        if (size_ == 1 || n == 0) return;
        std::vector<T> h(n);
        hip_ok(hipMemcpyAsync(h.data(), dev, n * sizeof(T), hipMemcpyDeviceToHost, stream), "TcpComm D2H");
        hip_ok(hipStreamSynchronize(stream), "TcpComm sync");
        reduce_host(h.data(), n, op);
        hip_ok(hipMemcpyAsync(dev, h.data(), n * sizeof(T), hipMemcpyHostToDevice, stream), "TcpComm H2D");
        hip_ok(hipStreamSynchronize(stream), "TcpComm sync");
    }
    template <typename T>
    void reduce_host(T* v, size_t n, ReduceOp op) {
        if (size_ == 1 || n == 0) return;
        const size_t nb = n * sizeof(T);
        if (rank_ == 0) {
            std::vector<T> tmp(n);
            for (int r = 1; r < size_; ++r) {  // fixed rank order: reproducible sums
                recv_all(fds_[r], tmp.data(), nb);
                if (op == ReduceOp::kSum)
                    for (size_t i = 0; i < n; ++i) v[i] += tmp[i];
                else
                    for (size_t i = 0; i < n; ++i) v[i] = std::max(v[i], tmp[i]);
            }
            for (int r = 1; r < size_; ++r) send_all(fds_[r], v, nb);
        } else {
            send_all(fds_[0], v, nb);
            recv_all(fds_[0], v, nb);
        }
    }
    static void tune(int fd, double timeout_s) {
        int one = 1;
        ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        timeval tv{};
        tv.tv_sec = (time_t)timeout_s;
        ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    }
    static void send_all(int fd, const void* p, size_t n) {
        const char* c = static_cast<const char*>(p);
        while (n > 0) {
            const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
            if (k <= 0) throw std::runtime_error("TcpComm: send failed (peer gone or timeout)");
            c += k, n -= (size_t)k;
        }
    }
    static void recv_all(int fd, void* p, size_t n) {
        char* c = static_cast<char*>(p);
        while (n > 0) {
            const ssize_t k = ::recv(fd, c, n, 0);
            if (k <= 0) throw std::runtime_error("TcpComm: recv failed (peer gone or timeout)");
            c += k, n -= (size_t)k;
        }
    }
    int rank_, size_;
    std::vector<int> fds_;
    int listen_fd_ = -1;
};

// ------------------------------------------------------------------------------------------------
class RcclComm final : public Communicator {
   public:
    RcclComm(int device, const std::string& uid, std::unique_ptr<Communicator> boot) : boot_(std::move(boot)) {
        if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclComm: bad unique id");
        ncclUniqueId id;
        std::memcpy(&id, uid.data(), sizeof(id));
        hip_ok(hipSetDevice(device), "hipSetDevice");
        nccl_ok(ncclCommInitRank(&comm_, boot_->size(), id, boot_->rank()), "ncclCommInitRank");
    }
    ~RcclComm() override {
        if (comm_) (void)ncclCommDestroy(comm_);
    }
    int rank() const override { return boot_->rank(); }
    int size() const override { return boot_->size(); }
    const char* backend() const override { return "rccl"; }
    void all_reduce(float* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        if (n) nccl_ok(ncclAllReduce(dev, dev, n, ncclFloat32, nop(op), comm_, stream), "ncclAllReduce");
    }
    void all_reduce(double* dev, size_t n, ReduceOp op, hipStream_t stream) override {
        if (n) nccl_ok(ncclAllReduce(dev, dev, n, ncclFloat64, nop(op), comm_, stream), "ncclAllReduce");
    }
    void all_reduce_host(double* v, size_t n, ReduceOp op) override { boot_->all_reduce_host(v, n, op); }
    void broadcast_host(void* buf, size_t nbytes, int root) override { boot_->broadcast_host(buf, nbytes, root); }
    void barrier() override { boot_->barrier(); }
    bool graph_capturable() const override { return true; }
    void abort() override {
        if (comm_) {
            (void)ncclCommAbort(comm_);
            comm_ = nullptr;
        }
    }

   private:
    static ncclRedOp_t nop(ReduceOp op) { return op == ReduceOp::kSum ? ncclSum : ncclMax; }
    std::unique_ptr<Communicator> boot_;
    ncclComm_t comm_ = nullptr;
};

}  // namespace

EnvWorld env_world() {
    static const char* kRank[] = {"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", nullptr};
    static const char* kSize[] = {"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", nullptr};
    static const char* kLocal[] = {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", nullptr};
    EnvWorld w;
    w.rank = env_int(kRank, 0);
    w.size = env_int(kSize, 1);
    w.local_rank = env_int(kLocal, w.rank);
    if (const char* a = std::getenv("MASTER_ADDR"); a && *a) w.master_addr = a;
    static const char* kPort[] = {"SART_COMM_PORT", nullptr};
    static const char* kMaster[] = {"MASTER_PORT", nullptr};
    const int own = env_int(kPort, -1);
    w.port = own > 0 ? own : env_int(kMaster, 29500) + 17;
    return w;
}

std::unique_ptr<Communicator> make_local_comm() { return std::make_unique<LocalComm>(); }

std::unique_ptr<Communicator> make_tcp_comm(int rank, int size, const std::string& host, int port, double timeout_s) {
    return std::make_unique<TcpComm>(rank, size, host, port, timeout_s);
}

std::string rccl_unique_id() {
    ncclUniqueId id;
    nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::unique_ptr<Communicator> make_rccl_comm(int device, const std::string& uid,
                                             std::unique_ptr<Communicator> bootstrap) {
    return std::make_unique<RcclComm>(device, uid, std::move(bootstrap));
}

std::unique_ptr<Communicator> comm_from_env(bool gpu, int device) {
    const EnvWorld w = env_world();
    if (w.size <= 1) return make_local_comm();
    auto tcp = make_tcp_comm(w.rank, w.size, w.master_addr, w.port);
    const char* be = std::getenv("SART_DIST_BACKEND");
    const bool want_rccl = gpu && !(be && (std::string(be) == "tcp" || std::string(be) == "gloo"));
    if (!want_rccl) return tcp;
    std::string uid(sizeof(ncclUniqueId), '\0');
    if (w.rank == 0) uid = rccl_unique_id();
    tcp->broadcast_host(uid.data(), uid.size(), 0);
    return make_rccl_comm(device, uid, std::move(tcp));
}

}  // namespace sart
