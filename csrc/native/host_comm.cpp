#include "host_comm.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace sart {

namespace {

int env_int(const char* const* names, int dflt) {
    for (const char* const* n = names; *n; ++n) {
        const char* v = std::getenv(*n);
        if (v && *v) return std::atoi(v);
    }
    return dflt;
}

class LocalHostComm final : public HostComm {
   public:
    int rank() const override { return 0; }
    int size() const override { return 1; }
    const char* backend() const override { return "local"; }
    void all_reduce_host(double*, size_t, ReduceOp) override {}
    void all_reduce_host(float*, size_t, ReduceOp) override {}
    void broadcast_host(void*, size_t, int) override {}
    void barrier() override {}
};

class TcpHostComm final : public HostComm {
   public:
    TcpHostComm(int rank, int size, const std::string& host, int port, double timeout_s)
        : rank_(rank), size_(size), fds_(size, -1) {
        if (size < 1 || rank < 0 || rank >= size) throw std::runtime_error("tcp comm: bad rank/size");
        if (size == 1) return;
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
        if (rank == 0) {
            listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
            if (listen_fd_ < 0) throw std::runtime_error("tcp comm: socket failed");
            int one = 1;
            ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_addr.s_addr = htonl(INADDR_ANY);
            a.sin_port = htons((uint16_t)port);
            if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0)
                throw std::runtime_error("tcp comm: bind to port " + std::to_string(port) + " failed: " +
                                         std::strerror(errno));
            if (::listen(listen_fd_, size) != 0) throw std::runtime_error("tcp comm: listen failed");
            tune(listen_fd_, timeout_s);  // SO_RCVTIMEO also bounds accept(): a peer that never comes is an error
            for (int k = 1; k < size; ++k) {
                int fd = ::accept(listen_fd_, nullptr, nullptr);
                if (fd < 0) throw std::runtime_error("tcp comm: accept failed");
                tune(fd, timeout_s);
                int32_t r = -1;
                recv_all(fd, &r, sizeof(r));
                if (r <= 0 || r >= size || fds_[r] >= 0) throw std::runtime_error("tcp comm: bad peer rank");
                fds_[r] = fd;
            }
        } else {
            addrinfo hints{}, *res = nullptr;
            hints.ai_family = AF_INET;
            hints.ai_socktype = SOCK_STREAM;
            if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
                throw std::runtime_error("tcp comm: cannot resolve " + host);
            int fd = -1;
            while (true) {
                fd = ::socket(AF_INET, SOCK_STREAM, 0);
                if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
                if (fd >= 0) ::close(fd);
                if (std::chrono::steady_clock::now() > deadline) {
                    ::freeaddrinfo(res);
                    throw std::runtime_error("tcp comm: rank " + std::to_string(rank) + " cannot reach " + host + ":" +
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
    ~TcpHostComm() override {
        for (int fd : fds_)
            if (fd >= 0) ::close(fd);
        if (listen_fd_ >= 0) ::close(listen_fd_);
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    const char* backend() const override { return "tcp"; }

    void all_reduce_host(double* v, size_t n, ReduceOp op) override { reduce_host(v, n, op); }
    void all_reduce_host(float* v, size_t n, ReduceOp op) override { reduce_host(v, n, op); }

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
            if (k <= 0) throw std::runtime_error("tcp comm: send failed (peer gone or timeout)");
            c += k, n -= (size_t)k;
        }
    }
    static void recv_all(int fd, void* p, size_t n) {
        char* c = static_cast<char*>(p);
        while (n > 0) {
            const ssize_t k = ::recv(fd, c, n, 0);
            if (k <= 0) throw std::runtime_error("tcp comm: recv failed (peer gone or timeout)");
            c += k, n -= (size_t)k;
        }
    }
    int rank_, size_;
    std::vector<int> fds_;
    int listen_fd_ = -1;
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

std::unique_ptr<HostComm> make_local_host_comm() { return std::make_unique<LocalHostComm>(); }

std::unique_ptr<HostComm> make_tcp_host_comm(int rank, int size, const std::string& host, int port, double timeout_s) {
    return std::make_unique<TcpHostComm>(rank, size, host, port, timeout_s);
}

std::unique_ptr<HostComm> host_comm_from_env(double timeout_s) {
    if (timeout_s < 0) {
        const char* e = std::getenv("SART_HOST_TIMEOUT_S");
        timeout_s = (e && *e && std::atof(e) > 0) ? std::atof(e) : 1800.0;
    }
    if (mpi_launch_detected()) return make_mpi_host_comm();
    const EnvWorld w = env_world();
    if (w.size <= 1) return make_local_host_comm();
    return make_tcp_host_comm(w.rank, w.size, w.master_addr, w.port, timeout_s);
}

Block block_partition(uint64_t n, int parts, int part) {
    if (parts <= 0 || part < 0 || part >= parts) throw std::invalid_argument("invalid partition request");
    const uint64_t base = n / (uint64_t)parts, rem = n % (uint64_t)parts;
    Block b;
    b.offset = (uint64_t)part * base + std::min<uint64_t>((uint64_t)part, rem);
    b.size = base + ((uint64_t)part < rem ? 1 : 0);
    return b;
}

}  // namespace sart
